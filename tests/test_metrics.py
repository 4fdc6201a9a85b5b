"""Metrics sink, CPU-usage logger and the CPU plot tool (reference src/plot_cpu_range.py)."""
import os
import subprocess
import sys
import time

from dcnn_amd.utils.metrics import CpuUsageLogger, MetricsSink, read_metrics

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_metrics_sink_jsonl(tmp_path):
    p = tmp_path / "m.jsonl"
    with MetricsSink(str(p), tag="t") as m:
        assert m.enabled
        m.log("batch", batch=1, loss=0.5)
        m.log("epoch", epoch=1, images_per_sec=123.0)
    recs = read_metrics(str(p))
    assert [r["event"] for r in recs] == ["batch", "epoch"]
    assert recs[0]["loss"] == 0.5 and recs[1]["images_per_sec"] == 123.0 and recs[0]["tag"] == "t"
    assert not MetricsSink("").enabled


def test_cpu_logger_and_plot(tmp_path):
    logs = tmp_path / "logs"
    with CpuUsageLogger(str(logs), "coordinator", interval=0.05) as lg:
        t0 = time.time()
        x = 0
        while time.time() - t0 < 0.4:  # burn CPU so the samples are non-trivial
            x += 1
    assert lg.samples >= 3
    with CpuUsageLogger(str(logs), "machine", interval=0.05, pid=0):
        time.sleep(0.2)
    lines = open(lg.path).read().splitlines()
    assert lines[0] == "t_sec,cpu_percent,tag"
    vals = [float(l.split(",")[1]) for l in lines[1:]]
    assert max(vals) > 20.0
    out = tmp_path / "cpu.png"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "plot_cpu_range.py"), "--logs", str(logs),
                        "--out", str(out), "--smooth", "2"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert out.exists() and out.stat().st_size > 1000


def test_trainer_writes_metrics(tmp_path, monkeypatch):
    from dcnn_amd.data import SyntheticDataLoader
    from dcnn_amd.models import create_model
    from dcnn_amd.nn import Adam, LossFactory, TrainingConfig
    from dcnn_amd.nn.train import train_classification_model
    p = tmp_path / "train.jsonl"
    monkeypatch.setenv("METRICS_FILE", str(p))
    model = create_model("mnist_cnn")
    model.set_device("CPU")
    model.initialize()
    tr = SyntheticDataLoader(64, (1, 28, 28), 10, seed=1)
    te = SyntheticDataLoader(32, (1, 28, 28), 10, seed=2)
    cfg = TrainingConfig()
    cfg.epochs, cfg.batch_size, cfg.progress_print_interval = 1, 32, 1
    cfg.snapshot_dir = str(tmp_path)
    train_classification_model(model, tr, te, Adam(1e-3), LossFactory.create("logsoftmax_crossentropy"), cfg)
    recs = read_metrics(str(p))
    ev = [r["event"] for r in recs]
    assert ev.count("batch") == 2 and ev[-1] == "epoch"
    assert recs[-1]["images_per_sec"] > 0 and "val_acc" in recs[-1]
