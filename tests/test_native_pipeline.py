"""Native pipeline stages (csrc/host/pipeline.cpp, dcnn_amd/bin/network_worker): separate C++
worker processes driven over TCP by the Python DistributedCoordinator train like the Python
stages of an in-process coordinator (same partitions, same initial weights pushed by
LOAD_PARAMS): the same losses and parameters after sync / semi-async / 1F1B steps, and the
full parameter + optimizer state survives a SEND_PARAMS "full" -> LOAD_PARAMS round trip
(the coordinator's recovery path). The native coordinator (csrc/host/coordinator.cpp,
bin/pipeline_coordinator) driving those workers matches the Python coordinator step for step.
Reference: examples/network_worker.cpp:14-194, include/pipeline/pipeline_stage.hpp:29-308,
include/pipeline/coordinator.hpp:30-599, examples/semi_async_pipeline_coordinator.cpp."""
import os
import socket
import subprocess

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORKER = os.path.join(ROOT, "dcnn_amd", "bin", "network_worker")


@pytest.fixture(scope="module")
def worker_bin():
    if not os.path.exists(WORKER):
        from dcnn_amd import _build
        _build.build_host()
    return WORKER


def _free_ports(n):
    socks, ports = [], []
    for _ in range(n):
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        socks.append(s)
        ports.append(s.getsockname()[1])
    for s in socks:
        s.close()
    return ports


def _model(seed=3):
    from dcnn_amd.nn import SequentialBuilder
    m = (SequentialBuilder("native_pipe").input([3, 12, 12])
         .conv2d(8, 3, 3, 1, 1, 1, 1).batchnorm().activation("relu").maxpool2d(2, 2, 2, 2)
         .conv2d(16, 3, 3, 1, 1, 1, 1).activation("relu")
         .flatten().dense(10).build())
    m.set_seed(seed)
    m.initialize()
    return m


class _Workers:
    def __init__(self, binary, n):
        self.ports = _free_ports(n)
        self.procs = [subprocess.Popen([binary, str(p), "--host", "127.0.0.1"], stdout=subprocess.PIPE,
                                       stderr=subprocess.STDOUT, text=True) for p in self.ports]
        for p in self.procs:  # wait for "listening"
            line = p.stdout.readline()
            assert "listening" in line, line

    def close(self):
        for p in self.procs:
            try:
                p.wait(timeout=20)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()


def _train(coord, steps, schedule, seed=5):
    g = torch.Generator().manual_seed(seed)
    losses = []
    for _ in range(steps):
        x = torch.randn(8, 3, 12, 12, generator=g)
        y = torch.randint(0, 10, (8,), generator=g)
        losses.append(float(coord.train_step(x, y, schedule=schedule)))
    return losses


@pytest.mark.parametrize("schedule", ["sync", "semi_async", "1f1b"])
@pytest.mark.parametrize("opt_name", ["adam", "sgd_momentum"])
def test_native_stages_train_like_python_stages(worker_bin, schedule, opt_name):
    from dcnn_amd.nn import SGD, Adam
    from dcnn_amd.parallel.pipeline import DistributedCoordinator, Endpoint, InProcessCoordinator
    mk_opt = (lambda: Adam(2e-3)) if opt_name == "adam" else (lambda: SGD(0.05, 0.9))
    ref_model = _model()
    ref = InProcessCoordinator(ref_model, mk_opt(), "softmax_crossentropy", num_stages=2, num_microbatches=2,
                               transport="message")
    ref.initialize()
    ref.deploy_stages()
    ref.start()
    ref.send_parameters(ref_model)
    ref_losses = _train(ref, 3, schedule)
    ref_params = ref.collect_parameters()
    ref.stop()

    w = _Workers(worker_bin, 2)
    try:
        model = _model()
        eps = [Endpoint.network("127.0.0.1", p) for p in w.ports]
        coord = DistributedCoordinator(model, mk_opt(), "softmax_crossentropy", eps, num_microbatches=2,
                                       host="127.0.0.1", timeout_s=60)
        coord.initialize()
        coord.deploy_stages()
        coord.start()
        coord.send_parameters(model)
        st = coord.status()
        assert all(s.get("native") for s in st), st
        losses = _train(coord, 3, schedule)
        params = coord.collect_parameters()
        # recovery path: full state out, perturb, full state back in -> identical next step
        full = coord.collect_parameters(full=True)
        coord.send_parameters(_model(seed=99))  # clobber the weights
        from dcnn_amd.parallel.pipeline import messages as M
        from dcnn_amd.parallel.pipeline.messages import CommandType as C
        for name, flat in zip(coord.stage_names, full):
            coord.comm.send(M.job_message(name, C.LOAD_PARAMS, 1, flat))
        coord.join(C.PARAMS_LOADED, coord.num_stages)
        full2 = coord.collect_parameters(full=True)
        coord.stop()
    finally:
        w.close()
    np.testing.assert_allclose(losses, ref_losses, rtol=2e-4, atol=1e-6)
    # (Adam normalises each update by sqrt(v): a weight whose gradients are ~0 moves by up to lr
    # per step on the sign of fp32 rounding noise, so its tolerance is a fraction of lr)
    atol = 5e-4 if opt_name == "adam" else 2e-5
    for a, b in zip(params, ref_params):
        np.testing.assert_allclose(a.numpy(), b.numpy(), rtol=1e-3, atol=atol)
    for a, b in zip(full, full2):
        assert torch.equal(a, b)
    assert all(p.returncode == 0 for p in w.procs), [p.returncode for p in w.procs]


COORD = os.path.join(ROOT, "dcnn_amd", "bin", "pipeline_coordinator")


@pytest.mark.parametrize("stage_loss", ["0", "1"])
@pytest.mark.parametrize("schedule", ["sync", "semi_async", "1f1b"])
def test_native_coordinator_trains_like_python_coordinator(worker_bin, tmp_path, schedule, stage_loss):
    """The C++ coordinator (csrc/host/coordinator.cpp, bin/pipeline_coordinator) driving native
    workers: the same per-step losses and the same trained model (gathered from the stages and
    saved by the C++ program, loaded in Python) as the Python coordinator on the same batches —
    with the loss on the coordinator (stage_loss 0) or on the last stage (1: labels to that stage,
    its backward starts there, only the loss value comes back)."""
    import json
    from dcnn_amd.nn import Adam, Sequential
    from dcnn_amd.parallel.pipeline import InProcessCoordinator
    init = str(tmp_path / "init")
    _model().save_to_file(init)
    g = torch.Generator().manual_seed(5)
    xs, ys = [], []
    for _ in range(3):
        xs.append(torch.randn(8, 3, 12, 12, generator=g))
        ys.append(torch.randint(0, 10, (8,), generator=g))
    torch.cat(xs).numpy().astype(np.float32).tofile(tmp_path / "x.f32")
    torch.cat(ys).numpy().astype(np.int64).tofile(tmp_path / "y.i64")

    ref_model = _model()
    ref = InProcessCoordinator(ref_model, Adam(2e-3), "softmax_crossentropy", num_stages=2, num_microbatches=2,
                               transport="message")
    ref.initialize()
    ref.deploy_stages()
    ref.start()
    ref.send_parameters(ref_model)
    ref_losses = _train(ref, 3, schedule)
    trained = ref.gather_model()
    ref.stop()

    w = _Workers(worker_bin, 2)
    try:
        out = subprocess.run(
            [COORD, "--workers", ",".join(f"127.0.0.1:{p}" for p in w.ports), "--init", init, "--schedule", schedule,
             "--microbatches", "2", "--batch", "8", "--steps", "3", "--optimizer", "adam", "--lr", "2e-3",
             "--data-x", str(tmp_path / "x.f32"), "--data-y", str(tmp_path / "y.i64"), "--input", "3,12,12",
             "--json", "--save", str(tmp_path / "out"), "--stage-loss", stage_loss],
            capture_output=True, text=True, timeout=120)
    finally:
        w.close()
    assert out.returncode == 0, out.stderr
    losses = [json.loads(l)["loss"] for l in out.stdout.splitlines() if l.startswith("{")]
    np.testing.assert_allclose(losses, ref_losses, rtol=2e-4, atol=1e-6)
    got = Sequential.from_file(str(tmp_path / "out"))
    for a, b in zip(got.parameters(), trained.parameters()):
        np.testing.assert_allclose(a.detach().numpy(), b.detach().numpy(), rtol=1e-3, atol=5e-4)
    bn_got = [l for l in got.layers if hasattr(l, "running_mean")]
    bn_ref = [l for l in trained.layers if hasattr(l, "running_mean")]
    assert len(bn_got) == len(bn_ref) == 1
    np.testing.assert_allclose(bn_got[0].running_var.numpy(), bn_ref[0].running_var.numpy(), rtol=1e-4)


@pytest.mark.gpu
def test_native_coordinator_gpu_stages(worker_bin):
    """All-native pipeline on the GPU: the C++ coordinator, two native GPU stages (routed MFMA
    kernels), ResNet-9 on CIFAR-shaped synthetic data, 1F1B; the loss falls."""
    import json
    out = subprocess.run([COORD, "--spawn", "2", "--model", "resnet9_cifar10", "--device", "GPU:0", "--input", "3,32,32",
                          "--classes", "10", "--batch", "64", "--microbatches", "4", "--steps", "12", "--schedule", "1f1b",
                          "--json"], capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-2000:]
    steps = [json.loads(l) for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(steps) == 12 and all(np.isfinite(s["loss"]) for s in steps)
    assert "GPU" in out.stderr
    assert np.mean([s["loss"] for s in steps[-3:]]) < np.mean([s["loss"] for s in steps[:3]])


@pytest.mark.gpu
def test_native_coordinator_ipc_transport_matches_messages(worker_bin):
    """Transport "ipc": stage-to-stage tensors stay on the device (HIP IPC buffers, only handles in
    the messages). The same bytes arrive as with inline payloads, so every step's loss is the same —
    with the host-waited hand-off (default) and with the device-ordered ones (DCNN_IPC_HANDOFF=event:
    an interprocess event; =flag: a flag the sender's stream writes and the receiver's stream waits
    on) — no host wait on either side, which also lets the first stage's backward finish before the
    last stage's loss report."""
    import json
    losses, samples = {}, {}
    modes = ("host", "event", "flag")
    for transport, wait in [("message", "host")] + [("ipc", w) for w in modes]:
        env = dict(os.environ, DCNN_IPC_HANDOFF=wait)
        out = subprocess.run([COORD, "--spawn", "3", "--model", "resnet9_cifar10", "--device", "GPU:0", "--input",
                              "3,32,32", "--classes", "10", "--batch", "64", "--microbatches", "4", "--steps", "6",
                              "--schedule", "1f1b", "--transport", transport, "--json"],
                             capture_output=True, text=True, timeout=240, env=env)
        assert out.returncode == 0, out.stderr[-2000:]
        rows = [json.loads(l) for l in out.stdout.splitlines() if l.startswith("{")]
        losses[transport, wait] = [r["loss"] for r in rows]
        samples[transport, wait] = [r["samples"] for r in rows]
    for k in [("ipc", w) for w in modes]:
        assert len(losses[k]) == 6 and all(np.isfinite(losses[k]))
        assert samples[k] == [64] * 6, samples  # every micro-batch's report inside its own step
        np.testing.assert_allclose(losses[k], losses["message", "host"], rtol=1e-6)


@pytest.mark.gpu
def test_native_stage_graphs_match_eager(worker_bin):
    """GPU stages capture one hipGraph per (phase, micro-batch) from the second step on and replay
    it after; the replays run the same kernels on the same data as the eager path, so every step's
    loss is the same with the graphs off (DCNN_STAGE_GRAPHS=0)."""
    import json
    import os
    losses = {}
    for graphs in ("0", "1"):
        env = dict(os.environ, DCNN_STAGE_GRAPHS=graphs)
        out = subprocess.run([COORD, "--spawn", "3", "--model", "resnet9_cifar10", "--device", "GPU:0", "--input",
                              "3,32,32", "--classes", "10", "--batch", "64", "--microbatches", "4", "--steps", "6",
                              "--schedule", "1f1b", "--transport", "ipc", "--json"],
                             capture_output=True, text=True, timeout=240, env=env)
        assert out.returncode == 0, out.stderr[-2000:]
        losses[graphs] = [json.loads(l)["loss"] for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(losses["1"]) == 6 and all(np.isfinite(losses["1"]))
    np.testing.assert_allclose(losses["1"], losses["0"], rtol=1e-6)


def test_native_ipc_transport_needs_gpu_stages(worker_bin):
    out = subprocess.run([COORD, "--spawn", "2", "--steps", "1", "--transport", "ipc"], capture_output=True, text=True,
                         timeout=60)
    assert out.returncode == 1 and "needs a GPU stage" in out.stderr


def test_native_rccl_transport_needs_distinct_gpus(worker_bin):
    """transport "rccl" pairs adjacent stages in two-rank RCCL communicators: CPU stages, or two
    stages on one GPU (RCCL refuses both ranks on one device), are rejected before any stage runs."""
    for devices in ("CPU,CPU", "GPU:0,GPU:0"):
        out = subprocess.run([COORD, "--spawn", "2", "--steps", "1", "--transport", "rccl", "--devices", devices],
                             capture_output=True, text=True, timeout=60)
        assert out.returncode == 1 and "adjacent stages need distinct GPUs" in out.stderr, out.stderr


def test_native_coordinator_rejects_bad_arguments(worker_bin):
    out = subprocess.run([COORD, "--workers", "", "--steps", "0"], capture_output=True, text=True, timeout=30)
    assert out.returncode == 1 and "no workers" in out.stderr
    out = subprocess.run([COORD, "--spawn", "2", "--schedule", "zigzag", "--steps", "1"], capture_output=True,
                         text=True, timeout=60)
    assert out.returncode == 1 and "unknown pipeline schedule" in out.stderr


def test_native_stage_reports_errors(worker_bin):
    """A stage failure comes back as a JOB_FAILURE the coordinator raises (not a hang)."""
    from dcnn_amd.nn import Adam
    from dcnn_amd.parallel.pipeline import DistributedCoordinator, Endpoint, PipelineError
    w = _Workers(worker_bin, 2)
    try:
        model = _model()
        eps = [Endpoint.network("127.0.0.1", p) for p in w.ports]
        coord = DistributedCoordinator(model, Adam(1e-3), "softmax_crossentropy", eps, num_microbatches=1,
                                       host="127.0.0.1", timeout_s=30)
        coord.initialize()
        coord.deploy_stages()
        coord.start()
        with pytest.raises(PipelineError, match="FORWARD_JOB failed"):
            coord.train_step(torch.randn(2, 5, 12, 12), torch.zeros(2, dtype=torch.long), schedule="sync")
        coord.stop()
    finally:
        w.close()


@pytest.mark.gpu
def test_native_gpu_stages_train_like_python_gpu_stages(worker_bin):
    """Native stages on the GPU backend (bf16 NHWC activations on the wire, flagged channels-last
    like the Python transport) against Python GPU stages: the same loss curve to bf16 accuracy."""
    from dcnn_amd.nn import Adam
    from dcnn_amd.parallel.pipeline import DistributedCoordinator, Endpoint, InProcessCoordinator
    kw = dict(num_microbatches=2, stage_devices=["GPU:0", "GPU:0"], device="GPU:0")
    ref_model = _model()
    ref = InProcessCoordinator(ref_model, Adam(1e-3), "softmax_crossentropy", num_stages=2, transport="message",
                               use_graph=False, **kw)
    ref.initialize()
    ref.deploy_stages()
    ref.start()
    ref.send_parameters(ref_model)
    ref_losses = _train(ref, 4, "semi_async")
    ref.stop()
    w = _Workers(worker_bin, 2)
    try:
        model = _model()
        eps = [Endpoint.network("127.0.0.1", p) for p in w.ports]
        coord = DistributedCoordinator(model, Adam(1e-3), "softmax_crossentropy", eps, host="127.0.0.1",
                                       timeout_s=120, **kw)
        coord.initialize()
        coord.deploy_stages()
        coord.start()
        coord.send_parameters(model)
        assert all(s.get("native") and s.get("device", "").startswith("GPU") for s in coord.status())
        losses = _train(coord, 4, "semi_async")
        coord.stop()
    finally:
        w.close()
    np.testing.assert_allclose(losses, ref_losses, rtol=3e-2)
