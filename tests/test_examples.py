"""Smoke runs of the example programs on tiny synthetic data (CPU)."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("script,args", [
    ("mnist_cnn_trainer.py", ["--synthetic", "128", "--batch-size", "32", "--max-batches", "2"]),
    ("cifar10_resnet9.py", ["--synthetic", "64", "--batch-size", "32", "--max-batches", "1"]),
    ("uji_ips_trainer.py", ["--synthetic", "1", "--batch-size", "64", "--max-batches", "2"]),
    ("semi_async_pipeline_coordinator.py", ["--local", "--synthetic", "64", "--batch-size", "16", "--max-batches", "1"]),
    ("sync_pipeline_coordinator.py", ["--local", "--synthetic", "64", "--batch-size", "16", "--max-batches", "1"]),
])
def test_example_runs(tmp_path, script, args):
    env = dict(os.environ, EPOCHS="1", PROGRESS_PRINT_INTERVAL="1", DEVICE_TYPE="CPU", OMP_NUM_THREADS="2")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "examples", script), *args], cwd=str(tmp_path), env=env,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
