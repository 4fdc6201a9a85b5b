"""bench.py's multi-process contract on the C++ engine, on the CPU backend (host TCP ring): the
torch.distributed launcher starts one bench.py per rank, each runs the C++ trainer as a child with
--dp, rank 0 prints one JSON line with the whole job's images/sec; when any rank's child fails,
every rank falls back to the Python engine (agreement over a CPU gloo group)."""
import json
import os
import socket
import subprocess
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "dcnn_amd", "bin", "tiny_imagenet_resnet18")


@pytest.fixture(scope="module")
def built():
    if not (os.path.exists(EXE) and torch.cuda.is_available()):
        from dcnn_amd import _build
        _build.build_host()


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _torchrun(world, extra_env=None):
    env = dict(os.environ, OMP_NUM_THREADS="2", **(extra_env or {}))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", str(world), "--steps", "1", "--warmup", "1", "--batch", "2", "--device", "cpu",
           "--dtype", "fp32", "--engine", "native"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=600)
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    return r, lines


def test_bench_native_two_ranks_cpu(built):
    r, lines = _torchrun(2)
    assert r.returncode == 0, r.stderr[-3000:]
    assert len(lines) == 1, r.stdout  # rank 0 only
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["global_batch"] == 4
    assert d["config"]["engine"].startswith("native") and d["config"]["data_plane"] == "tcp"
    assert d["config"]["dp_buckets"] >= 2 and d["value"] > 0


def test_bench_native_failure_falls_back_everywhere(built):
    r, lines = _torchrun(2, {"DCNN_BENCH_FAULT_RANK": "1", "DCNN_DIST_TIMEOUT": "5"})
    # rank 1 fails before its rendezvous, rank 0 gives up after DCNN_DIST_TIMEOUT; --engine native was
    # asked explicitly, so the agreed failure is an error (auto would run the Python engine)
    assert r.returncode != 0
    assert "C++ engine failed" in r.stderr
