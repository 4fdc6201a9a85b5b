"""C++ host API data parallelism (csrc/host/dist.cpp) across processes: the rendezvous, the host
TCP ring of the CPU device, broadcast_parameters and the bucketed gradient mean, run at world 2
and 4 as separate processes under the launcher's variables. Every rank's averaged shard gradient
and updated parameters must match a single process trained on the whole batch (fp32; only the
summation order differs), be bitwise equal across ranks, and replicas started from different seeds
must hold rank 0's values after the broadcast. A missing rank ends the rendezvous with an error
after DCNN_DIST_TIMEOUT instead of hanging. The GPU variant runs the same program on the RCCL
plane at world 1 (eager and captured step)."""
import os
import socket
import subprocess
import time

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "dcnn_amd", "bin", "dp_selftest")


@pytest.fixture(scope="module")
def exe():
    if not (os.path.exists(BIN) and torch.cuda.is_available()):
        from dcnn_amd import _build
        _build.build_host()
    return BIN


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _launch(exe, world, out, device="CPU", extra=(), timeout=120, env_extra=None):
    port = _port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), **(env_extra or {}))
        procs.append(subprocess.Popen([exe, "--device", device, "--out", str(out), *extra], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    outs = []
    for p in procs:
        try:
            o, _ = p.communicate(timeout=timeout)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        outs.append((p.returncode, o))
    return outs


def _load(path):
    blocks = []
    with open(path, "rb") as f:
        for _ in range(3):
            n = int(np.frombuffer(f.read(8), dtype=np.uint64)[0])
            blocks.append(np.frombuffer(f.read(4 * n), dtype=np.float32))
    return blocks


@pytest.mark.parametrize("world", [2, 4])
def test_cpp_dp_ranks_equal_single_process(exe, tmp_path, world):
    for rc, o in _launch(exe, 1, tmp_path):
        assert rc == 0, o
    outs = _launch(exe, world, tmp_path)
    for rc, o in outs:
        assert rc == 0, o
        assert '"plane": "tcp"' in o and '"buckets": 3' in o, o
        assert f'"max_rank": {world - 1}.0' in o, o
    g1, p1, b1 = _load(tmp_path / "w1r0.bin")
    ranks = [_load(tmp_path / f"w{world}r{r}.bin") for r in range(world)]
    for g, p, b in ranks[1:]:  # identical replicas
        assert np.array_equal(g, ranks[0][0]) and np.array_equal(p, ranks[0][1])
        assert np.array_equal(b, ranks[0][2])
    g, p, b = ranks[0]
    # mean of the shard gradients == the whole-batch gradient (fp32, summation order differs)
    np.testing.assert_allclose(g, g1, rtol=1e-4, atol=2e-6)
    np.testing.assert_allclose(p, p1, rtol=1e-4, atol=2e-6)
    assert np.abs(g1).max() > 1e-3  # (a real gradient)
    # broadcast_parameters: rank 0's seed and running statistics everywhere
    assert np.array_equal(b, b1)


def test_cpp_dp_deterministic_reruns(exe, tmp_path):
    a, b = tmp_path / "a", tmp_path / "b"
    a.mkdir()
    b.mkdir()
    for d in (a, b):
        for rc, o in _launch(exe, 3, d, extra=("--batch", "12")):
            assert rc == 0, o
    for r in range(3):
        for x, y in zip(_load(a / f"w3r{r}.bin"), _load(b / f"w3r{r}.bin")):
            assert np.array_equal(x, y)


@pytest.mark.parametrize("alone", [0, 1])
def test_cpp_dp_rendezvous_timeout(exe, tmp_path, alone):
    """One rank of a world-2 job started alone: rank 0's accept / rank 1's connect give up."""
    port = _port()
    env = dict(os.environ, RANK=str(alone), WORLD_SIZE="2", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
               DCNN_DIST_TIMEOUT="2")
    t0 = time.time()
    r = subprocess.run([exe, "--device", "CPU", "--out", str(tmp_path)], env=env, stdout=subprocess.PIPE,
                       stderr=subprocess.STDOUT, text=True, timeout=60)
    assert r.returncode != 0
    assert "timed out" in r.stdout, r.stdout
    assert time.time() - t0 < 30


@pytest.mark.gpu
@pytest.mark.parametrize("graph", [False, True])
def test_gpu_cpp_dp_rccl_world1(exe, tmp_path, graph):
    """The RCCL plane at world 1: the bucketed mean inside the (captured) step leaves the gradient
    and the update unchanged against the same program without the mean."""
    extra = ("--graph",) if graph else ()
    a, b = tmp_path / "dp", tmp_path / "nodp"
    a.mkdir()
    b.mkdir()
    for rc, o in _launch(exe, 1, a, device="GPU", extra=extra):
        assert rc == 0, o
        assert '"plane": "rccl"' in o and '"buckets": 3' in o, o
    for rc, o in _launch(exe, 1, b, device="GPU", extra=extra + ("--no-dp",)):
        assert rc == 0, o
    for x, y in zip(_load(a / "w1r0.bin"), _load(b / "w1r0.bin")):
        assert np.array_equal(x, y)


@pytest.mark.gpu
def test_gpu_cpp_dp_unique_id_rendezvous_world3(exe, tmp_path):
    """The GPU plane's rendezvous at world 3: rank 0's RCCL unique id reaches every rank over TCP
    (exchange_unique_id; the communicator itself needs one GPU per rank, which one box lacks)."""
    outs = _launch(exe, 3, tmp_path, device="UID", timeout=120)
    hashes = set()
    for rc, o in outs:
        assert rc == 0, o
        line = [l for l in o.splitlines() if l.startswith("{")][-1]
        d = __import__("json").loads(line)
        assert d["uid_bytes"] == 128
        hashes.add(d["uid_hash"])
    assert len(hashes) == 1, hashes
