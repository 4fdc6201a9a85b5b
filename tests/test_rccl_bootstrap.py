"""In-tree RCCL communicator bootstrap (parallel/rccl.py): the 128-byte unique id travels from
rank 0 to every rank over the native TCP control plane (csrc/native/comm.cpp), between real
processes. CPU only: the id is synthetic here; tests/test_gpu_rccl.py runs the communicator."""
import multiprocessing as mp
import os
import socket


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, q):
    from dcnn_amd.parallel.rccl import exchange_unique_id
    uid = exchange_unique_id(rank, world, "127.0.0.1", port, make_id=lambda: bytes(range(128)), timeout_s=30)
    q.put((rank, uid))


def test_unique_id_exchange_over_native_tcp():
    world, port = 4, _port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_rank, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(world))
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    assert sorted(got) == list(range(world))
    assert all(v == bytes(range(128)) for v in got.values())


def test_rccl_library_loads():
    from dcnn_amd.ops._ext import kernels
    K = kernels()
    assert K.rccl.available(), K.rccl.load_error()
    assert K.rccl.version() > 20000
