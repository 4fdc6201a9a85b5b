"""In-tree RCCL communicator (csrc/kernels/rccl.cpp) with its bootstrap over the framework's own
TCP control plane (csrc/native/comm.cpp).

``torch.distributed``'s ProcessGroupNCCL stays the default data plane; this is the framework-owned
alternative (``DCNN_DP_BACKEND=rccl`` / ``DataParallel(comm_backend="rccl")``):

* rank 0 creates the 128-byte ``ncclUniqueId`` and serves it from a native ``TcpCommunicator``;
  every other rank connects, sends ``STATUS_REQUEST`` and receives the id in a
  ``STATUS_RESPONSE`` text payload — no TCPStore / c10d rendezvous involved;
* ``ncclCommInitRank`` then builds the communicator; collectives take raw device pointers and
  the caller's current HIP stream, so they are captured into the step's hipGraph like any other
  kernel (no side stream, no host synchronisation).

Reference parity: the reference's only data plane is host fp32 over TCP
(include/pipeline/tcp_communicator.hpp:113-151 for the connection bootstrap); SURVEY §5.8 maps it
to RCCL on MI355X.
"""
from __future__ import annotations

import os
import time
from typing import Optional

import torch

DTYPES = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2, torch.int32: 3, torch.uint8: 4, torch.int8: 4}
OPS = {"sum": 0, "prod": 1, "max": 2, "min": 3, "avg": 4}


def _native():
    from ..ops._ext import native
    return native()


def exchange_unique_id(rank: int, world: int, host: str, port: int, make_id=None, timeout_s: float = 60.0) -> bytes:
    """Agree on one 128-byte id: rank 0 makes it (``make_id``, default ``rccl.unique_id``) and
    serves it on ``host:port``; ranks 1..world-1 fetch it. Uses only the native TCP communicator."""
    from .pipeline import messages as M
    comm_mod = _native().comm
    C = M.CommandType
    if rank == 0:
        if make_id is None:
            from ..ops._ext import kernels
            make_id = kernels().rccl.unique_id
        uid = make_id()
        srv = comm_mod.TcpCommunicator("rccl_root", "0.0.0.0", port)
        try:
            served = 0
            deadline = time.time() + timeout_s
            while served < world - 1:
                left = int(max(1.0, deadline - time.time()) * 1000)
                msg = srv.recv_command(int(C.STATUS_REQUEST), left)
                if msg is None:
                    raise TimeoutError(f"rccl bootstrap: {served}/{world - 1} ranks fetched the id")
                rep = comm_mod.Message(msg.sender, int(C.STATUS_RESPONSE))
                rep.text = uid
                srv.send(rep)
                served += 1
            # every requester has its reply queued: give the writers a moment before closing
            time.sleep(0.05)
        finally:
            srv.close()
        return uid
    cli = comm_mod.TcpCommunicator(f"rccl_rank{rank}", "0.0.0.0", 0)
    try:
        deadline = time.time() + timeout_s
        while True:
            try:
                cli.connect("rccl_root", host, port, 2000)
                break
            except Exception:
                if time.time() > deadline:
                    raise
                time.sleep(0.1)
        cli.send(comm_mod.Message("rccl_root", int(C.STATUS_REQUEST)))
        rep = cli.recv_command(int(C.STATUS_RESPONSE), int(timeout_s * 1000))
        if rep is None:
            raise TimeoutError("rccl bootstrap: no id from rank 0")
        uid = bytes(rep.text)
    finally:
        cli.close()
    if len(uid) != 128:
        raise RuntimeError(f"rccl bootstrap: id of {len(uid)} bytes")
    return uid


class RcclCommunicator:
    """One RCCL communicator over ``world`` processes (one per GPU)."""

    def __init__(self, rank: int, world: int, device: Optional[torch.device] = None,
                 host: Optional[str] = None, port: Optional[int] = None, unique_id: Optional[bytes] = None):
        from ..ops._ext import kernels
        K = kernels()
        if not K.rccl.available():
            raise RuntimeError(K.rccl.load_error())
        self.rank, self.world = int(rank), int(world)
        self.device = device if device is not None else torch.device("cuda", torch.cuda.current_device())
        if unique_id is None:
            host = host or os.environ.get("MASTER_ADDR", "127.0.0.1")
            port = port or int(os.environ.get("DCNN_RCCL_PORT", int(os.environ.get("MASTER_PORT", "29500")) + 17))
            unique_id = K.rccl.unique_id() if self.world == 1 else exchange_unique_id(self.rank, self.world, host, port)
        self._c = K.rccl.Comm(unique_id, self.world, self.rank, self.device.index or 0)

    @staticmethod
    def _stream(t):
        from ..ops._ext import stream_ptr
        return stream_ptr(t.device)

    def all_reduce(self, t: torch.Tensor, op: str = "sum", out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """In-place (or into ``out``) all-reduce of a contiguous device tensor on the current stream."""
        assert t.is_cuda and t.is_contiguous()
        out = t if out is None else out
        self._c.all_reduce(t.data_ptr(), out.data_ptr(), t.numel(), DTYPES[t.dtype], OPS[op], self._stream(t))
        return out

    def broadcast(self, t: torch.Tensor, root: int = 0) -> torch.Tensor:
        assert t.is_cuda and t.is_contiguous()
        self._c.broadcast(t.data_ptr(), t.data_ptr(), t.numel(), DTYPES[t.dtype], int(root), self._stream(t))
        return t

    def all_gather(self, out: torch.Tensor, t: torch.Tensor) -> torch.Tensor:
        assert out.numel() == t.numel() * self.world
        self._c.all_gather(t.data_ptr(), out.data_ptr(), t.numel(), DTYPES[t.dtype], self._stream(t))
        return out

    def reduce_scatter(self, out: torch.Tensor, t: torch.Tensor, op: str = "sum") -> torch.Tensor:
        assert t.numel() == out.numel() * self.world
        self._c.reduce_scatter(t.data_ptr(), out.data_ptr(), out.numel(), DTYPES[t.dtype], OPS[op], self._stream(t))
        return out

    def send(self, t: torch.Tensor, peer: int) -> None:
        self._c.send(t.data_ptr(), t.numel(), DTYPES[t.dtype], int(peer), self._stream(t))

    def recv(self, t: torch.Tensor, peer: int) -> torch.Tensor:
        self._c.recv(t.data_ptr(), t.numel(), DTYPES[t.dtype], int(peer), self._stream(t))
        return t

    def close(self) -> None:
        self._c.destroy()
