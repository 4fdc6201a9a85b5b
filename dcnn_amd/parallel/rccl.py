"""In-tree RCCL data plane (csrc/kernels/rccl.cpp) with its bootstrap over the framework's own
TCP control plane (csrc/native/comm.cpp) — the default gradient and pipeline data plane on GPUs
(``bench.py --dp-backend rccl``, ``DataParallel(comm_backend="rccl")``, pipeline ``--p2p rccl``);
``torch.distributed`` (ProcessGroupNCCL) is the fallback:

* rank / world come from the launcher's environment (RANK, WORLD_SIZE, MASTER_ADDR); rank 0
  creates the 128-byte ``ncclUniqueId`` (or several, one per communicator) and serves them from a
  native ``TcpCommunicator``; every other rank connects, sends ``STATUS_REQUEST`` and receives the
  ids in a ``STATUS_RESPONSE`` text payload — no TCPStore / c10d rendezvous involved;
* ``ncclCommInitRank`` then builds each communicator; collectives take raw device pointers and a
  HIP stream, so they are captured into the step's hipGraph like any other kernel.
* Streams: callers enqueue on framework comm streams forked from / joined to the compute stream
  with events (``CommStream``), so collectives overlap compute and, for pipeline P2P, forward and
  backward traffic never queue behind each other (``RcclP2P``: one communicator and one stream
  per direction).

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


def env_rank_world():
    """(rank, world, local_rank) from the launcher's environment (torchrun / the driver)."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def bootstrap_port(offset: int = 17) -> int:
    return int(os.environ.get("DCNN_RCCL_PORT", int(os.environ.get("MASTER_PORT", "29500")) + offset))


def exchange_unique_id(rank: int, world: int, host: str, port: int, make_id=None, timeout_s: float = 60.0,
                       nbytes: int = 128) -> bytes:
    """Agree on one ``nbytes`` id blob (one or more 128-byte ids): rank 0 makes it (``make_id``,
    default ``rccl.unique_id``) and serves it on ``host:port``; ranks 1..world-1 fetch it. Uses only
    the native TCP communicator."""
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
    if len(uid) != nbytes:
        raise RuntimeError(f"rccl bootstrap: id of {len(uid)} bytes (expected {nbytes})")
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
            port = port or bootstrap_port()
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

    # ---- host-side helpers (no c10d): a barrier and scalar reductions over the communicator
    def barrier(self) -> None:
        """Every rank has reached this point (a 1-element all-reduce, then a device sync)."""
        t = torch.ones(1, device=self.device)
        self.all_reduce(t)
        torch.cuda.synchronize(self.device)

    def reduce_scalar(self, v: float, op: str = "max") -> float:
        t = torch.tensor([float(v)], dtype=torch.float32, device=self.device)
        self.all_reduce(t, op)
        return float(t.item())


class CommStream:
    """A framework comm stream: ``fork()`` makes it wait for the compute stream (the data it will
    move is complete there), ``join()`` makes the compute stream wait for everything enqueued on
    it. Both are event edges, so inside a hipGraph capture they become graph dependencies and the
    collectives overlap the compute that follows the fork."""

    def __init__(self, device):
        self.device = torch.device(device)
        self.stream = torch.cuda.Stream(device=self.device)
        self.forked = False

    def fork(self):
        self.stream.wait_stream(torch.cuda.current_stream(self.device))
        self.forked = True
        return torch.cuda.stream(self.stream)

    def join(self):
        if self.forked:
            torch.cuda.current_stream(self.device).wait_stream(self.stream)
            self.forked = False


P2P_KEYS = ("fwd", "bwd", "cfwd", "cbwd")


class RcclP2P:
    """Pipeline point-to-point plane: one in-tree communicator and one HIP stream per direction
    (stage -> stage forward activations, stage -> stage backward gradients, and the coordinator's
    two directions). A send or receive waits for the compute stream (its data is produced, or its
    receive slot is free), runs on its direction's stream, and a receive's consumer waits for it —
    so a stage blocked in ``ncclSend`` of a large forward activation can never hold up the
    ``ncclRecv`` of a backward gradient (the hazard of one communicator on one stream: two
    neighbours each blocked in a send whose matching receive is queued behind the other's send).
    Within one direction traffic flows one way between any two ranks, so sends and receives pair
    up in message order."""

    def __init__(self, rank: int, world: int, device=None, host: Optional[str] = None, port: Optional[int] = None,
                 keys=P2P_KEYS):
        from ..ops._ext import kernels
        K = kernels()
        if not K.rccl.available():
            raise RuntimeError(K.rccl.load_error())
        self.rank, self.world = int(rank), int(world)
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.keys = tuple(keys)
        n = len(self.keys)
        make = lambda: b"".join(K.rccl.unique_id() for _ in range(n))
        if self.world == 1:
            blob = make()
        else:
            blob = exchange_unique_id(self.rank, self.world, host or os.environ.get("MASTER_ADDR", "127.0.0.1"),
                                      port or bootstrap_port(19), make_id=make, nbytes=128 * n)
        self.comms = {k: RcclCommunicator(self.rank, self.world, self.device, unique_id=blob[128 * i:128 * (i + 1)])
                      for i, k in enumerate(self.keys)}
        self.streams = {k: torch.cuda.Stream(device=self.device) for k in self.keys}

    def send(self, key: str, t: torch.Tensor, peer: int) -> None:
        s = self.streams[key]
        s.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(s):
            self.comms[key].send(t, peer)
        t.record_stream(s)  # the caching allocator keeps t until the send has left

    def recv(self, key: str, t: torch.Tensor, peer: int) -> torch.Tensor:
        main = torch.cuda.current_stream(self.device)
        s = self.streams[key]
        s.wait_stream(main)  # the receive slot's previous consumer has finished with it
        with torch.cuda.stream(s):
            self.comms[key].recv(t, peer)
        main.wait_stream(s)
        return t

    def barrier(self) -> None:
        self.comms[self.keys[0]].barrier()

    def close(self) -> None:
        for c in self.comms.values():
            c.close()
