"""Pipeline data plane: how FORWARD_JOB / BACKWARD_JOB tensors move between stages.

* ``MessageTransport`` — tensors inline in the control message (host copy; TCP between
  machines or processes without RCCL).  The reference's only mode
  (include/pipeline/binary_serializer.hpp:27-35).
* ``LocalTransport`` — peers in the same process (in-process coordinator, or coordinator +
  stage 0 sharing a rank): the tensor object is handed over through a process-wide mailbox,
  the message carries only metadata; a device change is one ``.to()`` (xGMI peer copy
  between GPUs). Every stage computes on its own stream, so a GPU tensor travels with an
  event recorded on the producer's stream: the consumer's stream waits on it (no host sync)
  and the tensor is marked as used by the consumer stream for the caching allocator.
* ``P2PTransport`` — one process per GPU under ``torch.distributed``: metadata rides the
  control plane, bytes go device-to-device with ``isend``/``irecv`` (RCCL over xGMI with the
  "nccl" backend, gloo on CPU).  Forward activations and backward gradients use *separate*
  process groups (separate RCCL communicators and streams), so a stage that interleaves
  forward and backward micro-batches can never head-of-line block a peer; the coordinator's
  traffic gets its own pair of groups as well.  Peers living in the same rank fall back to
  the local mailbox. With RCCL, ``Work.wait()`` on a receive makes the *current stream* wait for
  the communicator's stream — the host thread does not block — so a stage posts its receive
  and immediately enqueues the micro-batch's compute behind it.
"""
from __future__ import annotations

import threading
from collections import deque
from typing import Dict, Optional

import torch
import torch.distributed as dist

from . import messages as M


class _Mailbox:
    def __init__(self):
        self._d: Dict = {}
        self._cv = threading.Condition()

    def put(self, key, t):
        with self._cv:
            self._d.setdefault(key, deque()).append(t)
            self._cv.notify_all()

    def take(self, key, timeout=60.0):
        with self._cv:
            ok = self._cv.wait_for(lambda: bool(self._d.get(key)), timeout)
            if not ok:
                raise TimeoutError(f"local mailbox: no tensor for {key}")
            q = self._d[key]
            t = q.popleft()
            if not q:
                del self._d[key]
            return t

    def purge(self, target_prefix: str) -> int:
        """Drop every undelivered tensor addressed to a comm id starting with ``target_prefix``
        (pipeline recovery: activations of a failed attempt must not be claimed by its retry)."""
        with self._cv:
            dead = [k for k in self._d if str(k[0]).startswith(target_prefix)]
            for k in dead:
                del self._d[k]
            return len(dead)


MAILBOX = _Mailbox()


def _stamp(t: Optional[torch.Tensor]):
    """Mailbox entry: the tensor and, for a GPU tensor, an event on the producer's stream."""
    if t is not None and t.is_cuda:
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(t.device))
        return t, ev
    return t, None


def _claim(entry, device) -> torch.Tensor:
    """Order the consumer's stream(s) after the producer and move to ``device`` if needed."""
    t, ev = entry
    dev = torch.device(device) if device is not None else t.device
    if ev is not None:
        s = torch.cuda.current_stream(t.device)
        s.wait_event(ev)
        t.record_stream(s)
        if dev.type == "cuda" and dev != t.device:
            torch.cuda.current_stream(dev).wait_event(ev)
    if dev != t.device:
        t = t.to(dev, non_blocking=True)
    return t


class Transport:
    """send(comm, recipient, command, mb_id, tensor) / recv(msg, device)."""

    def send(self, comm, recipient: str, command: int, mb_id: int, t: Optional[torch.Tensor]) -> None:
        raise NotImplementedError

    def recv(self, msg, device) -> Optional[torch.Tensor]:
        raise NotImplementedError

    def flush(self) -> None:
        pass


class MessageTransport(Transport):
    def __init__(self, codec: str = "none", legacy: bool = False):
        self.codec = codec
        self.legacy = legacy

    def send(self, comm, recipient, command, mb_id, t):
        comm.send(M.job_message(recipient, command, mb_id, t, self.codec, self.legacy))

    def recv(self, msg, device):
        return M.message_tensor(msg, device)


class LocalTransport(Transport):
    """Tensor objects through the process mailbox; key = (recipient comm id, command, mb)."""

    def __init__(self, my_id: str, resolve=None):
        self.my_id = my_id
        self.resolve = resolve or (lambda name: name)

    def send(self, comm, recipient, command, mb_id, t):
        target = self.resolve(recipient)
        if t is not None:
            MAILBOX.put((target, int(command), int(mb_id)), _stamp(t))
        comm.send(M.meta_message(recipient, command, mb_id, t))

    def recv(self, msg, device):
        if not M.has_tensor(msg):
            return None
        return _claim(MAILBOX.take((self.my_id, int(msg.command), int(msg.mb_id))), device)


class P2PTransport(Transport):
    """Point-to-point data plane between ranks: torch.distributed isend/irecv (RCCL on GPU, gloo
    on CPU), or the framework's own RCCL plane (``rccl=`` a :class:`parallel.rccl.RcclP2P`: one
    communicator and one HIP stream per direction — forward, backward, and the coordinator's two —
    forked from / joined to the compute stream with events, no Work objects).

    Receive buffers are persistent slots keyed by (peer, command, micro-batch, shape, dtype): a
    steady-state step allocates nothing (the previous step's tensor in that slot is dead by then —
    a stage consumes a micro-batch's activation / gradient within the step)."""

    def __init__(self, my_id: str, ranks: Dict[str, int], groups, resolve=None, rccl=None):
        from ..rccl import RcclP2P
        if rccl is None and isinstance(groups, RcclP2P):  # the launcher hands the in-tree plane over
            rccl, groups = groups, None
        self.my_id = my_id
        self.ranks = dict(ranks)          # logical name / comm id -> rank
        self.groups = groups              # torch process groups {"fwd", "bwd", "cfwd", "cbwd"}
        self.rank = dist.get_rank() if rccl is None else rccl.rank
        self.local = LocalTransport(my_id, resolve)
        self.rccl = rccl
        self._pending = deque()
        self._slots: Dict = {}
        self.slot_allocs = 0              # receive buffers ever allocated (tests: flat after step 1)

    def _key(self, command, peer_name):
        coord = "coordinator" in (peer_name, self.my_id)
        if int(command) == M.CommandType.FORWARD_JOB:
            return "cfwd" if coord else "fwd"
        return "cbwd" if coord else "bwd"

    def _group(self, command, peer_name):
        return self.groups[self._key(command, peer_name)]

    def _prune(self):
        while self._pending and self._pending[0][0].is_completed():
            self._pending.popleft()

    def send(self, comm, recipient, command, mb_id, t):
        dst = self.ranks[recipient]
        if dst == self.rank:
            self.local.send(comm, recipient, command, mb_id, t)
            return
        if t is not None:
            phys, _ = M._physical(t.detach())
            if not phys.is_contiguous():
                phys = phys.contiguous()
            if self.rccl is not None:
                self.rccl.send(self._key(command, recipient), phys, dst)  # direction stream; phys kept alive
            else:
                w = dist.isend(phys, dst, group=self._group(command, recipient))
                self._pending.append((w, phys))
                self._prune()
        comm.send(M.meta_message(recipient, command, mb_id, t))

    def _slot(self, msg, src, dev):
        key = (src, int(msg.command), int(msg.mb_id), tuple(msg.shape), int(msg.dtype), str(dev))
        buf = self._slots.get(key)
        if buf is None:
            buf = self._slots[key] = M.alloc_for(msg, dev)
            self.slot_allocs += 1
        return buf

    def recv(self, msg, device):
        if not M.has_tensor(msg):
            return None
        src_name = msg.sender
        src = self.ranks.get(src_name)
        if src is None or src == self.rank:
            return self.local.recv(msg, device)
        dev = torch.device(device) if device is not None else torch.device("cpu")
        phys, logical = self._slot(msg, src, dev)
        if self.rccl is not None:
            self.rccl.recv(self._key(msg.command, src_name), phys, src)
        else:
            dist.irecv(phys, src, group=self._group(msg.command, src_name)).wait()
        return logical

    def flush(self):
        while self._pending:
            w, _ = self._pending.popleft()
            w.wait()


def make_groups(backend: Optional[str] = None) -> Dict[str, object]:
    """Create the four P2P process groups (all ranks must call this in the same order)."""
    world = list(range(dist.get_world_size()))
    return {k: dist.new_group(world, backend=backend) for k in ("fwd", "bwd", "cfwd", "cbwd")}
