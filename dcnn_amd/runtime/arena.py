"""Per-step activation arena on the native runtime (csrc/kernels/runtime.cpp ``ActArena``).

Inside ``with arena.step():`` every activation / statistics slab / workspace the GPU op layer
(:mod:`dcnn_amd.ops.hip`) creates is a strided view into a device chunk the native runtime owns:

* one bump pointer per step, reset at the next step — a training step makes no allocator call
  per tensor and reuses the same addresses every step (eager steps and the captured hipGraph see
  the same buffers);
* growth only on first use: an overrun appends a chunk, the next step coalesces the chunks into
  one of the high-water size; from the second step on nothing grows (``stats()["grows"]``);
* during a graph capture the arena is frozen (a chunk allocation would be recorded into the
  graph): requests that do not fit fall back to PyTorch's allocator (graph pool) and are counted
  as ``refused``;
* tensors that escape a step keep their chunk alive (DLPack shared ownership), but their
  contents are overwritten by the next step — only per-step data goes here; the persistent
  buffers (ticket words, weight operands) come from :meth:`Device.allocate`.

Reference parity: the reference allocates every activation through ``Tensor::ensure`` /
``device_ptr`` on its own pool (include/tensor/tensor.hpp:424-511,
include/device/device_ptr.hpp:184-217, include/nn/mem_pool.hpp:11-101).
"""
from __future__ import annotations

import os
import threading
import weakref
from contextlib import contextmanager
from typing import Dict, List, Optional

import torch

_tls = threading.local()
_registry: "weakref.WeakSet[ActivationArena]" = weakref.WeakSet()
_ENABLED = os.environ.get("DCNN_ARENA", "1") != "0"


def enabled() -> bool:
    return _ENABLED


def set_enabled(on: bool) -> None:
    global _ENABLED
    _ENABLED = bool(on)


def active() -> Optional["ActivationArena"]:
    """The arena of the step running on this thread, or None."""
    return getattr(_tls, "arena", None)


class ActivationArena:
    def __init__(self, device_index: int = 0, initial_mb: Optional[int] = None):
        from ..ops._ext import kernels
        mb = int(initial_mb if initial_mb is not None else os.environ.get("DCNN_ARENA_MB", "256"))
        self.device_index = int(device_index)
        self._n = kernels().rt.ActArena(self.device_index, mb << 20)
        self._bases: Dict[int, Dict[torch.dtype, torch.Tensor]] = {}
        self.fallbacks = 0
        _registry.add(self)

    # ------------------------------------------------------------------ allocation
    def _base(self, cid: int, dtype: torch.dtype) -> torch.Tensor:
        views = self._bases.get(cid)
        if views is None:
            views = {torch.uint8: torch.from_dlpack(self._n.chunk(cid))}
            self._bases[cid] = views
        b = views.get(dtype)
        if b is None:
            u = views[torch.uint8]
            es = torch.empty((), dtype=dtype).element_size()
            b = u[: u.numel() // es * es].view(dtype)
            views[dtype] = b
        return b

    def empty(self, shape, dtype, channels_last: bool = False) -> torch.Tensor:
        """An uninitialised (N,C,H,W)-shaped tensor (``channels_last``: NHWC strides) or a dense
        row-major one, carved from this step's chunk."""
        shape = tuple(int(s) for s in shape)
        numel = 1
        for s in shape:
            numel *= s
        es = _ES[dtype]
        cid, off = self._n.alloc(numel * es)
        if cid < 0:  # frozen (capture) and out of room: the graph pool takes it
            self.fallbacks += 1
            mf = torch.channels_last if channels_last else torch.contiguous_format
            return torch.empty(shape, dtype=dtype, device=torch.device("cuda", self.device_index), memory_format=mf)
        base = self._base(cid, dtype)
        if channels_last:
            N, C, H, W = shape
            stride = (H * W * C, 1, W * C, C)
        else:
            stride, acc = [], 1
            for s in reversed(shape):
                stride.append(acc)
                acc *= s
            stride = tuple(reversed(stride))
        return base.as_strided(shape, stride, off // es)

    # ------------------------------------------------------------------ step scope
    @contextmanager
    def step(self, capture: bool = False):
        """Scope of one training step on the current stream (``capture``: a graph is being
        captured — nothing may allocate)."""
        from ..ops._ext import stream_ptr
        prev = active()
        if self._n.reset(stream_ptr()):
            self._bases.clear()  # chunks were coalesced: the old views die with their tensors
        self._n.set_frozen(bool(capture))
        _tls.arena = self
        try:
            yield self
        finally:
            _tls.arena = prev
            self._n.set_frozen(False)

    def pin(self) -> List[torch.Tensor]:
        """The live chunks as tensors: a captured graph holds these so a later coalesce cannot
        return memory the graph still addresses."""
        return [v[torch.uint8] for v in self._bases.values()]

    def stats(self) -> dict:
        d = dict(self._n.stats())
        d["fallbacks"] = self.fallbacks
        return d


_ES = {torch.float32: 4, torch.float64: 8, torch.float16: 2, torch.bfloat16: 2, torch.int32: 4, torch.int64: 8,
       torch.int16: 2, torch.int8: 1, torch.uint8: 1, torch.bool: 1}


def empty(shape, dtype, device, channels_last: bool = False) -> torch.Tensor:
    """Per-step buffer: from the active arena when one is open on this thread for ``device``,
    else PyTorch's allocator."""
    a = getattr(_tls, "arena", None)
    if a is not None and device.type == "cuda" and (device.index or 0) == a.device_index:
        return a.empty(shape, dtype, channels_last)
    mf = torch.channels_last if channels_last else torch.contiguous_format
    return torch.empty(shape, dtype=dtype, device=device, memory_format=mf)


def persistent(shape, dtype, device, zero: bool = False) -> torch.Tensor:
    """Long-lived buffer (ticket words, weight operands) from the native device pool."""
    from ..device import get_device
    if device.type != "cuda":
        return torch.zeros(shape, dtype=dtype) if zero else torch.empty(shape, dtype=dtype)
    if torch.cuda.is_current_stream_capturing():
        # a pool allocation here would be recorded into the graph: the graph's own pool keeps it
        t = torch.empty(shape, dtype=dtype, device=device)
    else:
        t = get_device(f"GPU:{device.index or 0}").allocate(shape if not isinstance(shape, int) else [shape], dtype)
    if zero:
        from ..ops.hip import zero_
        zero_(t)
    return t


def device_stats(device_index: int) -> dict:
    """Summed statistics of the live arenas on one device (Device.allocator_stats)."""
    out = {"arenas": 0, "arena_capacity_bytes": 0, "arena_high_water_bytes": 0, "arena_grows": 0}
    for a in list(_registry):
        if a.device_index != device_index:
            continue
        st = a._n.stats()
        out["arenas"] += 1
        out["arena_capacity_bytes"] += int(st["capacity_bytes"])
        out["arena_high_water_bytes"] += int(st["high_water_bytes"])
        out["arena_grows"] += int(st["grows"])
    return out
