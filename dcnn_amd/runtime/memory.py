"""Memory pool / temporary buffers (reference include/nn/mem_pool.hpp:11-101, device_ptr
``ensure`` semantics include/device/device_ptr.hpp:184).

GPU allocations already go through PyTorch's stream-ordered caching allocator (graph-capture
aware), so this pool is a thin size-keyed free list on top of it for callers that want the
reference's explicit borrow/return discipline: ``with pool.borrow(numel, dtype) as buf: ...``.
``GrowBuffer`` reproduces ``device_ptr::ensure`` (grow-only reallocation).
"""
from __future__ import annotations

import bisect
import threading
from contextlib import contextmanager
from typing import Dict, List, Tuple

import torch


class MemPool:
    def __init__(self, device="cpu", max_cached: int = 64):
        self.device = torch.device(device) if not isinstance(device, torch.device) else device
        self.max_cached = max_cached
        self._free: Dict[torch.dtype, List[Tuple[int, int, torch.Tensor]]] = {}
        self._lock = threading.Lock()
        self._seq = 0
        self.hits = self.misses = 0

    def get(self, numel: int, dtype=torch.float32) -> torch.Tensor:
        """A flat buffer with at least ``numel`` elements (smallest cached fit, else new)."""
        with self._lock:
            lst = self._free.setdefault(dtype, [])
            i = bisect.bisect_left(lst, (numel, -1))
            if i < len(lst):
                _, _, t = lst.pop(i)
                self.hits += 1
                return t[:numel]
            self.misses += 1
        return torch.empty(numel, dtype=dtype, device=self.device)

    def put(self, t: torch.Tensor) -> None:
        base = t._base if t._base is not None else t
        with self._lock:
            lst = self._free.setdefault(base.dtype, [])
            self._seq += 1
            bisect.insort(lst, (base.numel(), self._seq, base))
            if sum(len(v) for v in self._free.values()) > self.max_cached:
                lst.pop(-1)  # drop the largest cached buffer

    @contextmanager
    def borrow(self, numel: int, dtype=torch.float32):
        """RAII temporary (reference TempBuffer)."""
        t = self.get(numel, dtype)
        try:
            yield t
        finally:
            self.put(t)

    def clear(self) -> None:
        with self._lock:
            self._free.clear()

    def cached_bytes(self) -> int:
        with self._lock:
            return sum(t.numel() * t.element_size() for v in self._free.values() for _, _, t in v)


class GrowBuffer:
    """Grow-only device buffer (``device_ptr::ensure``): reallocates only when more is needed."""

    def __init__(self, device="cpu", dtype=torch.float32):
        self.device, self.dtype = device, dtype
        self.buf = torch.empty(0, dtype=dtype, device=device)

    def ensure(self, numel: int) -> torch.Tensor:
        if self.buf.numel() < numel:
            self.buf = torch.empty(numel, dtype=self.dtype, device=self.device)
        return self.buf[:numel]

    @property
    def capacity(self) -> int:
        return self.buf.numel()
