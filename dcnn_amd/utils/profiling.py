"""Profiling helpers.

* ``ProfilerType`` — NONE / NORMAL (cleared every batch) / CUMULATIVE, as in the reference
  trainer (include/nn/train.hpp:37,87-94).
* ``roctx_range`` — ROCTx ranges (visible in ``rocprofv3 --marker-trace``) via torch's
  profiler hooks; no-op on the CPU.
* ``benchmark`` — host wall-clock timer helper (reference include/utils/misc.hpp:25).
* ``DeviceTimer`` — HIP-event device timing of a region on the current stream.
"""
from __future__ import annotations

import contextlib
import enum
import time
from typing import Callable

import torch


class ProfilerType(enum.Enum):
    NONE = 0
    NORMAL = 1
    CUMULATIVE = 2

    @classmethod
    def parse(cls, s) -> "ProfilerType":
        if isinstance(s, ProfilerType):
            return s
        return cls[str(s).strip().upper()] if str(s).strip() else cls.NONE


@contextlib.contextmanager
def roctx_range(name: str):
    on = torch.cuda.is_available()
    if on:
        torch.cuda.nvtx.range_push(name)  # routed to roctx on ROCm builds
    try:
        yield
    finally:
        if on:
            torch.cuda.nvtx.range_pop()


def benchmark(fn: Callable, iters: int = 1) -> float:
    """Average wall time of ``fn()`` in milliseconds."""
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    return (time.perf_counter() - t0) * 1e3 / max(iters, 1)


class DeviceTimer:
    """``with DeviceTimer() as t: ...; t.ms`` — GPU time of the enclosed stream work."""

    def __enter__(self):
        self.gpu = torch.cuda.is_available()
        if self.gpu:
            self.e0 = torch.cuda.Event(enable_timing=True)
            self.e1 = torch.cuda.Event(enable_timing=True)
            self.e0.record()
        else:
            self.t0 = time.perf_counter()
        return self

    def __exit__(self, *exc):
        if self.gpu:
            self.e1.record()
        else:
            self.t1 = time.perf_counter()

    @property
    def ms(self) -> float:
        if self.gpu:
            self.e1.synchronize()
            return self.e0.elapsed_time(self.e1)
        return (self.t1 - self.t0) * 1e3
