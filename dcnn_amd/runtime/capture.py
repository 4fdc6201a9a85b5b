"""Graph-capture hygiene shared by every hipGraph capture site.

A capture must not interleave with HIP object teardown: Python's cyclic garbage collector runs
finalizers on whichever thread crosses its allocation threshold, and a finalizer that destroys
a HIP event, stream or graph (an abandoned pipeline stage, a tensor exported from the native
pool) while another thread — or the capturing thread itself — is inside a stream capture can
invalidate that capture and abort the process. ``capture_guard`` keeps the collector off while
any capture is in progress anywhere in the process (counted, so overlapping captures on stage
threads compose) and runs one collection before the first capture starts, at a point where no
capture is active yet.

It also retires ProcessGroupNCCL's eager work before a capture starts. The process group's
watchdog thread polls the end event of every eager collective it still lists (one pass every
~100 ms). A capture that issues collectives pulls the group's internal stream into the capture; a
watchdog query of an eager work's event recorded on that stream, made while the capture is open,
fails (hipErrorCapturedEvent "operation not permitted on an event last recorded in a capturing
stream", or hipErrorStreamCaptureUnsupported), and the watchdog aborts the process. That was the
intermittent SIGABRT of the world-1 RCCL capture tests (gpurun_out/t_m9..t_m11 in round 5; probe:
tools/pg_capture_probe.py). ``drain_collective_watchdog`` synchronises the device and waits for
the watchdog passes that drop the completed works, so no listed event exists while a capture is
open; it runs once per outermost ``capture_guard`` when an NCCL process group exists.
"""
from __future__ import annotations

import contextlib
import gc
import threading
import time

_lock = threading.Lock()
_active = 0
_was_enabled = True
# watchdog period of ProcessGroupNCCL (kWatchdogThreadSleepMillis = 100 ms) x 3
_DRAIN_S = 0.3


def _nccl_group_exists() -> bool:
    try:
        import torch.distributed as dist
        if not (dist.is_available() and dist.is_initialized()):
            return False
        from torch.distributed import distributed_c10d as c10d
        return any(str(v[0]).lower() == "nccl" for v in c10d._world.pg_map.values())
    except Exception:
        return False


def drain_collective_watchdog(force: bool = False) -> bool:
    """Let ProcessGroupNCCL's watchdog retire every completed eager collective before a capture
    starts (module docstring). Returns whether it waited."""
    if not (force or _nccl_group_exists()):
        return False
    import torch
    torch.cuda.synchronize()
    time.sleep(_DRAIN_S)
    return True


@contextlib.contextmanager
def capture_guard():
    global _active, _was_enabled
    with _lock:
        if _active == 0:
            drain_collective_watchdog()
            _was_enabled = gc.isenabled()
            gc.collect()
            gc.disable()
        _active += 1
    try:
        yield
    finally:
        with _lock:
            _active -= 1
            if _active == 0 and _was_enabled:
                gc.enable()
