"""Graph-capture hygiene shared by every hipGraph capture site.

A capture must not interleave with HIP object teardown: Python's cyclic garbage collector runs
finalizers on whichever thread crosses its allocation threshold, and a finalizer that destroys
a HIP event, stream or graph (an abandoned pipeline stage, a tensor exported from the native
pool) while another thread — or the capturing thread itself — is inside a stream capture can
invalidate that capture and abort the process. ``capture_guard`` keeps the collector off while
any capture is in progress anywhere in the process (counted, so overlapping captures on stage
threads compose) and runs one collection before the first capture starts, at a point where no
capture is active yet.
"""
from __future__ import annotations

import contextlib
import gc
import threading

_lock = threading.Lock()
_active = 0
_was_enabled = True

@contextlib.contextmanager
def capture_guard():
    global _active, _was_enabled
    with _lock:
        if _active == 0:
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
