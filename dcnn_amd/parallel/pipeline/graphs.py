"""Per-micro-batch hipGraphs of a pipeline stage (forward and backward).

Reference: a stage runs every FORWARD_JOB / BACKWARD_JOB by walking its layers
(include/pipeline/pipeline_stage.hpp:95-197), one kernel launch per layer op. Here a GPU stage
runs its first training step eagerly (lazy allocations, per-layer profiling for the load
balancer) and from the second step on replays one captured graph per (micro-batch, direction):

* capture happens the first time a micro-batch id is seen in graph mode; the capture itself
  executes nothing, so the replay right after it is the micro-batch's one real execution —
  no warm-up runs, nothing to roll back;
* graphs are captured on a per-stage *capture stream* that never executes anything, and
  replayed on the stage's compute stream (``capture_error_mode="thread_local"``: the other
  stage threads keep launching on their streams while one thread captures). HIP rejects a wait
  on an event whose stream is capturing at the time of the wait, so the compute stream — the
  one other stages wait on through the transport's events — must never be the capturing one;
* every graph gets its own private memory pool. Tensors that outlive a graph (the static
  input/output slots and the forward's per-layer caches that the matching backward reads) can
  then never share memory with another graph's scratch, whatever order a schedule replays the
  graphs in (semi-async interleaves forwards and backwards differently from step to step); the
  cache tensors are also pinned in the forward's record;
* a backward graph is used only for a micro-batch whose last forward was a graph replay (its
  caches then live at the addresses the backward graph was captured against).
"""
from __future__ import annotations

import threading
from typing import Dict, List, Optional, Tuple

import torch

from ...runtime.capture import capture_guard

from ...nn.sequential import Sequential, _all_layers

_CAPTURE_LOCK = threading.Lock()  # one capture per process at a time


def _collect(v, out: List[torch.Tensor]) -> None:
    if isinstance(v, torch.Tensor):
        out.append(v)
    elif isinstance(v, (list, tuple)):
        for e in v:
            _collect(e, out)
    elif isinstance(v, dict):
        for e in v.values():
            _collect(e, out)
    elif v is not None and hasattr(v, "__dict__") and not isinstance(v, type):
        for e in vars(v).values():
            if isinstance(e, (torch.Tensor, list, tuple, dict)):
                _collect(e, out)


class _Record:
    __slots__ = ("graph", "static_in", "out", "keep")

    def __init__(self, graph, static_in, out, keep):
        self.graph, self.static_in, self.out, self.keep = graph, static_in, out, keep


def _key(mb: int, t: torch.Tensor) -> Tuple:
    return (int(mb), tuple(t.shape), t.dtype, tuple(t.stride()))


class StageGraphs:
    """Captured forward/backward graphs of one stage's model, keyed by micro-batch id + input layout."""

    def __init__(self, model: Sequential, stream: torch.cuda.Stream):
        self.model = model
        self.stream = stream
        self.capture_stream = torch.cuda.Stream(device=stream.device)
        self.fwd: Dict[Tuple, _Record] = {}
        self.bwd: Dict[Tuple, _Record] = {}
        self.graph_fwd_mbs = set()  # micro-batches whose most recent forward was a replay
        self.captures = 0
        self.replays = 0

    def reset(self) -> None:
        self.fwd.clear()
        self.bwd.clear()
        self.graph_fwd_mbs.clear()

    def _capture(self, fn, static_in):
        g = torch.cuda.CUDAGraph()
        m = self.model
        prof = m.enable_profiling_
        m.enable_profiling_ = False  # per-layer timing events are not capturable
        try:
            with _CAPTURE_LOCK, capture_guard(), torch.cuda.stream(self.capture_stream):
                g.capture_begin(capture_error_mode="thread_local")
                try:
                    out = fn(static_in)
                finally:
                    g.capture_end()
        finally:
            m.enable_profiling_ = prof
        self.captures += 1
        return g, out

    @staticmethod
    def _slot_like(t: torch.Tensor) -> torch.Tensor:
        return torch.empty_strided(t.shape, t.stride(), dtype=t.dtype, device=t.device)

    def forward(self, x: torch.Tensor, mb: int) -> torch.Tensor:
        key = _key(mb, x)
        rec = self.fwd.get(key)
        if rec is None:
            static_in = self._slot_like(x)
            g, out = self._capture(lambda t: self.model.forward(t, mb, return_on_input_device=False), static_in)
            keep: List[torch.Tensor] = []
            for l in _all_layers(self.model.layers):
                _collect(l._cache.get(mb), keep)
            rec = self.fwd[key] = _Record(g, static_in, out, keep)
        rec.static_in.copy_(x, non_blocking=True)
        rec.graph.replay()
        self.replays += 1
        self.graph_fwd_mbs.add(int(mb))
        return rec.out

    def can_backward(self, mb: int) -> bool:
        return int(mb) in self.graph_fwd_mbs

    def backward(self, g: torch.Tensor, mb: int) -> Optional[torch.Tensor]:
        key = _key(mb, g)
        rec = self.bwd.get(key)
        if rec is None:
            static_in = self._slot_like(g)
            gr, out = self._capture(lambda t: self.model.backward(t, mb, return_on_input_device=False), static_in)
            rec = self.bwd[key] = _Record(gr, static_in, out, [])
        rec.static_in.copy_(g, non_blocking=True)
        rec.graph.replay()
        self.replays += 1
        self.graph_fwd_mbs.discard(int(mb))
        return rec.out

    def forget_forward(self, mb: int) -> None:
        """An eager forward of ``mb`` replaced the graph's caches for it (eval / shape change)."""
        self.graph_fwd_mbs.discard(int(mb))
