"""One training step, optionally captured as hipGraphs.

Instead of a tracing compiler the whole per-step launch sequence (input layout conversion,
~150 HIP kernels of forward/backward, fused loss, fused optimizer) is captured once with
``torch.cuda.graph`` and replayed, removing host launch overhead.

Data-parallel steps are captured WHOLE: the bucket collectives that
:class:`~dcnn_amd.parallel.dp.DataParallel` fires from inside the backward pass are RCCL
kernels on the framework's comm stream (or the process group's internal stream), forked from the
capturing stream at each fire point and joined back before the optimizer, so one replay runs forward, backward, every
overlapped all-reduce and the update with no host involvement. ``DCNN_DP_CAPTURE=0`` selects
the older *segmented* capture instead: one graph per backward segment between fire points, the
host enqueuing each bucket's asynchronous all-reduce between two segment replays.
The optimizer's step scalars are uploaded to device memory before each replay
(``Optimizer.prepare_step``), so replays use the current learning rate / bias corrections.
"""
from __future__ import annotations

import os
from typing import List, Optional

import torch

from .capture import capture_guard
import torch.distributed as dist


class TrainStep:
    def __init__(self, dp, loss_fn, optimizer, use_graph: bool = False):
        from ..parallel.dp import DataParallel
        if not isinstance(dp, DataParallel):
            dp = DataParallel(dp, broadcast=False)
        self.dp = dp
        self.model = dp.model
        self.loss_fn = loss_fn
        self.opt = optimizer
        self.use_graph = use_graph
        self.graphs: Optional[List[torch.cuda.CUDAGraph]] = None
        self.capture_collectives = os.environ.get("DCNN_DP_CAPTURE", "1") != "0"
        self._whole = False
        self._cap_stream = None
        self.last_loss = None
        self.last_correct = None
        self._static_x = self._static_y = None
        # native per-step activation arena (runtime/arena.py): every activation / slab /
        # workspace of a step on the GPU; the captured graphs pin the chunks they address
        from . import arena as _arena
        dev = self.model.device
        self.arena = (_arena.ActivationArena(dev.index) if _arena.enabled() and dev.is_gpu() else None)
        self._pins = None

    def _arena_step(self, capture=False):
        import contextlib
        return self.arena.step(capture=capture) if self.arena is not None else contextlib.nullcontext()

    def _loss_grad(self, out, y):
        """Loss, gradient already carrying the data-parallel 1 / world factor, correct count. A
        user loss without ``grad_scale`` support gets the factor applied to its gradient instead."""
        sc = self.dp.grad_scale
        if sc == 1.0:
            return self.loss_fn.loss_and_grad(out, y)
        try:
            return self.loss_fn.loss_and_grad(out, y, grad_scale=sc)
        except TypeError:
            loss, grad, correct = self.loss_fn.loss_and_grad(out, y)
            return loss, grad * sc, correct

    # ------------------------------------------------------------------ eager
    def eager(self, x, y):
        with self._arena_step():
            self.opt.clear_gradients()
            out = self.dp.forward(x)
            loss, grad, correct = self._loss_grad(out, y)
            self.dp.backward(grad, prescaled=True)
            self.opt.update()
        self.last_loss, self.last_correct = loss, correct
        return loss

    # ------------------------------------------------------------------ graph
    def _segments(self):
        """Backward layer ranges [hi..lo] ending at each bucket fire point (descending)."""
        L = len(self.model.layers)
        fires = sorted(self.dp.fire.keys(), reverse=True) if self.dp.active else []
        segs = []
        hi = L - 1
        for f in fires:
            segs.append((hi, f))
            hi = f - 1
        if hi >= 0:
            segs.append((hi, 0))
        return segs, fires

    def _run_bwd(self, cur, hi, lo):
        from ..nn.layers.base import run_backward
        layers = self.model.layers
        for i in range(hi, lo - 1, -1):
            cur = run_backward(layers, i, cur, 0)
        return cur

    def _training_state(self):
        """Tensors a step mutates: fp32 master weights, optimizer moments, BN running stats."""
        from ..parallel.dp import _bn_buffers
        ts = [self.model.arena.data]
        for name in ("m", "v", "velocity"):
            ts += list(getattr(self.opt, name, None) or [])
        for l in self.model.layers:
            ts += _bn_buffers(l)
        return ts

    def _capture_stream(self):
        """The stream graphs are captured on, with its per-stream ticket words created eagerly."""
        if self._cap_stream is None:
            from ..ops import hip
            self._cap_stream = torch.cuda.Stream(device=self.model.device.torch_device)
            self._cap_stream.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(self._cap_stream):
                hip.prewarm_tickets(self.model.device.torch_device)
            torch.cuda.current_stream().wait_stream(self._cap_stream)
        return self._cap_stream

    def _capture(self, x, y):
        self._static_x = x.clone()
        self._static_y = y.clone()
        # the warm-up steps below must not train: snapshot the state and restore it afterwards,
        # so the first replay is the first update (as in eager mode)
        state = self._training_state()
        saved = [t.detach().clone() for t in state]
        saved_t = getattr(self.opt, "t", None)
        # warm up on a side stream (allocator pools, lazy init) as torch.cuda.graph requires
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(2):
                self.eager(self._static_x, self._static_y)
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        with torch.no_grad():
            for t, c in zip(state, saved):
                t.copy_(c)
        del saved
        if saved_t is not None:
            self.opt.t = saved_t
        self.opt._hyper_dirty = True  # device step scalars re-synced from the restored host state
        self.model.arena.sync_shadow(force=True)
        torch.cuda.synchronize()
        fused_opt = hasattr(self.opt, "fused") and self.opt.fused()
        if not fused_opt:
            raise RuntimeError("graph capture needs the fused flat-buffer optimizer on the GPU")
        torch_bf16 = self.dp.rccl is None and self.dp.grad_dtype == "bf16"
        if self.dp.active and self.capture_collectives and not torch_bf16 and (
                self.dp.rccl is not None or dist.get_backend(self.dp.pg) == "nccl"):
            # (gloo moves CUDA tensors through the host: not capturable, keeps the segments; the
            # bf16 wire on ProcessGroupNCCL keeps them too: its reduce-scatter / all-gather pair
            # issued from the forked comm stream crashed hipGraph capture (SIGSEGV) at world size
            # 1, while the same pair on the in-tree communicator captures and replays correctly,
            # tests/test_gpu_dp.py::test_gpu_dp_bf16_wire_captured_world1)
            t0 = getattr(self.opt, "t", None)
            err = None
            try:
                self._capture_whole()
            except Exception as e:  # e.g. a collective library build without capture support
                err = e
            # every rank must replay the same kind of step (a whole-graph rank and a segmented
            # rank would issue different collective sequences and hang): agree before the first
            # replay, falling back everywhere if any rank's capture failed
            if self.dp.world > 1:
                flag = torch.tensor([0 if err is not None else 1], dtype=torch.int32,
                                    device=self.model.device.torch_device)
                if self.dp.rccl is not None:
                    self.dp.rccl.all_reduce(flag, "min")
                else:
                    dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=self.dp.pg)
                if int(flag.item()) == 0 and err is None:
                    err = RuntimeError("another rank's capture failed")
            if err is None:
                return
            import warnings
            warnings.warn(f"capturing the bucket collectives into the step graph failed ({err}); "
                          "falling back to the segmented capture")
            self.dp._works.clear()
            if self.dp._comm_stream is not None:
                self.dp._comm_stream.forked = False
            if t0 is not None:
                self.opt.t = t0
            self.graphs, self._whole = None, False
            torch.cuda.synchronize()
        segs, fires = self._segments()
        self._segs, self._fires = segs, fires
        # thread_local capture (as the whole-step graph): ProcessGroupNCCL's watchdog thread queries
        # eager collectives' events while a segment is being captured; in the global mode that
        # query invalidates the capture ("operation not permitted when stream is capturing")
        self.graphs = []
        pool = None
        self.opt.prepare_step()  # upload scalars used during capture (replays re-upload)
        if hasattr(self.opt, "t"):
            self.opt.t -= 1  # the capture itself is not a training step
        active = self.dp.active
        arena_scope = self._arena_step(capture=True)
        arena_scope.__enter__()  # one arena step across the segments (segment k+1 reads k's carry)
        try:
            for k, (hi, lo) in enumerate(segs):
                g = torch.cuda.CUDAGraph()
                with capture_guard(), torch.cuda.graph(g, pool=pool, stream=self._capture_stream(),
                                                       capture_error_mode="thread_local"):
                    if k == 0:
                        self.opt.clear_gradients()
                        out = self.dp.forward(self._static_x)
                        loss, cur, correct = self._loss_grad(out, self._static_y)
                        self._g_loss, self._g_correct = loss, correct
                        self.model.prepare_backward()
                    else:
                        cur = self._carry
                    cur = self._run_bwd(cur, hi, lo)
                    self.model.flush_gradients()  # the bucket all-reduced after this segment is complete
                    self._carry = cur
                    if k == len(segs) - 1:
                        self.model.finish_backward()
                    if not active and k == len(segs) - 1:
                        self.opt.launch_step()
                if pool is None:
                    pool = g.pool()
                self.graphs.append(g)
            if active:
                g = torch.cuda.CUDAGraph()
                with capture_guard(), torch.cuda.graph(g, pool=pool, stream=self._capture_stream(),
                                                       capture_error_mode="thread_local"):
                    self.opt.launch_step()
                self.graphs.append(g)
        finally:
            arena_scope.__exit__(None, None, None)
        self._pins = self.arena.pin() if self.arena is not None else None
        torch.cuda.synchronize()

    def _capture_whole(self):
        """ONE graph: forward, loss, backward with the bucket collectives it fires, optimizer."""
        self.opt.prepare_step()
        if hasattr(self.opt, "t"):
            self.opt.t -= 1
        m = self.model
        prof = m.enable_profiling_
        m.enable_profiling_ = False
        g = torch.cuda.CUDAGraph()
        try:
            with self._arena_step(capture=True), capture_guard(), \
                    torch.cuda.graph(g, stream=self._capture_stream(), capture_error_mode="thread_local"):
                self.opt.clear_gradients()
                out = self.dp.forward(self._static_x)
                loss, grad, correct = self._loss_grad(out, self._static_y)
                self._g_loss, self._g_correct = loss, correct
                self.dp.backward(grad, sync=True, prescaled=True)
                self.opt.launch_step()
        finally:
            m.enable_profiling_ = prof
        self._pins = self.arena.pin() if self.arena is not None else None
        self.graphs = [g]
        self._whole = True
        torch.cuda.synchronize()

    def replay(self, x, y):
        self._static_x.copy_(x, non_blocking=True)
        self._static_y.copy_(y, non_blocking=True)
        self.opt.prepare_step()
        if self._whole:
            self.graphs[0].replay()
            self.last_loss, self.last_correct = self._g_loss, self._g_correct
            return self.last_loss
        active = self.dp.active
        for k, (hi, lo) in enumerate(self._segs):
            self.graphs[k].replay()
            if active and k < len(self._fires):
                # the same bucket collective as the eager / whole-graph steps (fp32 SUM, or the
                # bf16 wire pipeline when DataParallel(grad_dtype="bf16"))
                self.dp.reduce_bucket(*self.dp.fire[self._fires[k]])
        if active:
            self.dp.finish()
            self.graphs[-1].replay()
        self.last_loss, self.last_correct = self._g_loss, self._g_correct
        return self.last_loss

    def __call__(self, x, y):
        if not self.use_graph:
            return self.eager(x, y)
        if self.graphs is None:
            self._capture(x, y)
        return self.replay(x, y)
