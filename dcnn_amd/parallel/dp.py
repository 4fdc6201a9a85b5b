"""Data parallelism over RCCL (new in this framework — the reference has no DP).

One process per GPU (`torch.distributed`, backend "nccl" = RCCL on ROCm, "gloo" on CPU).
Gradients live in the model's flat fp32 arena; they are all-reduced in *buckets* that are
contiguous slices of that buffer, launched asynchronously from inside the backward pass as
soon as the layers covering a bucket have finished (last layers first), so RCCL traffic over
xGMI overlaps the remaining backward compute. Buckets default to ~4 MB (built from the last
layer backwards, so ResNet-18-tiny gets 19 / 15 / 4.7 / 4.9 / 1.5 MB buckets): the only
all-reduce that cannot overlap compute is the trailing one after the stem's backward, so it
should be small, while every bucket stays large enough to run near per-link xGMI bandwidth.

The 1/world factor of the gradient average is folded into the loss gradient (every gradient is
linear in it) — the fused loss kernel multiplies it in (``grad_scale``) — so the all-reduce is a
plain SUM and neither the gradient buffer nor the loss gradient needs an extra pass.

``grad_dtype="bf16"`` halves the wire bytes: a bucket is packed to bf16 (``comm.hip``), its
shards are reduce-scattered (RCCL sums bf16 shards hop by hop in a fixed ring order) and
all-gathered, and the result is expanded back into the fp32 arena. On the GPU that pipeline
runs on a side stream forked from the compute stream at the bucket's fire point, so backward
compute keeps running while it waits on RCCL. Over gloo (CPU) the shards are exchanged with
``all_to_all`` and each rank sums the world copies of its shard in fp32 in rank order.

Every collective is issued from the stream it depends on, with no host synchronisation, so the
whole step — forward, backward, bucket collectives and optimizer — can be captured as ONE
hipGraph (``runtime/step.py``): RCCL kernels are stream-capturable, and the NCCL process
group forks its internal stream from the capturing stream and joins it back on ``wait()``.
"""
from __future__ import annotations

from typing import List, Optional, Tuple

import torch
import torch.distributed as dist

from ..nn.layers.base import run_backward
from ..nn.sequential import Sequential, _leaf_param_layers


def init_distributed(backend: Optional[str] = None) -> Tuple[int, int, int]:
    """Initialise the default process group from torchrun env vars. Returns (rank, world, local_rank)."""
    import os
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and not dist.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group(backend, device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    return rank, world, local


class DataParallel:
    def __init__(self, model: Sequential, process_group=None, bucket_mb: float = 4.0, broadcast: bool = True,
                 grad_dtype: str = "fp32", comm_backend: Optional[str] = None):
        if not model.initialized:
            model.initialize()
        self.model = model
        self.pg = process_group
        # gradient data plane: "rccl" = the framework's own RCCL communicator (parallel/rccl.py):
        # rank / world from the launcher's environment, the unique id over the native TCP control
        # plane (no torch.distributed at all), bucket all-reduces on a framework comm stream forked
        # from / joined to the compute stream with events (captured in the step graph); "torch" =
        # torch.distributed (ProcessGroupNCCL = RCCL on ROCm, gloo on CPU). Default: "torch" for
        # world size > 1 (the in-tree plane is opt-in there until a multi-GPU run of it is on
        # record); "rccl" for a single GPU process without torch.distributed (forced world-1
        # collectives, tests).
        import os
        from .rccl import env_rank_world
        want = comm_backend or os.environ.get("DCNN_DP_BACKEND")
        if want is None:
            single = env_rank_world()[1] <= 1
            want = "rccl" if (single and not dist.is_initialized() and model.arena.grad.is_cuda) else "torch"
        if want not in ("torch", "rccl"):
            raise ValueError("comm_backend must be 'torch' or 'rccl'")
        if want == "rccl" and not model.arena.grad.is_cuda:
            want = "torch"  # (the in-tree plane is GPU-only)
        self.comm_backend = want
        self.force_collectives = os.environ.get("DCNN_DP_FORCE_COLLECTIVES", "0") == "1"
        if dist.is_initialized():
            self.world = dist.get_world_size(process_group)
            self.rank = dist.get_rank(process_group)
        elif want == "rccl":
            self.rank, self.world, _ = env_rank_world()
        else:
            self.rank, self.world = 0, 1
        # bucketed all-reduce runs whenever there is more than one replica, or a process group
        # exists / collectives are forced at world size 1 (exercises the RCCL + graph path on one
        # GPU); plain single-process training skips it
        self.active = dist.is_initialized() or self.world > 1 or (want == "rccl" and self.force_collectives)
        self.rccl = None
        if want == "rccl" and self.active:
            from .rccl import RcclCommunicator
            self.rccl = RcclCommunicator(self.rank, self.world, model.arena.grad.device)
        self.bucket_bytes = int(bucket_mb * 2**20)
        if grad_dtype not in ("fp32", "bf16"):
            raise ValueError("grad_dtype must be 'fp32' or 'bf16'")
        self.grad_dtype = grad_dtype
        # at world size 1 a SUM all-reduce is the identity: skip the RCCL launches (the --pg
        # bench and single-GPU runs pay nothing for the group). DCNN_DP_FORCE_COLLECTIVES=1 keeps
        # them, so a one-GPU box can still exercise RCCL capture / replay (tests/test_gpu_dp.py).
        self._works: List = []
        self._wire = {}          # (lo, hi) -> persistent bf16 wire buffers of that bucket
        self._comm_stream = None
        self._build_buckets()
        if broadcast and self.world > 1:
            self.broadcast_parameters()

    # ---------------------------------------------------------------- setup
    def _layer_ranges(self):
        arena = self.model.arena
        ranges = []
        k = 0
        for l in self.model.layers:
            n = sum(len(x.param_specs()) for x in _leaf_param_layers([l]))
            if n == 0:
                ranges.append(None)
            else:
                lo = arena.offsets[k]
                last = k + n - 1
                s = arena.specs[last]
                numel = 1
                for d in s.shape:
                    numel *= d
                hi = arena.offsets[last] + numel
                ranges.append((lo, hi))
            k += n
        return ranges

    def _build_buckets(self):
        ranges = self._layer_ranges()
        numel = self.model.arena.numel
        # fire[i] = (lo, hi) slice to all-reduce right after top-level layer i's backward
        self.fire = {}
        cur_hi = numel
        acc = 0
        lo_layer = None
        for i in range(len(ranges) - 1, -1, -1):
            r = ranges[i]
            if r is None:
                continue
            acc += (cur_hi - r[0]) * 4 if lo_layer is None else 0
            lo_layer = i
            size = (cur_hi - r[0]) * 4
            if size >= self.bucket_bytes:
                self.fire[i] = (r[0], cur_hi)
                cur_hi = r[0]
                lo_layer = None
        first = next((i for i, r in enumerate(ranges) if r is not None), None)
        if first is not None and cur_hi > 0:
            # remaining prefix (including arena padding before the first param) fires last
            self.fire[first] = (0, cur_hi)
        self.buckets = sorted(self.fire.values())

    def broadcast_parameters(self):
        if self.rccl is not None:
            self.rccl.broadcast(self.model.arena.data, 0)
            for l in self.model.layers:
                for t in _bn_buffers(l):
                    self.rccl.broadcast(t, 0)
            self.model.arena.sync_shadow(force=True)
            return
        dist.broadcast(self.model.arena.data, 0, group=self.pg)
        for l in self.model.layers:
            for t in _bn_buffers(l):
                dist.broadcast(t, 0, group=self.pg)
        self.model.arena.sync_shadow(force=True)

    # ---------------------------------------------------------------- compute
    def forward(self, x, mb_id: int = 0):
        return self.model.forward(x, mb_id, return_on_input_device=False)

    __call__ = forward

    @property
    def grad_scale(self) -> float:
        """Factor the loss gradient carries (``Loss.loss_and_grad(grad_scale=...)``): 1 / world."""
        return 1.0 / self.world if self.world > 1 else 1.0

    def backward(self, grad, mb_id: int = 0, sync: bool = True, prescaled: bool = False):
        """Backward + bucketed SUM all-reduce. ``prescaled``: ``grad`` already carries the 1 / world
        average (the fused loss kernel applied ``grad_scale``), else it is scaled here."""
        if self.world > 1 and not prescaled:
            grad = grad * (1.0 / self.world)
        m = self.model
        cur = grad
        flat = m.arena.grad
        m.prepare_backward()
        for i in range(len(m.layers) - 1, -1, -1):
            t0 = m._prof_begin()
            cur = run_backward(m.layers, i, cur, mb_id)
            m._prof_end(m.layers[i].name or m.layers[i].type(), t0, m.backward_times_us)
            if self.active and i in self.fire:
                m.flush_gradients()  # queued split-K reductions of this bucket's layers
                self.reduce_bucket(*self.fire[i])
        m.finish_backward()
        if sync:
            self.finish()
        return cur

    # ---------------------------------------------------------------- bucket collectives
    def reduce_bucket(self, lo: int, hi: int) -> None:
        """Start the SUM all-reduce of ``arena.grad[lo:hi]`` (completed by :meth:`finish`)."""
        if self.world == 1 and not self.force_collectives:
            return
        flat = self.model.arena.grad
        # (a forced world-1 run keeps the bf16 wire pipeline too, so one GPU exercises it)
        plain = self.grad_dtype == "fp32" or (self.world == 1 and not self.force_collectives)
        if self.rccl is not None:
            if plain:
                # on the comm stream: forked after the bucket's last gradient kernel, joined in
                # finish(); the remaining backward keeps the compute stream busy meanwhile
                cs = self._cstream(flat.device)
                with cs.fork():
                    self.rccl.all_reduce(flat[lo:hi])
                return
            self._reduce_bf16_gpu(lo, hi)
            return
        if plain:
            if flat.is_cuda:
                # blocking-form collective on the comm stream (forked after the bucket's gradients,
                # joined in finish()): it overlaps the rest of the backward like an async work, but
                # no Work handle is queued for ProcessGroupNCCL's watchdog. An async_op=True work
                # issued under hipGraph capture is queued although its end event was recorded in
                # the capture; the watchdog's query of that event fails (hipErrorCapturedEvent) and
                # aborts the rank (tools/pg_capture_probe.py --mode async, profiles/pg_capture_probe_r6.md)
                with self._cstream(flat.device).fork():
                    dist.all_reduce(flat[lo:hi], op=dist.ReduceOp.SUM, group=self.pg)
            else:
                self._works.append(dist.all_reduce(flat[lo:hi], op=dist.ReduceOp.SUM, group=self.pg, async_op=True))
            return
        if flat.is_cuda:
            self._reduce_bf16_gpu(lo, hi)
        else:
            self._reduce_bf16_cpu(lo, hi)

    def _wire_bufs(self, lo, hi, device):
        key = (lo, hi)
        b = self._wire.get(key)
        if b is None:
            n = hi - lo
            w = self.world
            shard = -(-n // (w * 64)) * 64   # 64-element shards keep every chunk 128-byte aligned
            z = lambda k: torch.zeros(k, dtype=torch.bfloat16, device=device)
            b = self._wire[key] = (n, shard, z(w * shard), z(w * shard), z(shard), z(w * shard))
        return b

    def _reduce_bf16_gpu(self, lo, hi):
        """bf16 wire on the GPU: pack -> reduce-scatter (RCCL sums the bf16 shards, fp32 inside
        each hop, a fixed ring order) -> all-gather -> unpack, on the comm stream. Collectives
        only (no grouped point-to-point calls, whose rank-to-self form crashed hipGraph capture
        in ncclGroupEnd at world size 1), so the whole pipeline is captured in the step graph."""
        from ..ops._ext import kernels, stream_ptr
        K = kernels()
        flat = self.model.arena.grad
        n, shard, packed, _, red, gathered = self._wire_bufs(lo, hi, flat.device)
        with self._cstream(flat.device).fork():  # the bucket's gradients are complete on the compute stream
            st = stream_ptr(flat.device)
            K.grad_pack_bf16(flat[lo:hi].data_ptr(), packed.data_ptr(), n, 1.0, st)
            if self.rccl is not None:
                self.rccl.reduce_scatter(red, packed)
                self.rccl.all_gather(gathered, red)
            else:
                # (blocking forms: no async Work for the watchdog, see reduce_bucket)
                dist.reduce_scatter_tensor(red, packed, op=dist.ReduceOp.SUM, group=self.pg)
                dist.all_gather_into_tensor(gathered, red, group=self.pg)
            K.grad_unpack_bf16(gathered.data_ptr(), flat[lo:hi].data_ptr(), n, st)

    def _reduce_bf16_cpu(self, lo, hi):
        """Same wire format over gloo (bf16 payloads moved as int32 bit-pattern pairs)."""
        flat = self.model.arena.grad
        n, shard, packed, recv, red, gathered = self._wire_bufs(lo, hi, flat.device)
        packed[:n].copy_(flat[lo:hi].to(torch.bfloat16))
        dist.all_to_all_single(recv.view(torch.int32), packed.view(torch.int32), group=self.pg)
        acc = torch.zeros(shard, dtype=torch.float32)
        for r in range(self.world):   # fixed rank order, fp32 accumulation
            acc += recv[r * shard:(r + 1) * shard].float()
        red.copy_(acc.to(torch.bfloat16))
        dist.all_gather_into_tensor(gathered.view(torch.int32), red.view(torch.int32), group=self.pg)
        flat[lo:hi].copy_(gathered[:n].float())

    def _cstream(self, device):
        if self._comm_stream is None:
            from .rccl import CommStream
            self._comm_stream = CommStream(device)
        return self._comm_stream

    def finish(self):
        for w in self._works:
            w.wait()
        self._works.clear()
        if self._comm_stream is not None:
            self._comm_stream.join()  # the compute stream (optimizer) waits for every bucket

    # ---------------------------------------------------------------- host-side sync (bench / timing)
    def barrier(self) -> None:
        if self.rccl is not None and self.world > 1:
            self.rccl.barrier()
        elif dist.is_initialized():
            dist.barrier(group=self.pg)

    def max_over_ranks(self, v: float) -> float:
        if self.world <= 1:
            return float(v)
        if self.rccl is not None:
            return self.rccl.reduce_scalar(v, "max")
        t = torch.tensor([float(v)], dtype=torch.float64,
                         device=self.model.arena.grad.device if dist.get_backend(self.pg) == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.pg)
        return float(t.item())

    def allreduce_gradients(self):
        """Non-overlapped fallback: one SUM all-reduce per bucket after backward."""
        if self.world > 1:
            for lo, hi in self.buckets:
                self.reduce_bucket(lo, hi)
            self.finish()

    def sync_batchnorm_buffers(self):
        """Average BN running statistics across replicas (before eval / checkpoint)."""
        if self.world <= 1:
            return
        for l in self.model.layers:
            for t in _bn_buffers(l):
                if self.rccl is not None:
                    self.rccl.all_reduce(t)
                else:
                    dist.all_reduce(t, group=self.pg)
                t.div_(self.world)


def _bn_buffers(layer):
    from ..nn.layers import BatchNorm, ResidualBlock
    if isinstance(layer, BatchNorm):
        return [layer.running_mean, layer.running_var]
    if isinstance(layer, ResidualBlock):
        out = []
        for s in layer.sublayers():
            out += _bn_buffers(s)
        return out
    return []
