"""Shared plumbing of the HIP front end (ops/hip.py and its siblings): activation buffers from the
per-step arena, layout conversions, the conv call recorder, the backward-BatchNorm fusion request
and the batched split-K weight-gradient reducer."""
from __future__ import annotations

import os
import threading

import torch

from ..runtime import arena as _arena
from . import fusion
from ._ext import dt_code, kernels, ptr, stream_ptr

CL = torch.channels_last
F32 = torch.float32
BF16 = torch.bfloat16

# backward-BN epilogue fusion operands (api.h BnbArgs): (y, x, mean, istd) pointers, 0 = off
_NOBNB = (0, 0, 0, 0)

# gather modes of gemm_nt
PLAIN, CONV_FWD, CONV_DGRAD = 0, 1, 2

def _empty(shape, dtype, device, cl=False):
    """Per-step buffer (activation, statistics slab, workspace): the native activation arena of
    the running step (runtime/arena.py), else PyTorch's allocator. ``cl``: NHWC strides."""
    return _arena.empty(shape, dtype, device, cl)


def _empty_like(x):
    """Per-step buffer shaped and laid out (dense or channels_last) like x."""
    cl = x.dim() == 4 and not x.is_contiguous() and x.is_contiguous(memory_format=CL)
    return _arena.empty(x.shape, x.dtype, x.device, cl)


def _check_act(x: torch.Tensor, what: str):
    if not x.is_cuda:
        raise ValueError(f"{what}: expected a GPU tensor")
    if x.dim() == 4 and not x.is_contiguous(memory_format=CL):
        raise ValueError(f"{what}: expected channels_last (NHWC) memory layout")


# ---- conv call recorder (tests/test_gpu_geometry.py): every conv2d_fwd / dgrad / wgrad call's
# shapes, epilogue options and routing-table decision, so a test can replay exactly the (kernel,
# shape, epilogue) tuples a model's training step launches against an fp32 reference
_RECORD = None


class record_convs:
    """``with record_convs() as calls:`` appends one dict per conv call made inside the block."""

    def __enter__(self):
        global _RECORD
        self._prev, self.calls = _RECORD, []
        _RECORD = self.calls
        return self.calls

    def __exit__(self, *exc):
        global _RECORD
        _RECORD = self._prev
        return False


def _rec(op, **kw):
    if _RECORD is not None:
        _RECORD.append(dict(op=op, **kw))


def to_act(x: torch.Tensor, dtype: torch.dtype) -> torch.Tensor:
    """Bring a (N,C,H,W) tensor into the GPU activation format: NHWC memory, compute dtype."""
    if x.dim() == 4 and x.dtype == dtype and x.is_contiguous(memory_format=CL):
        return x
    if x.dim() == 4 and x.dtype == F32 and x.is_contiguous():
        # fused NCHW fp32 -> NHWC (bf16|fp32) conversion kernel (network input path)
        N, C, H, W = x.shape
        y = _empty((N, C, H, W), dtype, x.device, True)
        kernels().nchw_to_nhwc(dt_code(dtype), x.data_ptr(), y.data_ptr(), N, C, H * W, stream_ptr())
        return y
    return x.to(dtype=dtype).contiguous(memory_format=CL)


def nchw_nhwc(x: torch.Tensor, to_nhwc: bool) -> torch.Tensor:
    """Physical layout change of a 4-D GPU activation (the NCHW-order Flatten of a spatial map):
    NCHW-contiguous -> channels_last (to_nhwc) or back, one transpose kernel per call (fp32 / bf16)."""
    N, C, H, W = x.shape
    if to_nhwc:
        assert x.is_contiguous()
        y = _empty((N, C, H, W), x.dtype, x.device, True)
        rows, cols = C, H * W
    else:
        assert x.is_contiguous(memory_format=CL)
        y = _empty((N, C, H, W), x.dtype, x.device, False)
        rows, cols = H * W, C
    if x.dtype == F32:
        kernels().transpose_batched(x.data_ptr(), y.data_ptr(), N, rows, cols, stream_ptr())
    else:
        assert x.element_size() == 2
        kernels().transpose_batched16(x.data_ptr(), y.data_ptr(), N, rows, cols, stream_ptr())
    return y


def conv_out_hw(H, W, kh, kw, sh, sw, ph, pw):
    return (H + 2 * ph - kh) // sh + 1, (W + 2 * pw - kw) // sw + 1


def _nbytes(t):
    return t.numel() * t.element_size()



class BnbRequest:
    """Backward-BatchNorm fusion request handed to a gradient producer (api.h ``BnbArgs``).

    ``bn`` is the consuming BatchNorm layer; ``y`` its (ReLU) output used as the mask (None: no
    ReLU was fused), ``x`` its input, ``mean``/``istd`` its saved batch statistics. A producer
    that honours the request returns dy' = dy * (y > 0) with ``dy'._bnb = (bn, slab, rows, sums)``
    attached: per-tile (sum dy', sum dy' * xhat) rows and the zeroed [2][C] sums to reduce into.
    """
    __slots__ = ("bn", "y", "x", "mean", "istd", "pooled")

    def __init__(self, bn, y, x, mean, istd, pooled=False):
        # pooled: the BatchNorm's forward fused ReLU + max-pool (no full-resolution y; only the
        # max-pool backward, masking with the pooled value, can honour the request)
        self.bn, self.y, self.x, self.mean, self.istd, self.pooled = bn, y, x, mean, istd, pooled

    def args(self):
        return (ptr(self.y), self.x.data_ptr(), self.mean.data_ptr(), self.istd.data_ptr())



class _DeferredReduce:
    """Split-K weight-gradient reductions queued during a model backward and launched together
    (``multi_splitk_reduce``: one kernel for the whole queue instead of one per layer, ~26 for
    ResNet-18). The slabs stay referenced until the flush; with 288 GB of HBM per GPU holding
    every layer's slab for one backward (< 2 GB for ResNet-18 at batch 256) is the cheap side of
    the trade. Active between ``begin()`` / ``end()`` (Sequential.prepare_backward /
    finish_backward); gradient consumers inside that window (the data-parallel bucket
    all-reduce) call ``flush()`` first. Outside it every reduction runs immediately."""

    def __init__(self):
        self.active = False
        self.pending = []  # (slab, out, n, splits) — tensors kept alive until the launch
        self.pending_bytes = 0

    def begin(self):
        self.active = fusion.DEFER_REDUCE

    def add(self, slab, out, n, splits):
        self.pending.append((slab, out, int(n), int(splits)))
        self.pending_bytes += int(n) * int(splits) * 4
        # a queue larger than the last-level cache would read its first slabs back from HBM:
        # launch once the pending slabs reach the threshold
        if self.pending_bytes >= _DEFER_REDUCE_BYTES:
            self.flush()

    def flush(self):
        if self.pending and _TRACE_REDUCE:
            import sys
            print(f"[splitk_reduce] {len(self.pending)} slabs, {self.pending_bytes / 2**20:.1f} MiB: "
                  + " ".join(f"{t[2]}x{t[3]}" for t in self.pending), file=sys.stderr)
        if self.pending:
            kernels().multi_splitk_reduce([(t[0].data_ptr(), t[1].data_ptr(), t[2], t[3]) for t in self.pending],
                                          stream_ptr())
            self.pending.clear()
            self.pending_bytes = 0

    def end(self):
        self.flush()
        self.active = False


_TRACE_REDUCE = os.environ.get("DCNN_TRACE_REDUCE", "0") == "1"  # print each batched reduce's slabs
_DEFER_REDUCE_BYTES = 1 << 50  # (one batched reduce per backward)
_tls = threading.local()


class _ThreadReducer:
    """``grad_reducer``: the calling thread's :class:`_DeferredReduce` (a pipeline stage's
    backward on its own thread and stream must not flush another stage's queue)."""

    def _get(self):
        r = getattr(_tls, "reducer", None)
        if r is None:
            r = _tls.reducer = _DeferredReduce()
        return r

    def __getattr__(self, k):
        return getattr(self._get(), k)


grad_reducer = _ThreadReducer()

def _dense(t):
    """A gradient tensor whose storage is exactly its numel() elements (any dim order)."""
    return t.is_contiguous() or t.is_contiguous(memory_format=CL)


def _reduce_wb(K, slab, grad_w, n, bslab, grad_b, nb, splits, st):
    """grad_w += sum over splits of slab, grad_b += sum of bslab — one launch for both (or
    queued on :data:`grad_reducer` inside a model backward)."""
    if grad_reducer.active and _dense(grad_w) and (grad_b is None or grad_b.is_contiguous()):
        grad_reducer.add(slab, grad_w, n, splits)
        if grad_b is not None:
            grad_reducer.add(bslab, grad_b, nb, splits)
        return
    if grad_b is None:
        K.splitk_reduce(slab.data_ptr(), grad_w.data_ptr(), n, splits, 1, st)
    else:
        K.splitk_reduce2(slab.data_ptr(), grad_w.data_ptr(), n, bslab.data_ptr(), grad_b.data_ptr(), nb, splits, 1, st)


def _g2_ok(Cs, N):
    return Cs % 8 == 0 and N % 8 == 0


def pool_out_hw(H, W, ph, pw, sh, sw, pdh, pdw):
    return (H + 2 * pdh - ph) // sh + 1, (W + 2 * pdw - pw) // sw + 1


def _rc(x):
    N, C, H, W = x.shape
    return N * H * W, C


_tickets = {}


def _ticket(device, C, slot="stat"):
    """Per-(stream, device, user) ticket words of the ticketed reductions (bn_stat_reduce, the
    loss): zeroed once, every launch leaves them zeroed again, and launches on one stream never
    overlap."""
    key = (stream_ptr(), device.index, slot)
    t = _tickets.get(key)
    need = (C + 63) // 64
    if t is None or t.numel() < need:
        t = _arena.persistent((max(need, 64),), torch.int32, torch.device(device), zero=True)
        _tickets[key] = t
    return t
