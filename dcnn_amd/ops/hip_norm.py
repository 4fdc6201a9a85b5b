"""BatchNorm / GroupNorm on the HIP kernels: statistics (from conv-epilogue slabs or standalone
partial passes, fixed-order Chan/Welford reduces), the forward apply (+ residual, ReLU, the paired
projection-shortcut apply, the fused ReLU + max-pool), and the backward."""
from __future__ import annotations

import os

import torch

from ..runtime import arena as _arena
from . import fusion
from ._ext import dt_code, kernels, ptr, stream_ptr
from .hip_base import BF16, CL, F32, _empty, _empty_like, _rc, _ticket, pool_out_hw


class Stats:
    """Per-channel statistics for the BN apply kernels: ``parts == 1`` -> ``buf`` is the finished
    [2][C] result; ``parts > 1`` -> ``buf`` holds [parts][3][C] level-1 partials that the
    consuming kernel merges in its prologue (norm.hip read_stats). Used as a tensor (tests,
    inspection) it materialises the finished [2][C] statistics (``final()``, torch ops: off the
    training hot path)."""
    __slots__ = ("buf", "parts", "mode", "_final")

    def __init__(self, buf, parts, mode=0):
        self.buf, self.parts, self.mode, self._final = buf, int(parts), int(mode), None

    def final(self):
        if self.parts == 1:
            return self.buf
        if self._final is None:
            p = self.buf.double()
            C = p.shape[2]
            parts = self.parts
            if self.mode == 0:  # Chan merges in part order (as read_stats)
                n, mean, m2 = p[0, 0].clone(), p[0, 1].clone(), p[0, 2].clone()
                for k in range(1, parts):
                    nb, mb, m2b = p[k, 0], p[k, 1], p[k, 2]
                    tot = n + nb
                    d = mb - mean
                    safe = torch.where(tot > 0, tot, torch.ones_like(tot))
                    mean = torch.where(tot > 0, mean + d * nb / safe, mean)
                    m2 = m2 + m2b + d * d * n * nb / safe
                    n = tot
                var = torch.where(n > 0, m2 / torch.where(n > 0, n, torch.ones_like(n)), torch.zeros_like(n))
                out = torch.cat([mean, var])
            else:
                out = torch.cat([p[:, 0].sum(0), p[:, 1].sum(0)])
            self._final = out.float().reshape(2 * C)
        return self._final

    def __getattr__(self, k):
        return getattr(self.final(), k)

    def __getitem__(self, i):
        return self.final()[i]


def prewarm_tickets(device, slots=("loss",)):
    """Create the calling stream's ticket words now (call it on a graph's capture stream before the
    capture): created during a capture, their zeroing would be re-run by every replay."""
    for s in slots:
        _ticket(torch.device(device), 0, slot=s)


def stat_reduce(mode, slab, rows, C, out):
    """Deterministic slab reduce (norm.hip bn_stat_reduce): mode 0 = Welford (count, mean, M2)
    tile triples -> (mean, biased var); mode 1 = (sum a, sum b) rows -> sums. Returns
    :class:`Stats` (``out`` when one block covered all rows, else the partials buffer).
    (Handing small slabs to the consumers raw instead measured no faster: the consumer prologue's
    merge costs what the launch saves, `profiles/experiment_raw_stats_r4.md`.)"""
    K = kernels()
    ny = K.bn_stat_parts(rows)
    part = _empty((ny, 3, C), F32, slab.device) if ny > 1 else None
    K.bn_stat_reduce(mode, slab.data_ptr(), rows, C, out.data_ptr(), ptr(part), 0, stream_ptr())
    return Stats(part if ny > 1 else out, ny, mode)


def _stats(s):
    """(pointer, parts) of a Stats / plain finished [2][C] tensor / None."""
    if s is None:
        return 0, 1
    if isinstance(s, Stats):
        return s.buf.data_ptr(), s.parts
    return s.data_ptr(), 1


_TRACE_PARTIAL = os.environ.get("DCNN_TRACE_PARTIAL", "0") == "1"
_traced_partial = set()


def _trace_partial(kind, x):
    """DCNN_TRACE_PARTIAL=1: report (once per call site and shape) every standalone BatchNorm
    statistics pass, i.e. a BatchNorm whose producer / consumer kernel could not emit its sums."""
    if not _TRACE_PARTIAL:
        return
    import sys
    import traceback
    fr = [f"{os.path.basename(f.filename)}:{f.lineno}:{f.name}" for f in traceback.extract_stack(limit=8)[:-2]]
    key = (kind, tuple(x.shape), tuple(fr))
    if key not in _traced_partial:
        _traced_partial.add(key)
        print(f"[bn_partial] {kind} {tuple(x.shape)} <- {' <- '.join(reversed(fr))}", file=sys.stderr)


def bn_stats_raw(x, partial=None):
    """The (slab, rows, sums) statistics rows of x before the reduce (the producing conv's
    epilogue slab, else a bn_partial pass)."""
    if partial is not None:
        return partial
    K = kernels()
    R, C = _rc(x)
    rows = K.bn_partial_rows(R, C)
    slab = _empty((rows, 3, C), F32, x.device)
    sums = _empty((2 * C,), F32, x.device)
    _trace_partial("fwd", x)
    K.bn_partial(dt_code(x.dtype), x.data_ptr(), 0, 0, 0, 0, 0, R, C, slab.data_ptr(), 0, 0, stream_ptr())
    return slab, rows, sums


def bn_bwd_stats_raw(dy, x, mean, istd):
    """Backward statistics rows (sum dy, sum dy * xhat) of x before the reduce: (slab, rows, sums)."""
    K = kernels()
    R, C = _rc(x)
    rows = K.bn_partial_rows(R, C)
    slab = _empty((rows, 2, C), F32, x.device)
    sums = _empty((2 * C,), F32, x.device)
    _trace_partial("bwd_raw", x)
    K.bn_partial(dt_code(x.dtype), x.data_ptr(), dy.data_ptr(), 0, 0, mean.data_ptr(), istd.data_ptr(), R, C,
                 slab.data_ptr(), 1, 0, stream_ptr())
    return slab, rows, sums


def bn_bwd_apply_dual(dy, a, b):
    """Data gradients of two training BatchNorms fed the same (masked) gradient ``dy`` in one pass
    (norm.hip bn_bwd_apply_dual); ``a``/``b`` = (layer, its forward cache entry (x, _, mean, istd,
    _), reduced backward :class:`Stats`). Accumulates each layer's dgamma / dbeta."""
    R, C = _rc(dy)
    outs, sides = [], []
    for layer, ent, st in (a, b):
        x, _, mean, istd, _ = ent
        dx = _empty(x.shape, x.dtype, x.device, True)
        sp, parts = _stats(st)
        dg = layer._grads[0].view(-1) if layer.affine else None
        db = layer._grads[1].view(-1) if layer.affine else None
        sides.append((x.data_ptr(), dx.data_ptr(), mean.data_ptr(), istd.data_ptr(), ptr(layer._gamma()), sp, parts,
                      float(R), ptr(dg), ptr(db)))
        outs.append(dx)
    if not kernels().bn_bwd_apply_dual(dy.data_ptr(), sides[0], sides[1], R, C, stream_ptr()):
        raise RuntimeError("bn_bwd_apply_dual: unsupported shape")
    return outs[0], outs[1]


def stat_reduce_pair(mode, a, b, C):
    """Two independent forward/backward statistics reduces of the same C in ONE launch
    (norm.hip bn_stat_reduce2); ``a``/``b`` = (slab, rows, out). Returns two :class:`Stats`."""
    K = kernels()
    res, ptrs = [], []
    for slab, rows, out in (a, b):
        ny = K.bn_stat_parts(rows)
        part = _empty((ny, 3, C), F32, slab.device) if ny > 1 else None
        ptrs.append((slab.data_ptr(), rows, out.data_ptr(), ptr(part)))
        res.append(Stats(part if ny > 1 else out, ny, mode))
    (s1, r1, o1, p1), (s2, r2, o2, p2) = ptrs
    K.bn_stat_reduce2(mode, s1, r1, o1, p1, s2, r2, o2, p2, C, stream_ptr())
    return res[0], res[1]


def bn_stats(x, partial=None):
    """Per-channel (mean, biased variance) of x (NHWC), as one [2][C] fp32 tensor. Uses the
    producing conv's epilogue Welford slab if given, else a bn_partial pass; the reduction is
    deterministic and cancellation-free (Chan merges of pivot-shifted tile statistics)."""
    K = kernels()
    R, C = _rc(x)
    st = stream_ptr()
    if partial is None:
        rows = K.bn_partial_rows(R, C)
        slab = _empty((rows, 3, C), F32, x.device)
        sums = _empty((2 * C,), F32, x.device)
        _trace_partial("fwd", x)
        K.bn_partial(dt_code(x.dtype), x.data_ptr(), 0, 0, 0, 0, 0, R, C, slab.data_ptr(), 0, 0, st)
    else:
        slab, rows, sums = partial
    return stat_reduce(0, slab, rows, C, sums)


def bn_apply(x, sums, count, gamma, beta, eps, *, residual=None, relu=False, save=None, running=None,
             momentum=0.1, use_running=False):
    R, C = _rc(x)
    y = _empty(x.shape, x.dtype, x.device, True)
    sm, si = save if save is not None else (None, None)
    rm, rv = running if running is not None else (None, None)
    sp, parts = _stats(sums)
    kernels().bn_apply(dt_code(x.dtype), x.data_ptr(), y.data_ptr(), R, C, sp, parts, float(count), ptr(gamma),
                       ptr(beta), float(eps), ptr(residual), int(relu), ptr(sm), ptr(si), ptr(rm), ptr(rv),
                       float(momentum), int(use_running), stream_ptr())
    return y


class BnDeferred:
    """A BatchNorm whose apply is deferred into the consumer (a residual block's tail BatchNorm
    applies its projection shortcut's BatchNorm on the fly: :func:`bn_apply_dual`)."""
    __slots__ = ("x", "sums", "count", "gamma", "beta", "eps", "save", "running", "momentum", "use_running")

    def __init__(self, x, sums, count, gamma, beta, eps, save, running, momentum, use_running):
        self.x, self.sums, self.count, self.gamma, self.beta, self.eps = x, sums, count, gamma, beta, eps
        self.save, self.running, self.momentum, self.use_running = save, running, momentum, use_running

    def reduced(self):
        """Reduce raw statistics rows (left raw so a consumer can pair the reduce with its own)."""
        if isinstance(self.sums, tuple):
            slab, rows, out = self.sums
            self.sums = stat_reduce(0, slab, rows, out.numel() // 2, out)
        return self

    def side(self):
        self.reduced()
        sp, parts = _stats(self.sums)
        sm, si = self.save if self.save is not None else (None, None)
        rm, rv = self.running if self.running is not None else (None, None)
        return (self.x.data_ptr(), sp, parts, float(self.count), ptr(self.gamma), ptr(self.beta), float(self.eps),
                ptr(sm), ptr(si), ptr(rm), ptr(rv), float(self.momentum), int(self.use_running))

    def materialize(self):
        """The deferred BatchNorm's output as a tensor (when the consumer cannot fuse it)."""
        self.reduced()
        return bn_apply(self.x, self.sums, self.count, self.gamma, self.beta, self.eps, save=self.save,
                        running=self.running, momentum=self.momentum, use_running=self.use_running)




def bn_dual_ok(x):
    return fusion.BN_DUAL and x.dtype == BF16 and bool(kernels().bn_apply_dual_supported(*_rc(x)))


def bn_apply_dual(x, sums, count, gamma, beta, eps, other: BnDeferred, *, relu=False, save=None, running=None,
                  momentum=0.1, use_running=False):
    """act(bn(x) + other's BatchNorm output) in one pass (norm.hip bn_apply_dual)."""
    R, C = _rc(x)
    assert tuple(other.x.shape) == tuple(x.shape) and other.x.dtype == x.dtype == BF16
    y = _empty(x.shape, x.dtype, x.device, True)
    me = BnDeferred(x, sums, count, gamma, beta, eps, save, running, momentum, use_running)
    if not kernels().bn_apply_dual(me.side(), other.side(), y.data_ptr(), R, C, int(relu), stream_ptr()):
        raise RuntimeError("bn_apply_dual: unsupported shape")
    return y


def bn_relu_maxpool_ok(x, ph, pw, sh, sw, pdh, pdw):
    """Can :func:`bn_relu_maxpool` take this BatchNorm+ReLU+max-pool? Its backward relies on the
    fused max-pool backward (:func:`maxpool_bwd` with ``bnb``), so both must be available."""
    if not fusion.BNB or x.dtype != BF16 or not x.is_contiguous(memory_format=CL):
        return False
    N, C, H, W = x.shape
    OH, OW = pool_out_hw(H, W, ph, pw, sh, sw, pdh, pdw)
    g = (N, H, W, C, OH, OW, ph, pw, sh, sw, pdh, pdw)
    K = kernels()
    return K.bn_relu_maxpool_supported(*g) and K.maxpool_bwd_bnb_supported(*g)


def bn_relu_maxpool(x, sums, count, gamma, beta, eps, pool, *, save, running, momentum=0.1):
    """Training BatchNorm (batch statistics ``sums``) + ReLU + max-pool ``pool`` = (ph, pw, sh, sw,
    pdh, pdw) in one pass: returns the pooled output and the window argmax (max-pool layout)."""
    N, C, H, W = x.shape
    ph, pw, sh, sw, pdh, pdw = pool
    OH, OW = pool_out_hw(H, W, ph, pw, sh, sw, pdh, pdw)
    y = _empty((N, C, OH, OW), BF16, x.device, True)
    idx = _empty((N, OH, OW, C), torch.uint8, x.device)
    sm, si = save
    rm, rv = running
    sp, parts = _stats(sums)
    kernels().bn_relu_maxpool(x.data_ptr(), y.data_ptr(), idx.data_ptr(), N, H, W, C, OH, OW, ph, pw, sh, sw, pdh, pdw,
                              sp, parts, float(count), ptr(gamma), ptr(beta), float(eps), sm.data_ptr(),
                              si.data_ptr(), ptr(rm), ptr(rv), float(momentum), stream_ptr())
    return y, idx


def bn_backward(dy, x, yout, mean, istd, gamma, dgamma, dbeta, *, want_masked=False, eval_mode=False, fused=None):
    """Returns (dx, masked_dy|None). yout given => ReLU was fused: dy' = dy * (yout > 0).

    ``fused`` = (slab, rows, sums) when the producer of ``dy`` already applied the ReLU mask and
    wrote the backward statistics in its epilogue (:class:`BnbRequest`): only the slab reduce
    and the apply pass remain.
    """
    K = kernels()
    R, C = _rc(x)
    st = stream_ptr()
    dt = dt_code(x.dtype)
    if fused is not None and not eval_mode:
        slab, rows, sums = fused
        sp, parts = _stats(stat_reduce(1, slab, rows, C, sums))
        dx = _empty(x.shape, x.dtype, x.device, True)
        K.bn_bwd_apply(dt, dy.data_ptr(), 0, x.data_ptr(), dx.data_ptr(), R, C, mean.data_ptr(), istd.data_ptr(),
                       ptr(gamma), sp, parts, float(R), ptr(dgamma), ptr(dbeta), 0, st)
        return dx, (dy if want_masked else None)
    dmask = _empty(dy.shape, dy.dtype, dy.device, True) if (want_masked and yout is not None) else None
    sums = None
    # the (sum dy', sum dy' * xhat) pass: the batch-statistics backward needs it, and so does a
    # frozen-statistics (eval-mode) backward that still accumulates the affine gradients or
    # returns the masked gradient (bn_bwd_apply adds the sums to dgamma / dbeta either way and
    # uses them for dx only in training mode)
    if not eval_mode or dgamma is not None or dbeta is not None or dmask is not None:
        rows = K.bn_partial_rows(R, C)
        slab = _empty((rows, 2, C), F32, x.device)
        sums = _empty((2 * C,), F32, x.device)
        _trace_partial("bwd", x)
        K.bn_partial(dt, x.data_ptr(), dy.data_ptr(), ptr(yout), ptr(dmask), mean.data_ptr(), istd.data_ptr(), R, C,
                     slab.data_ptr(), 1, 0, st)
        sums = stat_reduce(1, slab, rows, C, sums)
    dx = _empty(x.shape, x.dtype, x.device, True)
    src = dmask if dmask is not None else dy
    sp, parts = _stats(sums)
    K.bn_bwd_apply(dt, src.data_ptr(), 0 if dmask is not None else ptr(yout), x.data_ptr(), dx.data_ptr(), R, C,
                   mean.data_ptr(), istd.data_ptr(), ptr(gamma), sp, parts, float(R), ptr(dgamma), ptr(dbeta),
                   int(eval_mode), st)
    return dx, dmask


def gn_fwd(x, groups, gamma, beta, eps):
    N, C, H, W = x.shape
    y = _empty(x.shape, x.dtype, x.device, True)
    mean = _empty((N * groups,), F32, x.device)
    istd = _empty_like(mean)
    kernels().gn_fwd(dt_code(x.dtype), x.data_ptr(), y.data_ptr(), N, H * W, C, groups, ptr(gamma), ptr(beta),
                     float(eps), mean.data_ptr(), istd.data_ptr(), stream_ptr())
    return y, mean, istd


def gn_bwd(dy, x, groups, gamma, mean, istd, dgamma, dbeta):
    N, C, H, W = x.shape
    dx = _empty(x.shape, x.dtype, x.device, True)
    aff = _empty((N, 2, C), F32, x.device)  # per-image affine partials
    kernels().gn_bwd(dt_code(x.dtype), dy.data_ptr(), x.data_ptr(), dx.data_ptr(), N, H * W, C, groups, ptr(gamma),
                     mean.data_ptr(), istd.data_ptr(), ptr(dgamma), ptr(dbeta), aff.data_ptr(), stream_ptr())
    return dx
