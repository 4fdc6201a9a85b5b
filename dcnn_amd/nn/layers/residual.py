"""ResidualBlock: ``out = act(F(x) + S(x))`` (reference `include/nn/blocks_impl/residual_block.hpp:30-476`).

GPU path fuses the tail of the block: the last BatchNorm of F applies ``+ S(x)`` and the ReLU
in the same pass (no pre-activation tensor, no separate add/ReLU kernels), its backward emits
the ReLU-masked gradient once for both branches, and the branch sum ``dF + dS`` is fused into
the epilogue of the first conv's dgrad GEMM.
"""
from __future__ import annotations

import json
from typing import List, Optional

import torch

from ..activations import ActivationFactory
from .base import LayerConfig, Layer, run_backward
from .conv import Conv2D
from .misc import Activation, MaxPool2D
from .norm import BatchNorm


def fuse_kinds(layers: List[Layer]) -> List[int]:
    """Layer kinds for the shared fusion planner (csrc/kernels/fusion_plan.h)."""
    from ...ops._ext import kernels
    K = kernels()
    out = []
    for l in layers:
        if isinstance(l, Conv2D):
            out.append(K.FK_CONV)
        elif isinstance(l, BatchNorm):
            out.append(K.FK_BN)
        elif isinstance(l, Activation):
            out.append(K.FK_RELU if l.activation_name == "relu" else K.FK_ACT)
        elif isinstance(l, MaxPool2D):
            out.append(K.FK_MAXPOOL)
        else:
            out.append(K.FK_OTHER)
    return out


def plan_fusion(layers: List[Layer], on_gpu: bool) -> None:
    """Mark cross-layer fusions for the GPU path (no-op on CPU: pure reference semantics). The
    rules are the shared planner's (csrc/kernels/fusion_plan.cpp, plan_sequence_fusions) — the
    C++ host API's nn.cpp applies the same ones: conv -> BatchNorm statistics rows from the conv
    epilogue, BatchNorm -> ReLU in one apply pass, BatchNorm + ReLU + max-pool (the pool computed by
    the BatchNorm's forward when the shapes allow it at run time). The backward-BatchNorm requests
    of BatchNorm [+ ReLU] -> conv are made at run time here (BatchNorm.bwd_bn_spec)."""
    for l in layers:
        if isinstance(l, Conv2D):
            l.emit_bn_stats = False
        if isinstance(l, BatchNorm):
            l.fuse_relu = False
            l.fuse_pool = None
            l.emit_masked_grad = False
        if isinstance(l, Activation):
            l.passthrough = False
    if not on_gpu:
        return
    from ...ops._ext import kernels
    K = kernels()
    flags = K.plan_sequence_fusions(fuse_kinds(layers))
    for i, (l, f) in enumerate(zip(layers, flags)):
        if isinstance(l, Conv2D) and f & K.FF_EMIT_BN_STATS:
            l.emit_bn_stats = True
        if isinstance(l, BatchNorm) and f & K.FF_FUSE_RELU:
            l.fuse_relu = True
        if isinstance(l, Activation) and f & K.FF_PASSTHROUGH:
            l.passthrough = True
        if isinstance(l, BatchNorm) and f & K.FF_FUSE_POOL:
            l.fuse_pool = layers[i + 2]


class ResidualBlock(Layer):
    type_name = "residual_block"

    def __init__(self, main_path: List[Layer], shortcut_path: Optional[List[Layer]] = None,
                 activation: str = "relu", name: str = "residual_block"):
        super().__init__(name)
        self.main_path = list(main_path)
        self.shortcut_path = list(shortcut_path or [])
        self.activation_type = activation
        self.act = ActivationFactory.create(activation)
        self._fused = self._dual = False

    # structure -------------------------------------------------------------------------
    def sublayers(self) -> List[Layer]:
        return self.main_path + self.shortcut_path

    def get_main_path(self):
        return self.main_path

    def get_shortcut_path(self):
        return self.shortcut_path

    def has_parameters(self):
        return any(l.has_parameters() for l in self.sublayers())

    def parameters(self):
        return [p for l in self.sublayers() for p in l.parameters()]

    def gradients(self):
        return [g for l in self.sublayers() for g in l.gradients()]

    def set_training(self, training):
        super().set_training(training)
        for l in self.sublayers():
            l.set_training(training)

    def set_device(self, device):
        super().set_device(device)
        for l in self.sublayers():
            l.set_device(device)
        self._plan()

    def set_compute_dtype(self, dtype):
        super().set_compute_dtype(dtype)
        for l in self.sublayers():
            l.set_compute_dtype(dtype)

    def set_seed(self, seed):
        super().set_seed(seed)
        for i, l in enumerate(self.sublayers()):
            l.set_seed(seed + 1 + i)

    def initialize(self):
        for l in self.sublayers():
            l.initialize()
        self._plan()
        self.initialized = True

    def _plan(self):
        on_gpu = self.device.is_gpu()
        plan_fusion(self.main_path, on_gpu)
        plan_fusion(self.shortcut_path, on_gpu)
        act_ok = self.activation_type in ("relu", "none", "linear")
        self._fused = self._dual = False
        if on_gpu:  # the shared planner's residual rules (fusion_plan.cpp, plan_residual_fusions)
            from ...ops._ext import kernels
            K = kernels()
            rf = K.plan_residual_fusions(fuse_kinds(self.main_path), fuse_kinds(self.shortcut_path), act_ok)
            self._fused = bool(rf & K.RF_FUSED_TAIL)
            self._dual = bool(rf & K.RF_DUAL_SHORTCUT)
        if self._fused:
            self.main_path[-1].emit_masked_grad = True
        for l in self.sublayers():
            l.needs_input_grad = True
        if self.main_path:
            self.main_path[0].needs_input_grad = self.needs_input_grad
        if self.shortcut_path:
            self.shortcut_path[0].needs_input_grad = self.needs_input_grad

    def clear_cache(self, mb_id=None):
        super().clear_cache(mb_id)
        for l in self.sublayers():
            l.clear_cache(mb_id)

    # compute ---------------------------------------------------------------------------
    def forward(self, x, mb_id=0):
        x = self._to_layer_device(x)
        if self._fused:
            from ...ops import hip
            xa = hip.to_act(x, self.compute_dtype)
            s = xa
            sp = self.shortcut_path
            # a projection shortcut ending in BatchNorm is applied inside the tail BatchNorm's
            # pass (hip.bn_apply_dual): its normalised output is never written
            defer = self._dual and self.compute_dtype == torch.bfloat16
            for l in (sp[:-1] if defer else sp):
                s = l.forward(s, mb_id)
            if defer:
                s = sp[-1].forward_deferred(s, mb_id)
            h = xa
            for l in self.main_path[:-1]:
                h = l.forward(h, mb_id)
            out = self.main_path[-1].forward(h, mb_id, residual=s if defer else hip.to_act(s, self.compute_dtype),
                                             relu=self.activation_type == "relu")
            self._cache[mb_id] = ("fused", None)
            return out
        h = x
        for l in self.main_path:
            h = l.forward(h, mb_id)
        s = x
        for l in self.shortcut_path:
            s = l.forward(s, mb_id)
        pre = h + s
        out = self.act.apply(pre) if self.act is not None else pre
        self._cache[mb_id] = ("plain", (pre, out))
        return out

    def backward(self, grad, mb_id=0):
        kind, ent = self._cache.pop(mb_id)
        if kind == "fused":
            last = self.main_path[-1]
            d_pair = self._pair_backward_stats(grad, mb_id)
            g = last.backward(grad, mb_id)
            d_pre = last.pop_masked_grad(mb_id)
            d_s = d_pair if d_pair is not None else d_pre
            for l in reversed(self.shortcut_path):
                d_s = l.backward(d_s, mb_id)
            for k in range(len(self.main_path) - 2, 0, -1):
                # the BN below (after its passthrough ReLU) gets its mask + statistics fused into
                # this layer's dgrad epilogue
                g = run_backward(self.main_path, k, g, mb_id)
            first = self.main_path[0]
            if not self.needs_input_grad:
                first.backward(g, mb_id) if len(self.main_path) > 1 else None
                return None
            if len(self.main_path) == 1:
                return g + d_s
            if isinstance(first, Conv2D):
                # the block's input gradient dF + dS is consumed by the previous block's tail BN:
                # forward the outer container's fusion request to the conv that produces it
                first._bnb_request = self._bnb_request
                try:
                    return first.backward(g, mb_id, add_to=d_s)
                finally:
                    first._bnb_request = None
            return first.backward(g, mb_id) + d_s
        pre, out = ent
        g = self.act.gradient(pre, out, grad) if self.act is not None else grad
        d_main = g
        for l in reversed(self.main_path):
            d_main = l.backward(d_main, mb_id)
        d_s = g
        for l in reversed(self.shortcut_path):
            d_s = l.backward(d_s, mb_id)
        if not self.needs_input_grad:
            return None
        return d_main + d_s

    def _pair_backward_stats(self, grad, mb_id):
        """When the tail BatchNorm's backward statistics come fused from the producer of ``grad``
        (the ReLU-masked gradient that both the tail and the projection shortcut's BatchNorm
        receive), reduce the shortcut BatchNorm's statistics in the same launch as the tail's
        (hip.stat_reduce_pair). Returns the shortcut's incoming gradient carrying its reduced
        statistics, or None (unpaired path)."""
        from ...ops import fusion, hip
        sp = self.shortcut_path
        pre = getattr(grad, "_bnb", None)
        bns = sp[-1] if self._dual else None
        if (bns is None or pre is None or pre[0] is not self.main_path[-1] or not fusion.BN_DUAL
                or isinstance(pre[1], hip.Stats) or grad.dtype != torch.bfloat16
                or not grad.is_contiguous(memory_format=torch.channels_last)):
            return None
        ent = bns._cache.get(mb_id)
        if ent is None or not ent[4] or ent[0].dtype != torch.bfloat16 or tuple(ent[0].shape) != tuple(grad.shape):
            return None
        xs, _, ms, iss, _ = ent
        raw = hip.bn_bwd_stats_raw(grad, xs, ms, iss)
        sa, sb = hip.stat_reduce_pair(1, (pre[1], pre[2], pre[3]), raw, grad.shape[1])
        d = grad.detach()  # same storage, its own tag for the shortcut BatchNorm
        tail = self.main_path[-1]
        tent = tail._cache.get(mb_id)
        done = tent is not None and hip.bn_dual_ok(tent[0]) and tuple(tent[0].shape) == tuple(xs.shape)
        if done:
            # both data gradients from one read of the shared gradient (hip.bn_bwd_apply_dual)
            dx_t, dx_s = hip.bn_bwd_apply_dual(grad, (tail, tent, sa), (bns, ent, sb))
            grad._bnb = (tail, "done", dx_t)
            d._bnb = (bns, "done", dx_s)
        else:
            grad._bnb = (pre[0], sa, pre[2], pre[3])
            d._bnb = (bns, sb, raw[1], raw[2])
        return d

    def bwd_bn_spec(self, mb_id=0):
        ent = self._cache.get(mb_id)
        if not self._fused or ent is None or ent[0] != "fused":
            return None
        return self.main_path[-1].bwd_bn_spec(mb_id)

    # shapes / cost -----------------------------------------------------------------------
    def compute_output_shape(self, s):
        for l in self.main_path:
            s = l.compute_output_shape(s)
        return s

    def _flops(self, s, fwd):
        total = 0
        cur = list(s)
        for l in self.main_path:
            total += l.forward_flops(cur) if fwd else l.backward_flops(cur)
            cur = l.compute_output_shape(cur)
        cur2 = list(s)
        for l in self.shortcut_path:
            total += l.forward_flops(cur2) if fwd else l.backward_flops(cur2)
            cur2 = l.compute_output_shape(cur2)
        n = 1
        for d in cur:
            n *= d
        return total + 2 * n

    def forward_flops(self, s):
        return self._flops(s, True)

    def backward_flops(self, s):
        return self._flops(s, False)

    def cached_memory_bytes(self):
        return super().cached_memory_bytes() + sum(l.cached_memory_bytes() for l in self.sublayers())

    # config ------------------------------------------------------------------------------
    @staticmethod
    def _dump_path(path):
        arr = []
        for l in path:
            c = l.get_config()
            arr.append({"type": l.type(), "name": c.name, "parameters": c.parameters})
        return json.dumps(arr)

    def get_config(self):
        return LayerConfig(self.name, dict(activation=self.activation_type,
                                           has_projection=bool(self.shortcut_path),
                                           main_path=self._dump_path(self.main_path),
                                           shortcut_path=self._dump_path(self.shortcut_path)), self.type_name)

    @staticmethod
    def from_config(cfg):
        from . import create_layer
        p = cfg.parameters
        main = [create_layer(d["type"], LayerConfig(d.get("name", ""), d.get("parameters", {}), d["type"]))
                for d in json.loads(p.get("main_path", "[]"))]
        short = []
        if p.get("has_projection", False):
            short = [create_layer(d["type"], LayerConfig(d.get("name", ""), d.get("parameters", {}), d["type"]))
                     for d in json.loads(p.get("shortcut_path", "[]"))]
        return ResidualBlock(main, short, p.get("activation", "relu"), cfg.name or "residual_block")

    def clone(self):
        c = ResidualBlock([l.clone() for l in self.main_path], [l.clone() for l in self.shortcut_path],
                          self.activation_type, self.name)
        c.training = self.training
        return c
