"""Stateless layers: MaxPool2D, AvgPool2D, Dropout, Flatten, Activation.

Reference: `maxpool2d_layer.tpp`, `avgpool2d_layer.tpp`, `dropout_layer.tpp`,
`flatten_layer.tpp`, `activation_layer.tpp`. Semantics kept: max-pool ties -> first element,
implicit -inf padding, stride 0 -> pool size; avg-pool divides by the full window
(count_include_pad); inverted dropout 1/(1-p).
"""
from __future__ import annotations

import random

import torch

from ..activations import ActivationFactory
from .base import LayerConfig, StatelessLayer


class _Pool(StatelessLayer):
    def __init__(self, pool_h, pool_w, stride_h=0, stride_w=0, pad_h=0, pad_w=0, name=""):
        super().__init__(name)
        self.pool_h, self.pool_w = int(pool_h), int(pool_w)
        self.stride_h = int(stride_h) if stride_h else self.pool_h   # maxpool2d_layer.tpp:20-21
        self.stride_w = int(stride_w) if stride_w else self.pool_w
        self.pad_h, self.pad_w = int(pad_h), int(pad_w)

    def _geom(self):
        return self.pool_h, self.pool_w, self.stride_h, self.stride_w, self.pad_h, self.pad_w

    def compute_output_shape(self, s):
        return [s[0], s[1], (s[2] + 2 * self.pad_h - self.pool_h) // self.stride_h + 1,
                (s[3] + 2 * self.pad_w - self.pool_w) // self.stride_w + 1]

    def forward_flops(self, s):
        o = self.compute_output_shape(s)
        return o[0] * o[1] * o[2] * o[3] * self.pool_h * self.pool_w

    def backward_flops(self, s):
        o = self.compute_output_shape(s)
        return o[0] * o[1] * o[2] * o[3]

    def get_config(self):
        return LayerConfig(self.name, dict(pool_h=self.pool_h, pool_w=self.pool_w, stride_h=self.stride_h,
                                           stride_w=self.stride_w, pad_h=self.pad_h, pad_w=self.pad_w), self.type_name)


class MaxPool2D(_Pool):
    type_name = "maxpool2d"

    def __init__(self, pool_h, pool_w, stride_h=0, stride_w=0, pad_h=0, pad_w=0, name="maxpool2d"):
        super().__init__(pool_h, pool_w, stride_h, stride_w, pad_h, pad_w, name)

    def forward(self, x, mb_id=0):
        x = self._to_layer_device(x)
        if getattr(x, "_prepooled_by", None) is self:
            return x  # the preceding BatchNorm+ReLU already pooled and filled this layer's cache
        if x.is_cuda:
            from ...ops import hip
            xa = hip.to_act(x, self.compute_dtype)
            y, idx = hip.maxpool_fwd(xa, *self._geom())
            # the output is kept (it is the next layer's cached input anyway): its sign is the
            # ReLU mask when the producing BatchNorm's backward statistics are fused in backward
            self._cache[mb_id] = (idx, tuple(xa.shape), y)
            return y
        from ...ops import cpu
        y, idx = cpu.maxpool_fwd(x, (self.pool_h, self.pool_w), (self.stride_h, self.stride_w),
                                 (self.pad_h, self.pad_w))
        self._cache[mb_id] = (idx, tuple(x.shape), None)
        return y

    def backward(self, grad, mb_id=0):
        idx, shape, y = self._cache.pop(mb_id)
        if idx.is_cuda:
            from ...ops import hip
            g = hip.to_act(grad.to(idx.device), self.compute_dtype)
            return hip.maxpool_bwd(g, idx, shape, *self._geom(), ypool=y, bnb=self._bnb_request)
        from ...ops import cpu
        return cpu.maxpool_bwd(grad.to(self.compute_dtype), idx, shape)

    @staticmethod
    def from_config(cfg):
        p = cfg.parameters
        return MaxPool2D(p["pool_h"], p["pool_w"], p.get("stride_h", 0), p.get("stride_w", 0), p.get("pad_h", 0),
                         p.get("pad_w", 0), cfg.name or "maxpool2d")


class AvgPool2D(_Pool):
    type_name = "avgpool2d"

    def __init__(self, pool_h, pool_w, stride_h=1, stride_w=1, pad_h=0, pad_w=0, name="avgpool2d"):
        super().__init__(pool_h, pool_w, stride_h, stride_w, pad_h, pad_w, name)

    def forward(self, x, mb_id=0):
        x = self._to_layer_device(x)
        if x.is_cuda:
            from ...ops import hip
            xa = hip.to_act(x, self.compute_dtype)
            y = hip.avgpool_fwd(xa, *self._geom())
            self._cache[mb_id] = tuple(xa.shape)
            return y
        from ...ops import cpu
        self._cache[mb_id] = tuple(x.shape)
        return cpu.avgpool_fwd(x, (self.pool_h, self.pool_w), (self.stride_h, self.stride_w),
                               (self.pad_h, self.pad_w))

    def backward(self, grad, mb_id=0):
        shape = self._cache.pop(mb_id)
        if grad.is_cuda or self._on_gpu():
            from ...ops import hip
            g = hip.to_act(grad.to(self.device.torch_device), self.compute_dtype)
            return hip.avgpool_bwd(g, shape, *self._geom())
        from ...ops import cpu
        return cpu.avgpool_bwd(grad.to(self.compute_dtype), shape, (self.pool_h, self.pool_w),
                               (self.stride_h, self.stride_w), (self.pad_h, self.pad_w))

    @staticmethod
    def from_config(cfg):
        p = cfg.parameters
        return AvgPool2D(p["pool_h"], p["pool_w"], p.get("stride_h", 1), p.get("stride_w", 1), p.get("pad_h", 0),
                         p.get("pad_w", 0), cfg.name or "avgpool2d")


class Dropout(StatelessLayer):
    type_name = "dropout"

    def __init__(self, dropout_rate: float, name: str = "dropout"):
        super().__init__(name)
        if not 0.0 <= dropout_rate < 1.0:
            raise ValueError("dropout_rate must be in [0, 1)")
        self.dropout_rate = float(dropout_rate)
        self._counter = 0
        self._dev_ctr = None   # GPU: device draw counter, advanced in-stream (hipGraph replays too)
        self._slots = {}       # mb_id -> 1-element device tensor holding that forward's draw index

    def _next_seed(self):
        self._counter += 1
        base = self.seed if self.use_seed else random.getrandbits(62)
        return (base * 0x9E3779B97F4A7C15 + self._counter) & ((1 << 63) - 1)

    def forward(self, x, mb_id=0):
        x = self._to_layer_device(x)
        if not self.training or self.dropout_rate == 0.0:
            self._cache[mb_id] = None
            return x
        seed = self._next_seed()
        if x.is_cuda:
            from ...ops import hip
            xa = hip.to_act(x, self.compute_dtype) if x.dim() == 4 else x.to(self.compute_dtype).contiguous()
            # the host seed is a constant of a captured graph: the per-forward draw index is
            # bumped on the device so every replay (and every micro-batch) gets a fresh mask
            if self._dev_ctr is None or self._dev_ctr.device != xa.device:
                self._dev_ctr = torch.zeros(1, dtype=torch.int64, device=xa.device)
                self._slots = {}
            slot = self._slots.get(mb_id)
            if slot is None:
                slot = self._slots[mb_id] = torch.zeros(1, dtype=torch.int64, device=xa.device)
            hip.counter_bump(self._dev_ctr, slot)
            self._cache[mb_id] = (seed, slot)   # mask regenerated from Philox(seed, slot) in backward
            return hip.dropout(xa, self.dropout_rate, seed, slot)
        from ...ops import cpu
        u = cpu.fill_random(torch.empty(x.shape, dtype=x.dtype), 0.0, 1.0, seed, False)  # Philox, as on the GPU
        mask = cpu.elementwise(1, 7, u, s0=self.dropout_rate)             # u > p
        cpu.elementwise(1, 2, mask, out=mask, s0=1.0 / (1 - self.dropout_rate))
        self._cache[mb_id] = mask
        return cpu.elementwise(0, 2, x, mask)

    def backward(self, grad, mb_id=0):
        ent = self._cache.pop(mb_id, None)
        if ent is None:
            return grad
        if isinstance(ent, tuple):
            from ...ops import hip
            g = hip.to_act(grad, self.compute_dtype) if grad.dim() == 4 else grad.to(self.compute_dtype).contiguous()
            return hip.dropout(g, self.dropout_rate, ent[0], ent[1])
        from ...ops import cpu
        return cpu.elementwise(0, 2, grad.to(ent.dtype), ent)

    def forward_flops(self, s):
        n = 1
        for d in s:
            n *= d
        return 2 * n

    def backward_flops(self, s):
        return self.forward_flops(s) // 2

    def get_config(self):
        return LayerConfig(self.name, dict(dropout_rate=self.dropout_rate), self.type_name)

    @staticmethod
    def from_config(cfg):
        return Dropout(cfg.parameters["dropout_rate"], cfg.name or "dropout")


class Flatten(StatelessLayer):
    """[N,C,H,W] -> [N,C*H*W,1,1] in NCHW element order (checkpoint-compatible dense weights)."""
    type_name = "flatten"

    def forward(self, x, mb_id=0):
        x = self._to_layer_device(x)
        self._cache[mb_id] = tuple(x.shape)
        n = x.shape[0]
        if x.dim() == 4 and (x.shape[2] != 1 or x.shape[3] != 1) and not x.is_contiguous():
            if x.is_cuda and x.is_contiguous(memory_format=torch.channels_last):
                from ...ops import hip
                x = hip.nchw_nhwc(x, False)  # NHWC activation -> NCHW order (reference flatten order)
            else:
                x = x.contiguous()
        return x.reshape(n, -1, 1, 1)

    def backward(self, grad, mb_id=0):
        shape = self._cache.pop(mb_id)
        g = grad.reshape(shape)
        if g.is_cuda and len(shape) == 4 and not g.is_contiguous(memory_format=torch.channels_last):
            from ...ops import hip
            g = hip.nchw_nhwc(g.contiguous(), True)
        return g

    def compute_output_shape(self, s):
        f = 1
        for d in s[1:]:
            f *= d
        return [s[0], f, 1, 1]

    def get_config(self):
        return LayerConfig(self.name, {}, self.type_name)

    @staticmethod
    def from_config(cfg):
        return Flatten(cfg.name or "flatten")


class Activation(StatelessLayer):
    type_name = "activation"

    def __init__(self, activation: str = "relu", name: str = "activation"):
        super().__init__(name)
        self.activation_name = activation
        self.fn = ActivationFactory.create(activation)
        self.passthrough = False  # set by the planner when fused into the preceding BatchNorm

    def forward(self, x, mb_id=0):
        x = self._to_layer_device(x)
        if self.passthrough or self.fn is None:
            return x
        if x.is_cuda:
            from ...ops import hip
            x = hip.to_act(x, self.compute_dtype) if x.dim() == 4 else x.to(self.compute_dtype).contiguous()
        y = self.fn.apply(x)
        self._cache[mb_id] = (x, y)
        return y

    def backward(self, grad, mb_id=0):
        if self.passthrough or self.fn is None:
            return grad
        x, y = self._cache.pop(mb_id)
        grad = grad.to(x.device)
        if x.is_cuda:
            from ...ops import hip
            grad = hip.to_act(grad, self.compute_dtype) if grad.dim() == 4 else grad.to(self.compute_dtype)
        return self.fn.gradient(x, y, grad)

    def forward_flops(self, s):
        n = 1
        for d in s:
            n *= d
        return n

    def backward_flops(self, s):
        return self.forward_flops(s)

    def get_config(self):
        return LayerConfig(self.name, dict(activation=self.activation_name), self.type_name)

    @staticmethod
    def from_config(cfg):
        return Activation(cfg.parameters.get("activation", "relu"), cfg.name or "activation")
