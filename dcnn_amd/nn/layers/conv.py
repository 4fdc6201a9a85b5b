"""Conv2D and Dense layers.

Reference: `include/nn/layers_impl/conv2d_layer.tpp` (im2col -> cuBLAS -> CNHW->NCHW -> bias,
cuDNN variant) and `include/nn/layers_impl/dense_layer.tpp`. GPU path here: implicit-GEMM on
MFMA (no im2col buffer, no layout transposes, bias/residual/BN-statistics fused into the
epilogue, split-K wgrad accumulating into the fp32 master gradient). CPU path: the native
backend's per-sample im2col + blocked GEMM (``ops/cpu.py``), float32 or float64.
"""
from __future__ import annotations

import math
from typing import List, Optional

import torch

from ..params import ParamSpec
from .base import LayerConfig, ParameterizedLayer


class Conv2D(ParameterizedLayer):
    type_name = "conv2d"

    def __init__(self, in_channels: int, out_channels: int, kernel_h: int, kernel_w: int, stride_h: int = 1,
                 stride_w: int = 1, pad_h: int = 0, pad_w: int = 0, use_bias: bool = True, name: str = "conv2d"):
        super().__init__(name)
        self.in_channels, self.out_channels = int(in_channels), int(out_channels)
        self.kernel_h, self.kernel_w = int(kernel_h), int(kernel_w)
        self.stride_h, self.stride_w = int(stride_h), int(stride_w)
        self.pad_h, self.pad_w = int(pad_h), int(pad_w)
        self.use_bias = bool(use_bias)
        # GPU fusion hooks set by the Sequential planner
        self.emit_bn_stats = False

    # params ---------------------------------------------------------------------------
    def param_specs(self):
        s = [ParamSpec("weights", (self.out_channels, self.in_channels, self.kernel_h, self.kernel_w), True)]
        if self.use_bias:
            s.append(ParamSpec("bias", (self.out_channels, 1, 1, 1)))
        return s

    def init_values(self, gen):
        fan_in = self.in_channels * self.kernel_h * self.kernel_w
        bound = 1.0 / math.sqrt(fan_in)  # conv2d_layer.tpp:70-86
        vals = [torch.empty(self.param_specs()[0].shape).uniform_(-bound, bound, generator=gen)]
        if self.use_bias:
            vals.append(torch.empty((self.out_channels, 1, 1, 1)).uniform_(-bound, bound, generator=gen))
        return vals

    @property
    def weights(self):
        return self._params[0]

    @property
    def bias(self):
        return self._params[1] if self.use_bias else None

    def _bias_vec(self):
        return self._params[1].view(-1) if self.use_bias else None

    # compute --------------------------------------------------------------------------
    def forward(self, x, mb_id=0):
        if not self.initialized:
            raise RuntimeError(f"Conv2D '{self.name}' must be initialized before forward")
        x = self._to_layer_device(x)
        if x.shape[1] != self.in_channels:
            raise ValueError(f"Conv2D '{self.name}': input has {x.shape[1]} channels, expected {self.in_channels}")
        if x.is_cuda:
            from ...ops import hip
            st, pd = (self.stride_h, self.stride_w), (self.pad_h, self.pad_w)
            if (self.compute_dtype == torch.bfloat16 and not self.needs_input_grad
                    and hip.stem_ok(x, self.weights.shape, st, pd)):
                # RGB stem straight from the fp32 NCHW input (stem.hip): no layout/pad pass
                y, partial = hip.stem_conv_fwd(x, self.weight_operand(0), self._bias_vec(),
                                               stats=self.emit_bn_stats and self.training)
                if partial is not None:
                    y._bn_partial = partial
                self._cache[mb_id] = (x, tuple(x.shape), "stem")
                return y
            if self.in_channels < 8 and self.compute_dtype == torch.bfloat16:
                # RGB stem: zero-pad channels to 8 so every 16-byte chunk is one tap (vector path)
                xa = hip.to_act_padded(x, 8)
                w = hip.pad_weight_channels(self.weight_operand(0), 8, out=getattr(self, "_wpad", None))
                self._wpad = w  # padding channels stay zero: later steps copy only the real ones
            else:
                xa = hip.to_act(x, self.compute_dtype)
                w = self.weight_operand(0)
            y, partial = hip.conv2d_fwd(xa, w, self._bias_vec(), (self.stride_h, self.stride_w),
                                        (self.pad_h, self.pad_w), stats=self.emit_bn_stats and self.training)
            if partial is not None:
                y._bn_partial = partial
            self._cache[mb_id] = (xa, tuple(x.shape))
            return y
        from ...ops import cpu
        y = cpu.conv2d_fwd(x, self.weights, self._bias_vec(), (self.stride_h, self.stride_w), (self.pad_h, self.pad_w))
        self._cache[mb_id] = x
        return y

    def backward(self, grad, mb_id=0, add_to: Optional[torch.Tensor] = None):
        x = self._cache.pop(mb_id, None)
        if x is None:
            raise RuntimeError(f"Conv2D '{self.name}': no cached input for micro-batch {mb_id}")
        stem = isinstance(x, tuple) and len(x) == 3
        if isinstance(x, tuple):
            x, x_shape = x[0], x[1]
        else:
            x_shape = tuple(x.shape)
        grad = grad.to(x.device)
        if x.is_cuda:
            from ...ops import hip
            g = hip.to_act(grad, self.compute_dtype)
            gb = self._grads[1].view(-1) if self.use_bias else None
            if stem:  # forward ran stem.hip (never with an input gradient)
                hip.stem_conv_wgrad(g, x, self._grads[0], gb)
                return None
            hip.conv2d_wgrad(g, x, self.weights.shape, (self.stride_h, self.stride_w), (self.pad_h, self.pad_w),
                             self._grads[0], gb)
            if not self.needs_input_grad:
                return None
            if getattr(self, "_wt_valid", False):
                wt = self._wt_buf  # refreshed by the model's batched WeightTransposer this step
            else:
                wt = hip.conv_weight_t(self.weight_operand(0), dtype=self.compute_dtype)
            res = hip.to_act(add_to, self.compute_dtype) if add_to is not None else None
            return hip.conv2d_dgrad(g, wt, x_shape, (self.stride_h, self.stride_w), (self.pad_h, self.pad_w),
                                    residual=res, bnb=self._bnb_request)
        from ...ops import cpu
        st, pd = (self.stride_h, self.stride_w), (self.pad_h, self.pad_w)
        dx = cpu.conv2d_bwd(x, self.weights, grad.to(x.dtype), st, pd, self._grads[0],
                            self._grads[1].view(-1) if self.use_bias else None, need_dx=self.needs_input_grad)
        if dx is not None and add_to is not None:
            cpu.elementwise(0, 0, dx, add_to.to(dx.dtype), out=dx)
        return dx

    # shapes / cost ----------------------------------------------------------------------
    def _out_hw(self, h, w):
        return ((h + 2 * self.pad_h - self.kernel_h) // self.stride_h + 1,
                (w + 2 * self.pad_w - self.kernel_w) // self.stride_w + 1)

    def compute_output_shape(self, s):
        oh, ow = self._out_hw(s[2], s[3])
        return [s[0], self.out_channels, oh, ow]

    def forward_flops(self, s):
        oh, ow = self._out_hw(s[2], s[3])
        out = s[0] * oh * ow
        k = self.in_channels * self.kernel_h * self.kernel_w
        f = 2 * self.out_channels * k * out
        if self.use_bias:
            f += self.out_channels * out
        return f

    def backward_flops(self, s):
        oh, ow = self._out_hw(s[2], s[3])
        out = s[0] * oh * ow
        k = self.in_channels * self.kernel_h * self.kernel_w
        f = 4 * self.out_channels * k * out  # weight grad + input grad
        if self.use_bias:
            f += self.out_channels * out
        return f

    def get_config(self):
        return LayerConfig(self.name, dict(
            in_channels=self.in_channels, out_channels=self.out_channels, kernel_h=self.kernel_h,
            kernel_w=self.kernel_w, stride_h=self.stride_h, stride_w=self.stride_w, pad_h=self.pad_h,
            pad_w=self.pad_w, use_bias=self.use_bias, optimized="mfma"), self.type_name)

    @staticmethod
    def from_config(cfg):
        p = cfg.parameters
        return Conv2D(p["in_channels"], p["out_channels"], p["kernel_h"], p["kernel_w"], p.get("stride_h", 1),
                      p.get("stride_w", 1), p.get("pad_h", 0), p.get("pad_w", 0), p.get("use_bias", True),
                      cfg.name or "conv2d")


class Dense(ParameterizedLayer):
    type_name = "dense"

    def __init__(self, input_features: int, output_features: int, use_bias: bool = True, name: str = "dense"):
        super().__init__(name)
        self.input_features, self.output_features = int(input_features), int(output_features)
        self.use_bias = bool(use_bias)

    def param_specs(self):
        s = [ParamSpec("weights", (self.output_features, self.input_features, 1, 1))]
        if self.use_bias:
            s.append(ParamSpec("bias", (self.output_features, 1, 1, 1)))
        return s

    def init_values(self, gen):
        bound = 1.0 / math.sqrt(self.input_features)  # dense_layer.tpp:39-55
        vals = [torch.empty((self.output_features, self.input_features, 1, 1)).uniform_(-bound, bound, generator=gen)]
        if self.use_bias:
            vals.append(torch.empty((self.output_features, 1, 1, 1)).uniform_(-bound, bound, generator=gen))
        return vals

    @property
    def weights(self):
        return self._params[0]

    @property
    def bias(self):
        return self._params[1] if self.use_bias else None

    def _flat_in(self, x):
        n = x.shape[0]
        feat = x.numel() // n
        if feat != self.input_features:
            raise ValueError(f"Dense '{self.name}': got {feat} input features, expected {self.input_features}")
        if x.dim() == 4 and (x.shape[2] != 1 or x.shape[3] != 1):
            x = x.contiguous()  # NCHW flatten order (checkpoint compatible)
        return x.reshape(n, feat)

    def forward(self, x, mb_id=0):
        if not self.initialized:
            raise RuntimeError(f"Dense '{self.name}' must be initialized before forward")
        x = self._to_layer_device(x)
        x2 = self._flat_in(x)
        n = x2.shape[0]
        if x2.is_cuda:
            from ...ops import hip
            x2 = x2.to(self.compute_dtype).contiguous()
            w = self.weight_operand(0).view(self.output_features, self.input_features)
            b = self._params[1].view(-1) if self.use_bias else None
            y = hip.dense_fwd(x2, w, b)
        else:
            from ...ops import cpu
            y = cpu.dense_fwd(x2, self.weights.view(self.output_features, self.input_features),
                              self._params[1].view(-1) if self.use_bias else None)
        self._cache[mb_id] = (x2, tuple(x.shape))
        return y.view(n, self.output_features, 1, 1)

    def backward(self, grad, mb_id=0):
        ent = self._cache.pop(mb_id, None)
        if ent is None:
            raise RuntimeError(f"Dense '{self.name}': no cached input for micro-batch {mb_id}")
        x2, in_shape = ent
        n = x2.shape[0]
        g2 = grad.to(x2.device).reshape(n, self.output_features)
        if x2.is_cuda:
            from ...ops import hip
            g2 = g2.to(self.compute_dtype).contiguous()
            hip.dense_wgrad(g2, x2, self._grads[0], self._grads[1].view(-1) if self.use_bias else None)
            if not self.needs_input_grad:
                return None
            w = self.weight_operand(0)
            wt = hip.conv_weight_t(w.view(self.output_features, self.input_features, 1, 1),
                                   dtype=self.compute_dtype).view(
                self.input_features, self.output_features)
            dx = hip.dense_dgrad(g2, wt)
        else:
            from ...ops import cpu
            w = self.weights.view(self.output_features, self.input_features)
            dx = cpu.dense_bwd(x2, w, g2.to(x2.dtype), self._grads[0].view(self.output_features, self.input_features),
                               self._grads[1].view(-1) if self.use_bias else None, need_dx=self.needs_input_grad)
            if dx is None:
                return None
        if len(in_shape) == 4 and (in_shape[2] != 1 or in_shape[3] != 1):
            dx = dx.view(in_shape)
            if dx.is_cuda:
                from ...ops import hip
                dx = hip.nchw_nhwc(dx, True)  # NCHW-order rows -> the NHWC activation layout
            return dx
        return dx.view(in_shape)

    def compute_output_shape(self, s):
        return [s[0], self.output_features, 1, 1]

    def forward_flops(self, s):
        return 2 * s[0] * self.input_features * self.output_features + (s[0] * self.output_features if self.use_bias else 0)

    def backward_flops(self, s):
        return 4 * s[0] * self.input_features * self.output_features + (s[0] * self.output_features if self.use_bias else 0)

    def get_config(self):
        return LayerConfig(self.name, dict(input_features=self.input_features, output_features=self.output_features,
                                           use_bias=self.use_bias, optimized="mfma"), self.type_name)

    @staticmethod
    def from_config(cfg):
        p = cfg.parameters
        return Dense(p["input_features"], p["output_features"], p.get("use_bias", True), cfg.name or "dense")
