"""BatchNorm and GroupNorm layers.

Reference: `include/nn/layers_impl/batchnorm_layer.tpp:27-369`,
`include/nn/layers_impl/groupnorm_layer.tpp:21-321`. GPU path: split-reduction statistics
(or the preceding conv's epilogue partials), one fused apply pass (+ReLU, +residual add of a
ResNet block), fused ReLU-masked backward; x_hat is recomputed rather than stored. CPU path:
the native backend (two-pass statistics in double, fused affine/residual/ReLU, one pass per
channel for the backward).
dgamma/dbeta ACCUMULATE on both devices (reference defect G4).
"""
from __future__ import annotations

from typing import Optional

import torch

from ...runtime.arena import empty as _arena_empty
from ..params import ParamSpec
from .base import LayerConfig, ParameterizedLayer


# BatchNorm cache marker: the forward fused ReLU + max-pool (see BatchNorm.forward)
_POOLED = object()


class BatchNorm(ParameterizedLayer):
    type_name = "batchnorm"

    def __init__(self, num_features: int, epsilon: float = 1e-5, momentum: float = 0.1, affine: bool = True,
                 name: str = "batchnorm"):
        super().__init__(name)
        self.num_features = int(num_features)
        self.epsilon = float(epsilon)
        self.momentum = float(momentum)
        self.affine = bool(affine)
        self.running_mean = torch.zeros(self.num_features)
        self.running_var = torch.ones(self.num_features)
        # GPU fusion flags (set by the Sequential/ResidualBlock planner)
        self.fuse_relu = False          # apply ReLU in the same pass (next Activation is passthrough)
        self.emit_masked_grad = False   # backward also returns dy*(y>0) for a residual branch
        self._last_masked = {}

    def param_specs(self):
        if not self.affine:
            return []
        return [ParamSpec("gamma", (self.num_features, 1, 1, 1)), ParamSpec("beta", (self.num_features, 1, 1, 1))]

    def init_values(self, gen):
        if not self.affine:
            return []
        return [torch.ones((self.num_features, 1, 1, 1)), torch.zeros((self.num_features, 1, 1, 1))]

    def has_parameters(self):
        return self.affine

    def initialize(self):
        super().initialize()
        self._move_buffers(self.device)

    def _move_buffers(self, device):
        td = device.torch_device
        self.running_mean = self.running_mean.to(td)
        self.running_var = self.running_var.to(td)

    def _gamma(self):
        return self._params[0].view(-1) if self.affine else None

    def _beta(self):
        return self._params[1].view(-1) if self.affine else None

    def forward(self, x, mb_id=0, residual: Optional[torch.Tensor] = None, relu: Optional[bool] = None):
        """``residual``/``relu`` are used by a ResidualBlock to fuse ``act(bn(x) + shortcut)``."""
        x = self._to_layer_device(x)
        if x.shape[1] != self.num_features:
            raise ValueError(f"BatchNorm '{self.name}': {x.shape[1]} channels, expected {self.num_features}")
        do_relu = self.fuse_relu if relu is None else relu
        if x.is_cuda:
            from ...ops import hip
            xa = hip.to_act(x, self.compute_dtype)
            C = self.num_features
            pool = self.fuse_pool
            if (self.training and pool is not None and do_relu and residual is None
                    and hip.bn_relu_maxpool_ok(xa, *pool._geom())):
                # BatchNorm + ReLU + max-pool in one pass: the full-resolution output is never
                # stored; the pool layer finds its cache filled and passes the result through
                sums = hip.bn_stats(xa, getattr(x, "_bn_partial", None))
                mean = _arena_empty((C,), torch.float32, xa.device)
                istd = _arena_empty((C,), torch.float32, xa.device)
                y, idx = hip.bn_relu_maxpool(xa, sums, xa.numel() // C, self._gamma(), self._beta(), self.epsilon,
                                             pool._geom(), save=(mean, istd),
                                             running=(self.running_mean, self.running_var), momentum=self.momentum)
                pool._cache[mb_id] = (idx, tuple(xa.shape), y)
                y._prepooled_by = pool
                # backward: the pool's fused backward masks with the pooled value (y > 0) and
                # hands this layer its statistics; there is no full-resolution ReLU output
                self._cache[mb_id] = (xa, _POOLED, mean, istd, True)
                return y
            dual = isinstance(residual, hip.BnDeferred)
            if dual and not hip.bn_dual_ok(xa):
                residual, dual = residual.materialize(), False
            apply = hip.bn_apply_dual if dual else hip.bn_apply
            args = dict(other=residual) if dual else dict(residual=residual)
            if self.training:
                part = getattr(x, "_bn_partial", None)
                if dual and isinstance(residual.sums, tuple):
                    # this layer's and the deferred shortcut BatchNorm's reduces in one launch
                    sums, residual.sums = hip.stat_reduce_pair(0, hip.bn_stats_raw(xa, part), residual.sums, C)
                else:
                    sums = hip.bn_stats(xa, part)
                count = xa.numel() // C
                mean = _arena_empty((C,), torch.float32, xa.device)
                istd = _arena_empty((C,), torch.float32, xa.device)
                y = apply(xa, sums, count, self._gamma(), self._beta(), self.epsilon, relu=do_relu, save=(mean, istd),
                          running=(self.running_mean, self.running_var), momentum=self.momentum, **args)
            else:
                y = apply(xa, None, 1, self._gamma(), self._beta(), self.epsilon, relu=do_relu,
                          running=(self.running_mean, self.running_var), use_running=True, **args)
                mean = self.running_mean
                istd = torch.rsqrt(self.running_var + self.epsilon)
            self._cache[mb_id] = (xa, y if do_relu else None, mean, istd, self.training)
            return y
        # ---- CPU: native backend (two-pass per-channel statistics, fused affine/residual/ReLU)
        from ...ops import cpu
        if self.running_mean.dtype != x.dtype:
            self.running_mean = self.running_mean.to(x.dtype)
            self.running_var = self.running_var.to(x.dtype)
        res = residual.to(x.dtype) if residual is not None else None
        y, mean, istd = cpu.batchnorm_fwd(x, self._gamma(), self._beta(), self.epsilon, self.training,
                                          self.running_mean, self.running_var, self.momentum, relu=do_relu,
                                          residual=res)
        self._cache[mb_id] = (x, y if do_relu else None, mean, istd, self.training)
        return y

    def forward_deferred(self, x, mb_id=0):
        """GPU: statistics now, the apply deferred into the consumer (:class:`hip.BnDeferred`,
        fused by a residual block's tail BatchNorm). The backward is the plain one: it needs
        only this layer's input and statistics, which the consumer's kernel saves."""
        from ...ops import hip
        x = self._to_layer_device(x)
        xa = hip.to_act(x, self.compute_dtype)
        C = self.num_features
        if self.training:
            part = getattr(x, "_bn_partial", None)
            # raw statistics rows: the consumer reduces them together with its own
            sums = hip.bn_stats_raw(xa, part)
            mean = _arena_empty((C,), torch.float32, xa.device)
            istd = _arena_empty((C,), torch.float32, xa.device)
            d = hip.BnDeferred(xa, sums, xa.numel() // C, self._gamma(), self._beta(), self.epsilon, (mean, istd),
                               (self.running_mean, self.running_var), self.momentum, False)
        else:
            mean = self.running_mean
            istd = torch.rsqrt(self.running_var + self.epsilon)
            d = hip.BnDeferred(xa, None, 1, self._gamma(), self._beta(), self.epsilon, None,
                               (self.running_mean, self.running_var), self.momentum, True)
        self._cache[mb_id] = (xa, None, mean, istd, self.training)
        return d

    def backward(self, grad, mb_id=0):
        ent = self._cache.pop(mb_id, None)
        if ent is None:
            raise RuntimeError(f"BatchNorm '{self.name}': no cached data for micro-batch {mb_id}")
        x, yout, mean, istd, was_training = ent
        grad = grad.to(x.device)
        dg = self._grads[0].view(-1) if self.affine else None
        db = self._grads[1].view(-1) if self.affine else None
        if x.is_cuda:
            from ...ops import hip
            pre = getattr(grad, "_bnb", None)
            if pre is not None and pre[0] is self and isinstance(pre[1], str) and pre[1] == "done":
                # data gradient (and dgamma / dbeta) already produced by a residual block's paired
                # backward (hip.bn_bwd_apply_dual); the incoming gradient is the masked one
                if self.emit_masked_grad:
                    self._last_masked[mb_id] = grad
                return pre[2]
            fused = pre[1:] if (pre is not None and pre[0] is self) else None
            if yout is _POOLED:
                if fused is None:
                    raise RuntimeError(f"BatchNorm '{self.name}': forward fused the max-pool, so the backward "
                                       "needs the fused max-pool backward statistics")
                yout = None
            g = hip.to_act(grad, self.compute_dtype)
            dx, dmask = hip.bn_backward(g, x, yout, mean, istd, self._gamma(), dg, db,
                                        want_masked=self.emit_masked_grad, eval_mode=not was_training,
                                        fused=fused)
            if self.emit_masked_grad:
                self._last_masked[mb_id] = dmask if dmask is not None else g
            return dx
        from ...ops import cpu
        dx, masked = cpu.batchnorm_bwd(x, grad.to(x.dtype), yout, mean, istd, self._gamma(), dg, db,
                                       training=was_training, want_masked=self.emit_masked_grad)
        if self.emit_masked_grad:
            self._last_masked[mb_id] = masked
        return dx

    def bwd_bn_spec(self, mb_id=0):
        ent = self._cache.get(mb_id)
        if ent is None:
            return None
        x, yout, mean, istd, was_training = ent
        # (fp32: only the exact-fp32 halo data gradient honours the request; every other producer
        # ignores it and the BatchNorm runs its own statistics pass)
        if not (was_training and x.is_cuda and x.dtype in (torch.bfloat16, torch.float32)
                and x.is_contiguous(memory_format=torch.channels_last)):
            return None
        from ...ops.hip import BnbRequest
        if yout is _POOLED:  # only the max-pool's fused backward can honour this request
            return BnbRequest(self, None, x, mean, istd, pooled=True)
        return BnbRequest(self, yout, x, mean, istd)

    def pop_masked_grad(self, mb_id=0):
        return self._last_masked.pop(mb_id)

    def forward_flops(self, s):
        n = 1
        for d in s:
            n *= d
        return 6 * n  # stats (2) + normalize (2) + affine (2)

    def backward_flops(self, s):
        n = 1
        for d in s:
            n *= d
        return 9 * n

    def get_config(self):
        return LayerConfig(self.name, dict(num_features=self.num_features, epsilon=self.epsilon,
                                           momentum=self.momentum, affine=self.affine), self.type_name)

    @staticmethod
    def from_config(cfg):
        p = cfg.parameters
        return BatchNorm(p["num_features"], p.get("epsilon", 1e-5), p.get("momentum", 0.1), p.get("affine", True),
                         cfg.name or "batchnorm")

    def state_buffers(self):
        return {"running_mean": self.running_mean, "running_var": self.running_var}


class GroupNorm(ParameterizedLayer):
    type_name = "groupnorm"

    def __init__(self, num_groups: int, num_channels: int, epsilon: float = 1e-5, affine: bool = True,
                 name: str = "groupnorm"):
        super().__init__(name)
        self.num_groups = int(num_groups)
        self.num_channels = int(num_channels)
        if self.num_channels % self.num_groups:
            raise ValueError("num_channels must be divisible by num_groups")
        self.epsilon = float(epsilon)
        self.affine = bool(affine)

    def param_specs(self):
        if not self.affine:
            return []
        return [ParamSpec("gamma", (self.num_channels, 1, 1, 1)), ParamSpec("beta", (self.num_channels, 1, 1, 1))]

    def init_values(self, gen):
        if not self.affine:
            return []
        return [torch.ones((self.num_channels, 1, 1, 1)), torch.zeros((self.num_channels, 1, 1, 1))]

    def has_parameters(self):
        return self.affine

    def forward(self, x, mb_id=0):
        x = self._to_layer_device(x)
        G = self.num_groups
        gamma = self._params[0].view(-1) if self.affine else None
        beta = self._params[1].view(-1) if self.affine else None
        if x.is_cuda:
            from ...ops import hip
            xa = hip.to_act(x, self.compute_dtype)
            y, mean, istd = hip.gn_fwd(xa, G, gamma, beta, self.epsilon)
            self._cache[mb_id] = (xa, mean, istd)
            return y
        from ...ops import cpu
        y, mean, istd = cpu.groupnorm_fwd(x, G, gamma, beta, self.epsilon)
        self._cache[mb_id] = (x, mean, istd)
        return y

    def backward(self, grad, mb_id=0):
        ent = self._cache.pop(mb_id, None)
        if ent is None:
            raise RuntimeError(f"GroupNorm '{self.name}': no cached data for micro-batch {mb_id}")
        x, mean, istd = ent
        G = self.num_groups
        gamma = self._params[0].view(-1) if self.affine else None
        dg = self._grads[0].view(-1) if self.affine else None
        db = self._grads[1].view(-1) if self.affine else None
        if x.is_cuda:
            from ...ops import hip
            g = hip.to_act(grad.to(x.device), self.compute_dtype)
            return hip.gn_bwd(g, x, G, gamma, mean, istd, dg, db)
        from ...ops import cpu
        return cpu.groupnorm_bwd(x, grad.to(x.dtype), G, gamma, mean, istd, dg, db)

    def forward_flops(self, s):
        n = 1
        for d in s:
            n *= d
        return 6 * n

    def backward_flops(self, s):
        n = 1
        for d in s:
            n *= d
        return 9 * n

    def get_config(self):
        return LayerConfig(self.name, dict(num_groups=self.num_groups, num_channels=self.num_channels,
                                           epsilon=self.epsilon, affine=self.affine), self.type_name)

    @staticmethod
    def from_config(cfg):
        p = cfg.parameters
        return GroupNorm(int(p["num_groups"]), p["num_channels"], p.get("epsilon", 1e-5), p.get("affine", True),
                         cfg.name or "groupnorm")
