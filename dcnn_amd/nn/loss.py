"""Loss functions (reference `include/nn/loss.hpp:23-470`, `src/nn/loss_impl/*`).

Targets are one-hot ``[N, C, 1, 1]`` (or ``[N, C]``); integer class labels ``[N]`` are also
accepted. Loss = batch mean; gradient scaled by 1/N of the tensor given (1/(N*C) for the
regression losses) exactly as `src/nn/loss_impl/cpu/loss_ops.cpp`.

GPU: ``loss_and_grad`` is ONE fused HIP kernel (loss + gradient + correct count, device
scalars, no host sync — graph-capturable); CPU: the same fused pass in the native backend
(``ops/cpu.py``). The ATen formulas in ``_cpu_loss`` / ``_cpu_grad`` are the test oracle.
``compute_loss`` keeps the reference's host-scalar API (it synchronises, like the reference's
D2H copy).
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch

_ALIASES = {
    "crossentropy": "crossentropy", "ce": "crossentropy",
    "softmax_crossentropy": "softmax_crossentropy", "softmax_ce": "softmax_crossentropy",
    "logsoftmax_crossentropy": "logsoftmax_crossentropy", "logsoftmax_ce": "logsoftmax_crossentropy",
    "mse": "mse", "mean_squared_error": "mse",
    "mae": "mae", "mean_absolute_error": "mae",
    "huber": "huber",
}


class LossConfig(dict):
    def __init__(self, type: str, name: str = "", parameters: Optional[dict] = None):
        super().__init__(type=type, name=name or type, parameters=dict(parameters or {}))

    @property
    def type(self):
        return self["type"]


class Loss:
    kind = "softmax_crossentropy"

    def __init__(self, param: float = 0.0):
        self.param = param

    def name(self) -> str:
        return self.kind

    def get_config(self) -> LossConfig:
        return LossConfig(self.kind, self.kind, {"param": self.param})

    def clone(self):
        return type(self)(self.param) if self.param else type(self)()

    @staticmethod
    def _2d(t: torch.Tensor) -> torch.Tensor:
        return t.reshape(t.shape[0], -1)

    def _targets(self, pred2d, target) -> Tuple[Optional[torch.Tensor], Optional[torch.Tensor]]:
        if target.dtype in (torch.int64, torch.int32) and target.dim() == 1:
            return None, target.to(pred2d.device)
        return self._2d(target).to(pred2d.device), None

    # ---- fused device path
    def loss_and_grad(self, pred, target, want_grad: bool = True, grad_scale: float = 1.0):
        """(loss[1] device tensor, grad shaped like pred | None, correct[1] int32). The gradient is
        scaled by an extra ``grad_scale`` (data parallel folds its 1 / world average in here)."""
        p2 = self._2d(pred)
        if p2.is_cuda:
            from ..ops import hip
            t2, lab = self._targets(p2, target)
            loss, grad, correct = hip.loss_fused(p2, t2, lab, self.kind, self.param, want_grad, grad_scale)
            return loss, (grad.view(pred.shape) if grad is not None else None), correct
        from ..ops import cpu
        t2, lab = self._targets(p2, target)
        if p2.dtype not in (torch.float32, torch.float64):
            p2 = p2.float()
        loss, grad, correct = cpu.loss_fused(p2, t2, lab, self.kind, self.param, want_grad)
        if grad is not None and grad_scale != 1.0:
            grad.mul_(grad_scale)
        return loss, (grad.view(pred.shape) if grad is not None else None), correct

    # ---- reference API
    def compute_loss(self, pred, target) -> float:
        return float(self.loss_and_grad(pred, target, want_grad=False)[0].item())

    def compute_gradient(self, pred, target) -> torch.Tensor:
        return self.loss_and_grad(pred, target, want_grad=True)[1]

    # ---- CPU reference math (loss_ops.cpp)
    def _hot(self, t2):
        # first class whose target > 0.5
        m = t2 > 0.5
        has = m.any(1)
        idx = m.float().argmax(1)
        return idx, has

    def _cpu_loss(self, p, t):
        raise NotImplementedError

    def _cpu_grad(self, p, t):
        raise NotImplementedError


class CrossEntropyLoss(Loss):
    """CE on probabilities (epsilon-clamped); gradient (p - t)/N as loss_ops.cpp:39."""
    kind = "crossentropy"

    def __init__(self, epsilon: float = 1e-15):
        super().__init__(epsilon)

    def _cpu_loss(self, p, t):
        idx, has = self._hot(t)
        v = p.gather(1, idx.view(-1, 1)).view(-1).clamp(self.param, 1 - self.param)
        return torch.where(has, -torch.log(v), torch.zeros_like(v)).sum() / p.shape[0]

    def _cpu_grad(self, p, t):
        return (p - t) / p.shape[0]


class SoftmaxCrossEntropyLoss(Loss):
    kind = "softmax_crossentropy"

    def _cpu_loss(self, p, t):
        idx, has = self._hot(t)
        lse = torch.logsumexp(p.double(), 1)
        v = lse - p.double().gather(1, idx.view(-1, 1)).view(-1)
        return (torch.where(has, v, torch.zeros_like(v)).sum() / p.shape[0]).float()

    def _cpu_grad(self, p, t):
        return (torch.softmax(p.double(), 1).float() - t) / p.shape[0]


class LogSoftmaxCrossEntropyLoss(SoftmaxCrossEntropyLoss):
    kind = "logsoftmax_crossentropy"


class MSELoss(Loss):
    kind = "mse"

    def _cpu_loss(self, p, t):
        return ((p - t) ** 2).double().sum().float() / p.numel()

    def _cpu_grad(self, p, t):
        return 2.0 * (p - t) / p.numel()


class MAELoss(Loss):
    kind = "mae"

    def _cpu_loss(self, p, t):
        return (p - t).abs().double().sum().float() / p.numel()

    def _cpu_grad(self, p, t):
        d = p - t
        s = 1.0 / p.numel()
        return torch.where(d > 0, torch.full_like(d, s), torch.full_like(d, -s))


class HuberLoss(Loss):
    kind = "huber"

    def __init__(self, delta: float = 1.0):
        super().__init__(delta)

    def _cpu_loss(self, p, t):
        d = (p - t).abs()
        l = torch.where(d <= self.param, 0.5 * d * d, self.param * d - 0.5 * self.param ** 2)
        return l.double().sum().float() / p.numel()

    def _cpu_grad(self, p, t):
        d = p - t
        s = 1.0 / p.numel()
        return torch.where(d.abs() <= self.param, d * s, torch.sign(d) * self.param * s)


class LossFactory:
    @staticmethod
    def create(name: str, **kw) -> Loss:
        k = _ALIASES.get(name)
        if k is None:
            raise ValueError(f"Unknown loss type: {name}")
        if k == "crossentropy":
            return CrossEntropyLoss(kw.get("epsilon", 1e-15))
        if k == "softmax_crossentropy":
            return SoftmaxCrossEntropyLoss()
        if k == "logsoftmax_crossentropy":
            return LogSoftmaxCrossEntropyLoss()
        if k == "mse":
            return MSELoss()
        if k == "mae":
            return MAELoss()
        return HuberLoss(kw.get("delta", 1.0))

    @staticmethod
    def create_from_config(cfg) -> Loss:
        p = cfg.get("parameters", {})
        t = cfg["type"]
        if _ALIASES.get(t) == "crossentropy":
            return CrossEntropyLoss(p.get("param", p.get("epsilon", 1e-15)))
        if _ALIASES.get(t) == "huber":
            return HuberLoss(p.get("param", p.get("delta", 1.0)))
        return LossFactory.create(t)

    # reference-named helpers
    create_crossentropy = staticmethod(lambda epsilon=1e-15: CrossEntropyLoss(epsilon))
    create_softmax_crossentropy = staticmethod(lambda: SoftmaxCrossEntropyLoss())
    create_logsoftmax_crossentropy = staticmethod(lambda: LogSoftmaxCrossEntropyLoss())
    create_mse = staticmethod(lambda: MSELoss())
    create_mae = staticmethod(lambda: MAELoss())
    create_huber = staticmethod(lambda delta=1.0: HuberLoss(delta))
