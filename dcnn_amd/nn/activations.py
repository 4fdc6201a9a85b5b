"""Activation functions + factory (reference `include/nn/activations.hpp:27-64`,
`include/nn/activations_impl/*`): relu, leaky_relu(0.01), elu(1.0), sigmoid, tanh,
softmax (over the channel dim per spatial location), linear; "none" -> None.

Each function has a CPU (native C++ backend, csrc/native/cpu_ops.cpp) and a GPU (HIP kernel)
implementation of ``apply(x)`` and ``gradient(x, y, grad)`` (x = input, y = output); the ATen
formulas kept in ``_cpu`` / ``_cpu_grad`` are the test oracle.
"""
from __future__ import annotations

from typing import Callable, Dict, List, Optional

import torch


class ActivationFunction:
    name_str = "linear"

    def __init__(self, alpha: float = 0.0):
        self.alpha = alpha

    def name(self) -> str:
        return self.name_str

    def apply(self, x: torch.Tensor) -> torch.Tensor:
        if x.is_cuda:
            from ..ops import hip
            return hip.act_fwd(x, self.name_str, self.alpha)
        from ..ops import cpu
        return cpu.act_fwd(x, self.name_str, self.alpha)

    def gradient(self, x: torch.Tensor, y: torch.Tensor, grad: torch.Tensor) -> torch.Tensor:
        if x.is_cuda:
            from ..ops import hip
            return hip.act_bwd(x, grad, self.name_str, self.alpha)
        from ..ops import cpu
        return cpu.act_bwd(x, grad.to(x.dtype), self.name_str, self.alpha)

    def _cpu(self, x):
        return x.clone()

    def _cpu_grad(self, x, y, g):
        return g.clone()


class ReLU(ActivationFunction):
    name_str = "relu"

    def _cpu(self, x):
        return torch.relu(x)

    def _cpu_grad(self, x, y, g):
        return g * (x > 0)


class LeakyReLU(ActivationFunction):
    name_str = "leaky_relu"

    def __init__(self, negative_slope: float = 0.01):
        super().__init__(negative_slope)

    def _cpu(self, x):
        return torch.where(x > 0, x, x * self.alpha)

    def _cpu_grad(self, x, y, g):
        return torch.where(x > 0, g, g * self.alpha)


class ELU(ActivationFunction):
    name_str = "elu"

    def __init__(self, alpha: float = 1.0):
        super().__init__(alpha)

    def _cpu(self, x):
        return torch.where(x > 0, x, self.alpha * (torch.exp(x) - 1))

    def _cpu_grad(self, x, y, g):
        return torch.where(x > 0, g, g * self.alpha * torch.exp(x))


class Sigmoid(ActivationFunction):
    name_str = "sigmoid"

    def _cpu(self, x):
        return torch.sigmoid(x)

    def _cpu_grad(self, x, y, g):
        s = torch.sigmoid(x)
        return g * s * (1 - s)


class Tanh(ActivationFunction):
    name_str = "tanh"

    def _cpu(self, x):
        return torch.tanh(x)

    def _cpu_grad(self, x, y, g):
        t = torch.tanh(x)
        return g * (1 - t * t)


class Linear(ActivationFunction):
    name_str = "linear"

    def apply(self, x):
        return x

    def gradient(self, x, y, grad):
        return grad


class Softmax(ActivationFunction):
    """Softmax over channels for every (n, h, w) (`softmax.tpp:19-75`)."""
    name_str = "softmax"

    def apply(self, x):
        if x.is_cuda:
            from ..ops import hip
            return hip.softmax_channels(x)
        from ..ops import cpu
        return cpu.softmax_channels(x)

    def gradient(self, x, y, grad):
        if x.is_cuda:
            from ..ops import hip
            return hip.softmax_channels_bwd(y, grad)
        from ..ops import cpu
        return cpu.softmax_channels_bwd(y, grad.to(y.dtype))


class ActivationFactory:
    _creators: Dict[str, Callable[[], Optional[ActivationFunction]]] = {}

    @classmethod
    def register_activation(cls, name: str, creator: Callable[[], Optional[ActivationFunction]]) -> None:
        cls._creators[name] = creator

    @classmethod
    def register_defaults(cls) -> None:
        cls.register_activation("none", lambda: None)
        cls.register_activation("relu", ReLU)
        cls.register_activation("leaky_relu", lambda: LeakyReLU(0.01))
        cls.register_activation("sigmoid", Sigmoid)
        cls.register_activation("softmax", Softmax)
        cls.register_activation("linear", Linear)
        cls.register_activation("tanh", Tanh)
        cls.register_activation("elu", lambda: ELU(1.0))

    @classmethod
    def create(cls, name: str) -> Optional[ActivationFunction]:
        if not cls._creators:
            cls.register_defaults()
        if name not in cls._creators:
            raise ValueError(f"Unknown activation function: {name}")
        return cls._creators[name]()

    @classmethod
    def get_available_activations(cls) -> List[str]:
        if not cls._creators:
            cls.register_defaults()
        return list(cls._creators)


ActivationFactory.register_defaults()
