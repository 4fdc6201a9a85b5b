"""Layer ABI (reference: `include/nn/layers_impl/base_layer.hpp:37-116`,
`parameterized_layer.hpp:17-31`, `stateless_layer.hpp:17`).

Every layer implements explicit ``forward(x, mb_id)`` / ``backward(grad, mb_id)`` with
per-micro-batch caches keyed by ``mb_id`` (so one layer object can hold several in-flight
micro-batches of a pipeline schedule). Two execution paths are chosen per call from the
tensor's device:

* CPU: the reference semantics in NCHW, fp32 (or fp64), on the native C++ backend
  (``ops/cpu.py`` over csrc/native/cpu_ops.cpp + the blocked GEMM); ATen is only the test oracle.
* GPU (MI355X): the HIP/CDNA4 kernel library, NHWC (channels_last) activations in the
  model's compute dtype (bf16 by default, fp32 accumulation / master weights).
"""
from __future__ import annotations

import copy
import random
import time
from typing import Any, Dict, List, Optional

import torch

from ...device import Device, get_cpu, get_device
from ..params import ParamArena, ParamSpec


class LayerConfig(dict):
    """``{name, parameters}`` with typed ``get`` (reference `LayerConfig`, base_layer.hpp:20)."""

    def __init__(self, name: str = "", parameters: Optional[Dict[str, Any]] = None, type: str = ""):
        super().__init__(name=name, parameters=dict(parameters or {}), type=type)

    @property
    def name(self) -> str:
        return self["name"]

    @property
    def parameters(self) -> Dict[str, Any]:
        return self["parameters"]

    def get(self, key, default=None):  # type: ignore[override]
        if key in ("name", "parameters", "type"):
            return super().get(key, default)
        return self["parameters"].get(key, default)


def run_backward(layers, i: int, grad, mb_id: int = 0):
    """``layers[i].backward(grad, mb_id)`` inside a layer chain, with the backward-BN fusion
    request of the layer that will consume its output (the nearest non-passthrough layer below
    it, see ``Layer.bwd_bn_spec``) attached for the duration of the call."""
    l = layers[i]
    req = None
    if l.needs_input_grad:
        j = i - 1
        while j >= 0 and layers[j].passthrough:
            j -= 1
        if j >= 0:
            req = layers[j].bwd_bn_spec(mb_id)
    l._bnb_request = req
    try:
        return l.backward(grad, mb_id)
    finally:
        l._bnb_request = None


class Layer:
    type_name = "layer"

    def __init__(self, name: str = ""):
        self.name = name
        self.training = True
        self.device: Device = get_cpu()
        self.compute_dtype = torch.float32
        self.use_seed = False
        self.seed = 0
        self.enable_profiling = False
        self.perf_timers: Dict[str, float] = {}
        self.needs_input_grad = True
        self.initialized = False
        self._cache: Dict[int, Any] = {}

    # ---------------------------------------------------------------- lifecycle / state
    def type(self) -> str:
        return self.type_name

    def initialize(self) -> None:
        self.initialized = True

    def set_seed(self, seed: int) -> None:
        self.use_seed = True
        self.seed = int(seed)

    def set_training(self, training: bool) -> None:
        self.training = bool(training)

    def is_training(self) -> bool:
        return self.training

    def set_device(self, device) -> None:
        self.device = get_device(device)

    def get_device(self) -> Device:
        return self.device

    def set_compute_dtype(self, dtype: torch.dtype) -> None:
        self.compute_dtype = dtype

    def clear_cache(self, mb_id: Optional[int] = None) -> None:
        if mb_id is None:
            self._cache.clear()
        else:
            self._cache.pop(mb_id, None)

    def cached_memory_bytes(self) -> int:
        total = 0

        def acc(v):
            nonlocal total
            if isinstance(v, torch.Tensor):
                total += v.numel() * v.element_size()
            elif isinstance(v, (list, tuple)):
                for e in v:
                    acc(e)
            elif isinstance(v, dict):
                for e in v.values():
                    acc(e)

        for v in self._cache.values():
            acc(v)
        return total

    def print_profiling_info(self) -> None:
        print(f"Profiling info for layer: {self.name}")
        for k, v in self.perf_timers.items():
            print(f"  {k}: {v} ms")

    def reset_profiling_info(self) -> None:
        self.perf_timers.clear()

    # ---------------------------------------------------------------- compute
    def forward(self, x: torch.Tensor, mb_id: int = 0) -> torch.Tensor:
        raise NotImplementedError

    def backward(self, grad: torch.Tensor, mb_id: int = 0) -> Optional[torch.Tensor]:
        raise NotImplementedError

    # ---------------------------------------------------------------- backward fusion hooks
    # A container asks the layer that will RECEIVE a gradient for a fusion request
    # (``bwd_bn_spec``) and hands it to the layer that PRODUCES that gradient via
    # ``_bnb_request`` for the duration of its backward call (see ``run_backward``).
    _bnb_request = None
    passthrough = False

    def bwd_bn_spec(self, mb_id: int = 0):
        """``ops.hip.BnbRequest`` when this layer's backward starts with a BatchNorm whose ReLU mask
        and statistics the gradient's producer may fuse into its epilogue; None otherwise."""
        return None

    def _on_gpu(self) -> bool:
        return self.device.is_gpu()

    def _to_layer_device(self, x: torch.Tensor) -> torch.Tensor:
        """Reference semantics: inputs are moved to the layer's device (conv2d_layer.tpp:100)."""
        td = self.device.torch_device
        if x.device != td:
            x = x.to(td, non_blocking=True)
        if not self._on_gpu() and x.dtype != self.compute_dtype:
            x = x.to(self.compute_dtype)
        return x

    # ---------------------------------------------------------------- params
    def parameters(self) -> List[torch.Tensor]:
        return []

    def gradients(self) -> List[torch.Tensor]:
        return []

    def has_parameters(self) -> bool:
        return False

    def param_specs(self) -> List[ParamSpec]:
        return []

    def clear_gradients(self) -> None:
        for g in self.gradients():
            g.zero_()

    # ---------------------------------------------------------------- shapes / cost
    def compute_output_shape(self, input_shape: List[int]) -> List[int]:
        return list(input_shape)

    def forward_flops(self, input_shape: List[int]) -> int:
        return 0

    def backward_flops(self, input_shape: List[int]) -> int:
        return 0

    def forward_complexity(self, input_shape: List[int]) -> int:
        return min(self.forward_flops(input_shape), 0xFFFFFFFF)

    def backward_complexity(self, input_shape: List[int]) -> int:
        return min(self.backward_flops(input_shape), 0xFFFFFFFF)

    # ---------------------------------------------------------------- config
    def get_config(self) -> LayerConfig:
        return LayerConfig(self.name, {}, self.type_name)

    def clone(self) -> "Layer":
        from ..layers import create_layer
        c = create_layer(self.type_name, self.get_config())
        c.training = self.training
        if self.use_seed:
            c.set_seed(self.seed)
        return c


class StatelessLayer(Layer):
    pass


class ParameterizedLayer(Layer):
    """Parameters live in a :class:`ParamArena` (own arena when used standalone, the model's
    arena when part of a Sequential)."""

    def __init__(self, name: str = ""):
        super().__init__(name)
        self._params: List[torch.Tensor] = []
        self._grads: List[torch.Tensor] = []
        self._shadows: List[Optional[torch.Tensor]] = []
        self.arena: Optional[ParamArena] = None

    def has_parameters(self) -> bool:
        return True

    def init_values(self, gen: torch.Generator) -> List[torch.Tensor]:
        raise NotImplementedError

    def make_generator(self) -> torch.Generator:
        g = torch.Generator(device="cpu")
        g.manual_seed(self.seed if self.use_seed else (time.time_ns() ^ random.getrandbits(48)) & ((1 << 63) - 1))
        return g

    def bind(self, arena: ParamArena, indices: List[int]) -> None:
        self.arena = arena
        self._params = [arena.param(i) for i in indices]
        self._grads = [arena.grad_view(i) for i in indices]
        self._shadows = [arena.shadow_view(i) for i in indices]
        self._on_bind()
        self.initialized = True

    def _on_bind(self) -> None:
        pass

    def shadow_dtype(self) -> Optional[torch.dtype]:
        return torch.bfloat16 if (self._on_gpu() and self.compute_dtype == torch.bfloat16) else None

    def master_dtype(self) -> torch.dtype:
        return torch.float64 if (not self._on_gpu() and self.compute_dtype == torch.float64) else torch.float32

    def initialize(self) -> None:
        if self.initialized and self.arena is not None:
            return
        specs = self.param_specs()
        arena = ParamArena(specs, self.device.torch_device, self.shadow_dtype(), self.master_dtype())
        vals = self.init_values(self.make_generator())
        for i, v in enumerate(vals):
            arena.param(i).copy_(v)
        arena.sync_shadow(force=True)
        self.bind(arena, list(range(len(specs))))

    def parameters(self) -> List[torch.Tensor]:
        return list(self._params)

    def gradients(self) -> List[torch.Tensor]:
        return list(self._grads)

    def set_device(self, device) -> None:
        new = get_device(device)
        if self.initialized and self.arena is not None and new != self.device:
            old_vals = [p.detach().to("cpu").clone() for p in self._params]
            self.device = new
            self.initialized = False
            self.arena = None
            specs = self.param_specs()
            arena = ParamArena(specs, new.torch_device, self.shadow_dtype(), self.master_dtype())
            for i, v in enumerate(old_vals):
                arena.param(i).copy_(v)
            arena.sync_shadow(force=True)
            self.bind(arena, list(range(len(specs))))
            self._move_buffers(new)
        else:
            self.device = new
            self._move_buffers(new)

    def _move_buffers(self, device: Device) -> None:
        pass

    def weight_operand(self, i: int = 0) -> torch.Tensor:
        """bf16 shadow of parameter i for the MFMA kernels (refreshed if the master changed)."""
        if self.arena is not None:
            self.arena.sync_shadow()
        s = self._shadows[i]
        return s if s is not None else self._params[i]
