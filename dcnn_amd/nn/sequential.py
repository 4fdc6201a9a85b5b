"""Sequential model container + SequentialBuilder (reference `include/nn/sequential.hpp:32-1340`).

Same API and file formats as the reference:
  * ``save_to_file(path)`` -> ``path.json`` (architecture) + ``path.bin`` (for every parameter in
    layer order: uint64 shape[4] little-endian + float32 data, NCHW / {Cout,Cin,KH,KW});
  * ``from_file``, ``load_weights_file``, ``get_config`` / ``load_from_config``, ``split``.
MI355X-specific underneath:
  * all parameters of the model live in ONE :class:`ParamArena` (flat fp32 master + grad +
    bf16 shadow), so clear_gradients is one memset and the optimizer one kernel;
  * GPU compute dtype defaults to bf16 (fp32 accumulation/master weights);
  * a fusion planner wires conv->BN statistics, BN->ReLU and residual tails (GPU only);
  * profiling uses HIP events per layer (device time), not host wall-clock around async
    launches (reference §5.1 measured launch time only);
  * extended checkpoint sidecar ``path.state`` (BN running stats, optional optimizer state)
    fixes reference gap G11.
"""
from __future__ import annotations

import io
import json
import os
import struct
import time
from collections import OrderedDict
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

from ..device import Device, DeviceType, get_cpu, get_device
from .layers import (Activation, AvgPool2D, BatchNorm, Conv2D, Dense, Dropout, Flatten, GroupNorm, Layer,
                     LayerBuilder, LayerConfig, LayerFactory, MaxPool2D, ParameterizedLayer, ResidualBlock,
                     create_layer, plan_fusion)
from .layers.base import run_backward
from .params import ParamArena


class Partition:
    def __init__(self, start_layer: int, end_layer: int):
        self.start_layer = int(start_layer)
        self.end_layer = int(end_layer)  # exclusive

    def __repr__(self):
        return f"Partition({self.start_layer}, {self.end_layer})"

    def __eq__(self, o):
        return isinstance(o, Partition) and (o.start_layer, o.end_layer) == (self.start_layer, self.end_layer)


def _leaf_param_layers(layers: Sequence[Layer]) -> List[ParameterizedLayer]:
    out = []
    for l in layers:
        if isinstance(l, ResidualBlock):
            out.extend(_leaf_param_layers(l.sublayers()))
        elif isinstance(l, ParameterizedLayer):
            out.append(l)
    return out


def _all_layers(layers: Sequence[Layer]) -> List[Layer]:
    out = []
    for l in layers:
        out.append(l)
        if isinstance(l, ResidualBlock):
            out.extend(_all_layers(l.sublayers()))
    return out


def save_tensor(f, t: torch.Tensor) -> None:
    """Reference `Tensor::save` (tensor.hpp:625): size_t shape[4] + raw fp32 NCHW data."""
    c = t.detach().to("cpu", torch.float32).contiguous()
    shape = list(c.shape) + [1] * (4 - c.dim())
    f.write(struct.pack("<4Q", *shape[:4]))
    f.write(c.numpy().tobytes())


def load_tensor(f) -> torch.Tensor:
    hdr = f.read(32)
    if len(hdr) != 32:
        raise RuntimeError("Failed to read tensor shape from file")
    shape = struct.unpack("<4Q", hdr)
    n = int(np.prod(shape))
    buf = f.read(4 * n)
    if len(buf) != 4 * n:
        raise RuntimeError("Failed to read tensor data from file")
    return torch.from_numpy(np.frombuffer(buf, dtype="<f4").copy()).view(*shape)


class Sequential:
    def __init__(self, name: str = "sequential"):
        self.name_ = name
        self.layers: List[Layer] = []
        self.training = True
        self.device: Device = get_cpu()
        self.compute_dtype = torch.float32
        self.dtype_pref: Optional[torch.dtype] = None  # None: bf16 on GPU, fp32 on CPU
        self.arena: Optional[ParamArena] = None
        self.initialized = False
        self.enable_profiling_ = False
        self.forward_times_us: Dict[str, float] = OrderedDict()
        self.backward_times_us: Dict[str, float] = OrderedDict()
        self._pending_events = []
        self._seed: Optional[int] = None
        self.first_layer_input_grad = True

    # ------------------------------------------------------------------ structure
    def name(self) -> str:
        return self.name_

    def set_name(self, n: str) -> None:
        self.name_ = n

    def add(self, layer: Layer) -> "Sequential":
        layer.set_training(self.training)
        self.layers.append(layer)
        self.initialized = False
        return self

    def insert(self, index: int, layer: Layer) -> None:
        self.layers.insert(index, layer)
        self.initialized = False

    def remove(self, index: int) -> None:
        del self.layers[index]
        self.initialized = False

    def layer_size(self) -> int:
        return len(self.layers)

    def size(self) -> int:
        return len(self.layers)

    def __len__(self):
        return len(self.layers)

    def __getitem__(self, i) -> Layer:
        return self.layers[i]

    def get_layers(self) -> List[Layer]:
        return list(self.layers)

    # ------------------------------------------------------------------ mode / device
    def set_training(self, training: bool) -> None:
        self.training = bool(training)
        for l in self.layers:
            l.set_training(training)

    def train(self):
        self.set_training(True)

    def eval(self):
        self.set_training(False)

    def is_training(self) -> bool:
        return self.training

    def set_seed(self, seed: int) -> None:
        self._seed = int(seed)
        for i, l in enumerate(self.layers):
            l.set_seed(self._seed * 1000003 + i)

    def set_device(self, device) -> None:
        if isinstance(device, DeviceType):
            device = get_device(device)
        dev = get_device(device)
        was_init = self.initialized
        vals = None
        bufs = None
        if was_init:
            vals = [p.detach().to("cpu").clone() for p in self.parameters()]
            bufs = self._collect_buffers()
        self.device = dev
        if dev.is_gpu():
            pref = self.dtype_pref if self.dtype_pref in (torch.float32, torch.bfloat16) else None
            self.compute_dtype = pref or torch.bfloat16
        else:
            self.compute_dtype = torch.float64 if self.dtype_pref == torch.float64 else torch.float32
        for l in _all_layers(self.layers):
            l.device = dev
            l.set_compute_dtype(self.compute_dtype)
        if was_init:
            self.initialized = False
            self._build_arena(init_values=False)
            for p, v in zip(self.parameters(), vals):
                p.copy_(v)
            self.arena.sync_shadow(force=True)
            self._restore_buffers(bufs)
        self._plan()

    def set_compute_dtype(self, dtype: torch.dtype) -> None:
        """GPU: bfloat16 (default) or float32. CPU: float32 (default) or float64 — the native
        backend's double-precision path (reference dkernels.cpp / dgemm.cpp)."""
        ok = (torch.float32, torch.bfloat16) if self.device.is_gpu() else (torch.float32, torch.float64)
        if dtype not in ok:
            raise ValueError(f"compute dtype on {'GPU' if self.device.is_gpu() else 'CPU'} must be one of {ok}")
        self.dtype_pref = dtype
        self.compute_dtype = dtype
        for l in _all_layers(self.layers):
            l.set_compute_dtype(dtype)
        if self.initialized:
            self.set_device(self.device)

    def get_device(self) -> Device:
        return self.device

    def _plan(self) -> None:
        on_gpu = self.device.is_gpu()
        plan_fusion(self.layers, on_gpu)
        for l in self.layers:
            if isinstance(l, ResidualBlock):
                l._plan()
        for l in self.layers:
            l.needs_input_grad = True
        if self.layers:
            self.layers[0].needs_input_grad = self.first_layer_input_grad
            if isinstance(self.layers[0], ResidualBlock):
                self.layers[0]._plan()
        self._transposer = None
        if on_gpu and self.initialized and self.compute_dtype in (torch.bfloat16, torch.float32):
            from ..ops.hip import WeightTransposer
            convs = [l for l in _all_layers(self.layers) if isinstance(l, Conv2D)]
            if convs:
                self._transposer = WeightTransposer(convs, self.compute_dtype)

    def prepare_backward(self) -> None:
        """Per-step setup of the backward pass: all dgrad weight operands in one launch, and the
        split-K weight-gradient reductions queued for one batched launch (ops.hip.grad_reducer)."""
        if getattr(self, "_transposer", None) is not None:
            self._transposer.run()
        if self.device.is_gpu():
            from ..ops.hip import grad_reducer
            grad_reducer.begin()

    def flush_gradients(self) -> None:
        """Complete every queued weight-gradient reduction (before a gradient is consumed
        mid-backward, e.g. a data-parallel bucket all-reduce)."""
        if self.device.is_gpu():
            from ..ops.hip import grad_reducer
            grad_reducer.flush()

    def finish_backward(self) -> None:
        if getattr(self, "_transposer", None) is not None:
            self._transposer.invalidate()
        if self.device.is_gpu():
            from ..ops.hip import grad_reducer
            grad_reducer.end()

    def set_first_layer_input_grad(self, need: bool) -> None:
        """Skip the (unused) input gradient of the first layer (reference G9 wasted it)."""
        self.first_layer_input_grad = bool(need)
        self._plan()

    # ------------------------------------------------------------------ params
    def _build_arena(self, init_values: bool = True) -> None:
        leaves = _leaf_param_layers(self.layers)
        specs, owners = [], []
        for l in leaves:
            for s in l.param_specs():
                specs.append(s)
                owners.append(l)
        shadow = torch.bfloat16 if (self.device.is_gpu() and self.compute_dtype == torch.bfloat16) else None
        adt = torch.float64 if self.compute_dtype == torch.float64 else torch.float32
        self.arena = ParamArena(specs, self.device.torch_device, shadow, adt)
        idx = 0
        for l in leaves:
            n = len(l.param_specs())
            l.device = self.device
            if init_values:
                vals = l.init_values(l.make_generator())
                for j, v in enumerate(vals):
                    self.arena.param(idx + j).copy_(v)
            l.bind(self.arena, list(range(idx, idx + n)))
            idx += n
        for l in _all_layers(self.layers):
            if isinstance(l, BatchNorm):
                l._move_buffers(self.device)
            l.initialized = True
        self.arena.sync_shadow(force=True)
        self.initialized = True

    def initialize(self) -> None:
        if self.initialized:
            return
        for l in _all_layers(self.layers):
            l.device = self.device
            l.set_compute_dtype(self.compute_dtype)
        self._build_arena(init_values=True)
        self._plan()

    def parameters(self, part: Optional[Partition] = None) -> List[torch.Tensor]:
        layers = self.layers if part is None else self.layers[part.start_layer:part.end_layer]
        return [p for l in layers for p in l.parameters()]

    def gradients(self, part: Optional[Partition] = None) -> List[torch.Tensor]:
        layers = self.layers if part is None else self.layers[part.start_layer:part.end_layer]
        return [g for l in layers for g in l.gradients()]

    def clear_gradients(self) -> None:
        if self.arena is not None:
            self.arena.zero_grad()

    def num_parameters(self) -> int:
        return sum(p.numel() for p in self.parameters())

    def load_parameters(self, params: List[torch.Tensor]) -> None:
        mine = self.parameters()
        if len(params) != len(mine):
            raise RuntimeError(f"Parameter count mismatch: expected {len(mine)} but got {len(params)}")
        for i, (p, v) in enumerate(zip(mine, params)):
            if tuple(p.shape) != tuple(v.shape):
                raise RuntimeError(f"Parameter shape mismatch at index {i}: {tuple(p.shape)} vs {tuple(v.shape)}")
            p.copy_(v)
        if self.arena is not None:
            self.arena.sync_shadow(force=True)

    def _collect_buffers(self) -> Dict[str, torch.Tensor]:
        out = {}
        for l in _all_layers(self.layers):
            if isinstance(l, BatchNorm):
                out[f"{id(l)}"] = (l.running_mean.detach().cpu().clone(), l.running_var.detach().cpu().clone())
        return out

    def _restore_buffers(self, bufs):
        for l in _all_layers(self.layers):
            if isinstance(l, BatchNorm) and f"{id(l)}" in bufs:
                m, v = bufs[f"{id(l)}"]
                l.running_mean = m.to(self.device.torch_device)
                l.running_var = v.to(self.device.torch_device)

    # ------------------------------------------------------------------ compute
    def _prof_begin(self):
        if not self.enable_profiling_:
            return None
        if self.device.is_gpu():
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            return e
        return time.perf_counter()

    def _prof_end(self, key, start, table):
        if start is None:
            return
        if self.device.is_gpu():
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            self._pending_events.append((table, key, start, e))
        else:
            table[key] = table.get(key, 0.0) + (time.perf_counter() - start) * 1e6

    def _resolve_events(self):
        if not self._pending_events:
            return
        torch.cuda.synchronize(self.device.torch_device)
        for table, key, s, e in self._pending_events:
            table[key] = table.get(key, 0.0) + s.elapsed_time(e) * 1000.0
        self._pending_events.clear()

    def forward(self, x: torch.Tensor, mb_id: int = 0, return_on_input_device: bool = True) -> torch.Tensor:
        if not self.layers:
            raise RuntimeError("Cannot forward through empty sequential model")
        if not self.initialized:
            self.initialize()
        in_dev = x.device
        cur = x.to(self.device.torch_device, non_blocking=True) if x.device != self.device.torch_device else x
        for i, l in enumerate(self.layers):
            t0 = self._prof_begin()
            try:
                cur = l.forward(cur, mb_id)
            except Exception as e:
                raise RuntimeError(f"Error while forward in layer {i} ({l.name}): {e}") from e
            self._prof_end(l.name or l.type(), t0, self.forward_times_us)
        if return_on_input_device and cur.device != in_dev:
            cur = cur.to(in_dev).float()
            if cur.dim() == 4:
                cur = cur.contiguous()
        return cur

    __call__ = forward

    def backward(self, grad: torch.Tensor, mb_id: int = 0, return_on_input_device: bool = True):
        if not self.layers:
            raise RuntimeError("Cannot backward through empty sequential model")
        g_dev = grad.device
        cur = grad.to(self.device.torch_device) if grad.device != self.device.torch_device else grad
        self.prepare_backward()
        for i in range(len(self.layers) - 1, -1, -1):
            l = self.layers[i]
            t0 = self._prof_begin()
            try:
                cur = run_backward(self.layers, i, cur, mb_id)
            except Exception as e:
                raise RuntimeError(f"Error in backward pass of layer {i} ({l.type()}): {e}") from e
            self._prof_end(l.name or l.type(), t0, self.backward_times_us)
        self.finish_backward()
        if cur is not None and return_on_input_device and cur.device != g_dev:
            cur = cur.to(g_dev).float().contiguous()
        return cur

    def clear_cache(self, mb_id: Optional[int] = None) -> None:
        for l in self.layers:
            l.clear_cache(mb_id)

    # ------------------------------------------------------------------ shapes / cost
    def compute_output_shape(self, input_shape: List[int]) -> List[int]:
        s = list(input_shape)
        for l in self.layers:
            s = l.compute_output_shape(s)
        return s

    def _complexities(self, input_shape, fwd, part=None):
        layers = self.layers if part is None else self.layers[part.start_layer:part.end_layer]
        s = list(input_shape)
        if part is not None:
            for l in self.layers[:part.start_layer]:
                s = l.compute_output_shape(s)
        out = []
        for l in layers:
            out.append(l.forward_complexity(s) if fwd else l.backward_complexity(s))
            s = l.compute_output_shape(s)
        return out

    def forward_complexity(self, input_shape, part=None) -> List[int]:
        return self._complexities(input_shape, True, part)

    def backward_complexity(self, input_shape, part=None) -> List[int]:
        return self._complexities(input_shape, False, part)

    def forward_flops(self, input_shape) -> int:
        s, total = list(input_shape), 0
        for l in self.layers:
            total += l.forward_flops(s)
            s = l.compute_output_shape(s)
        return total

    def backward_flops(self, input_shape) -> int:
        s, total = list(input_shape), 0
        for l in self.layers:
            total += l.backward_flops(s)
            s = l.compute_output_shape(s)
        return total

    # ------------------------------------------------------------------ reporting
    def print_summary(self, input_shape: List[int]) -> str:
        lines = ["=" * 75, f"Model Summary: {self.name_}", "=" * 75,
                 f"{'Layer (Type)':<22}{'Input Shape':<20}{'Output Shape':<20}{'Fwd FLOPs':>14}{'Bwd FLOPs':>14}"]
        s = list(input_shape)
        for l in self.layers:
            o = l.compute_output_shape(s)
            lines.append(f"{(l.name or l.type())[:21]:<22}{str(tuple(s)):<20}{str(tuple(o)):<20}"
                         f"{l.forward_flops(s):>14}{l.backward_flops(s):>14}")
            s = o
        lines.append("-" * 75)
        n = sum(p.numel() for p in self.parameters()) if self.initialized else None
        if n is not None:
            lines.append(f"Parameters: {n}")
        txt = "\n".join(lines)
        print(txt)
        return txt

    def enable_profiling(self, enable: bool = True) -> None:
        self.enable_profiling_ = bool(enable)
        for l in _all_layers(self.layers):
            l.enable_profiling = bool(enable)

    def get_forward_times(self) -> Dict[str, float]:
        self._resolve_events()
        return dict(self.forward_times_us)

    def get_backward_times(self) -> Dict[str, float]:
        self._resolve_events()
        return dict(self.backward_times_us)

    def clear_profiling_data(self) -> None:
        self._pending_events.clear()
        self.forward_times_us.clear()
        self.backward_times_us.clear()

    def print_profiling_summary(self) -> str:
        f, b = self.get_forward_times(), self.get_backward_times()
        keys = list(OrderedDict.fromkeys(list(f) + list(b)))
        lines = ["=" * 60, f"Profiling summary ({'HIP events, device time' if self.device.is_gpu() else 'host time'})",
                 f"{'Layer':<28}{'Forward (ms)':>15}{'Backward (ms)':>15}", "-" * 60]
        tf = tb = 0.0
        for k in keys:
            a, c = f.get(k, 0.0) / 1000, b.get(k, 0.0) / 1000
            tf += a
            tb += c
            lines.append(f"{k[:27]:<28}{a:>15.3f}{c:>15.3f}")
        lines += ["-" * 60, f"{'TOTAL':<28}{tf:>15.3f}{tb:>15.3f}"]
        txt = "\n".join(lines)
        print(txt)
        return txt

    def print_cache_memory_summary(self) -> str:
        lines = [f"{'Layer':<28}{'Cached MB':>12}"]
        tot = 0
        for l in self.layers:
            b = l.cached_memory_bytes()
            tot += b
            lines.append(f"{(l.name or l.type())[:27]:<28}{b / 2**20:>12.3f}")
        lines.append(f"{'TOTAL':<28}{tot / 2**20:>12.3f}")
        txt = "\n".join(lines)
        print(txt)
        return txt

    # ------------------------------------------------------------------ config / io
    def get_config(self, part: Optional[Partition] = None) -> dict:
        if part is not None:
            if not (0 <= part.start_layer < part.end_layer <= len(self.layers)):
                raise IndexError("Partition indices out of range")
            layers = self.layers[part.start_layer:part.end_layer]
            name = f"{self.name_}_part_{part.start_layer}_{part.end_layer}"
        else:
            layers, name = self.layers, self.name_
        return {"name": name, "is_training": self.training,
                "layers": [{"type": l.type(), "name": l.get_config().name, "parameters": l.get_config().parameters}
                           for l in layers]}

    def print_config(self) -> None:
        print(json.dumps(self.get_config(), indent=2))

    @staticmethod
    def load_from_config(config) -> "Sequential":
        if isinstance(config, str):
            config = json.loads(config)
        m = Sequential(config.get("name", "sequential"))
        for lj in config.get("layers", []):
            cfg = LayerConfig(lj.get("name", ""), lj.get("parameters", {}), lj.get("type", ""))
            m.add(LayerFactory.create(lj.get("type", ""), cfg))
        m.set_training(config.get("is_training", True))
        return m

    def save_config(self, filepath: str) -> None:
        with open(filepath, "w") as f:
            json.dump(self.get_config(), f, indent=2)

    @staticmethod
    def load_from_config_file(filepath: str) -> "Sequential":
        with open(filepath) as f:
            return Sequential.load_from_config(json.load(f))

    def save_to_file(self, path: str, save_state: bool = True) -> None:
        d = os.path.dirname(path)
        if d:
            os.makedirs(d, exist_ok=True)
        with open(path + ".json", "w") as f:
            json.dump(self.get_config(), f, indent=4)
        with open(path + ".bin", "wb") as f:
            for p in self.parameters():
                save_tensor(f, p)
        if save_state:
            self.save_state(path + ".state")
        self.save_bn_stats(path + ".bnstats")

    def load_weights_file(self, path: str) -> None:
        if not self.initialized:
            self.initialize()
        with open(path, "rb") as f:
            for p in self.parameters():
                t = load_tensor(f)
                if t.numel() != p.numel():
                    raise RuntimeError(f"checkpoint tensor {tuple(t.shape)} does not match parameter {tuple(p.shape)}")
                p.copy_(t.view(p.shape))
        self.arena.sync_shadow(force=True)

    @staticmethod
    def from_file(path: str, device=None) -> "Sequential":
        with open(path + ".json") as f:
            m = Sequential.load_from_config(json.load(f))
        if device is not None:
            m.set_device(device)
        m.initialize()
        m.load_weights_file(path + ".bin")
        if os.path.exists(path + ".state"):
            m.load_state(path + ".state")
        elif os.path.exists(path + ".bnstats"):
            m.load_bn_stats(path + ".bnstats")
        return m

    # language-neutral BatchNorm running statistics (.bin records: running_mean, running_var per
    # BatchNorm in layer order) shared with the C++ host API (csrc/host/nn.cpp)
    def save_bn_stats(self, path: str) -> None:
        with open(path, "wb") as f:
            for l in _all_layers(self.layers):
                if isinstance(l, BatchNorm):
                    save_tensor(f, l.running_mean.detach().reshape(-1, 1, 1, 1))
                    save_tensor(f, l.running_var.detach().reshape(-1, 1, 1, 1))

    def load_bn_stats(self, path: str) -> None:
        with open(path, "rb") as f:
            for l in _all_layers(self.layers):
                if isinstance(l, BatchNorm):
                    dev = l.running_mean.device
                    l.running_mean = load_tensor(f).reshape(-1).to(dev)
                    l.running_var = load_tensor(f).reshape(-1).to(dev)

    # sidecar: BN running statistics (not in the reference .bin, gap G11)
    def save_state(self, path: str, extra: Optional[dict] = None) -> None:
        state = {}
        for i, l in enumerate(_all_layers(self.layers)):
            if isinstance(l, BatchNorm):
                state[f"{i}:{l.name}:running_mean"] = l.running_mean.detach().cpu()
                state[f"{i}:{l.name}:running_var"] = l.running_var.detach().cpu()
        if extra:
            state.update(extra)
        torch.save(state, path)

    def load_state(self, path: str) -> dict:
        state = torch.load(path, map_location="cpu", weights_only=True)
        for i, l in enumerate(_all_layers(self.layers)):
            if isinstance(l, BatchNorm):
                k = f"{i}:{l.name}:running_mean"
                if k in state:
                    l.running_mean = state[k].to(self.device.torch_device)
                    l.running_var = state[f"{i}:{l.name}:running_var"].to(self.device.torch_device)
        return state

    def clone(self) -> "Sequential":
        c = Sequential(self.name_)
        c.set_training(self.training)
        for l in self.layers:
            c.add(l.clone())
        return c

    def split(self, partitions: List[Partition]) -> List["Sequential"]:
        if not partitions:
            raise ValueError("Partitions vector is empty")
        stages = []
        for k, part in enumerate(partitions):
            if not (0 <= part.start_layer < part.end_layer <= len(self.layers)):
                raise IndexError("Invalid partition range")
            st = Sequential(f"{self.name_}_part_{k}")
            for l in self.layers[part.start_layer:part.end_layer]:
                st.add(l.clone())
            st.set_training(self.training)
            stages.append(st)
        return stages


class SequentialBuilder:
    """Fluent builder with shape inference (reference `include/nn/sequential.hpp:1154-1340`)."""

    def __init__(self, name: str = "sequential"):
        self.model = Sequential(name)
        self.lb = LayerBuilder()

    def _n(self, name, prefix):
        return name if name else f"{prefix}_{self.model.layer_size()}"

    def _push(self):
        for l in self.lb.build():
            self.model.add(l)
            self.lb.layers.append  # noqa: B018 (builder keeps shape through the model)

    def input(self, shape):
        self.lb.input(shape)
        self._shape = [1] + list(shape)
        return self

    def get_current_shape(self):
        return list(self._shape)

    def _add(self, layer):
        self._shape = layer.compute_output_shape(self._shape)
        self.model.add(layer)
        return self

    def conv2d(self, out_channels, kernel_h, kernel_w, stride_h=1, stride_w=1, pad_h=0, pad_w=0, use_bias=True,
               name=""):
        return self._add(Conv2D(self._shape[1], out_channels, kernel_h, kernel_w, stride_h, stride_w, pad_h, pad_w,
                                use_bias, self._n(name, "conv2d")))

    def dense(self, output_features, use_bias=True, name=""):
        feat = 1
        for d in self._shape[1:]:
            feat *= d
        return self._add(Dense(feat, output_features, use_bias, self._n(name, "dense")))

    def batchnorm(self, epsilon=1e-5, momentum=0.1, affine=True, name=""):
        return self._add(BatchNorm(self._shape[1], epsilon, momentum, affine, self._n(name, "batchnorm")))

    def groupnorm(self, num_groups, epsilon=1e-5, affine=True, name=""):
        return self._add(GroupNorm(int(num_groups), self._shape[1], epsilon, affine, self._n(name, "groupnorm")))

    def activation(self, activation_name, name=""):
        return self._add(Activation(activation_name, self._n(name, "activation")))

    def maxpool2d(self, pool_h, pool_w, stride_h=1, stride_w=1, pad_h=0, pad_w=0, name=""):
        # NOTE: SequentialBuilder's default stride is 1 (reference G10), LayerBuilder's is the pool size
        return self._add(MaxPool2D(pool_h, pool_w, stride_h, stride_w, pad_h, pad_w, self._n(name, "maxpool2d")))

    def avgpool2d(self, pool_h, pool_w, stride_h=1, stride_w=1, pad_h=0, pad_w=0, name=""):
        return self._add(AvgPool2D(pool_h, pool_w, stride_h, stride_w, pad_h, pad_w, self._n(name, "avgpool2d")))

    def dropout(self, dropout_rate, name=""):
        return self._add(Dropout(dropout_rate, self._n(name, "dropout")))

    def flatten(self, name=""):
        return self._add(Flatten(self._n(name, "flatten")))

    def add_layer(self, layer: Layer):
        return self._add(layer)

    def residual(self, main_path: List[Layer], shortcut_path: List[Layer], activation="relu", name=""):
        return self._add(ResidualBlock(main_path, shortcut_path, activation, self._n(name, "residual_block")))

    def basic_residual_block(self, in_channels, out_channels, stride=1, name="basic_residual_block"):
        shape = [in_channels, self._shape[2], self._shape[3]]
        main = (LayerBuilder().input(shape)
                .conv2d(out_channels, 3, 3, stride, stride, 1, 1, True)
                .batchnorm(1e-5, 0.1, True, "bn0")
                .activation("relu")
                .conv2d(out_channels, 3, 3, 1, 1, 1, 1, True)
                .batchnorm(1e-5, 0.1, True, "bn0")
                .build())
        short = []
        if stride != 1 or in_channels != out_channels:
            short = (LayerBuilder().input(shape).conv2d(out_channels, 1, 1, stride, stride, 0, 0, False)
                     .batchnorm(1e-5, 0.1, True, "bn0").build())
        nm = name if name else f"basic_residual_block_{self.model.layer_size()}"
        return self._add(ResidualBlock(main, short, "relu", nm))

    def bottleneck_residual_block(self, in_channels, mid_channels, out_channels, stride=1,
                                  name="bottleneck_residual_block"):
        shape = [in_channels, self._shape[2], self._shape[3]]
        main = (LayerBuilder().input(shape)
                .conv2d(mid_channels, 1, 1, 1, 1, 0, 0, False)
                .batchnorm(1e-3, 0.1, True, "bn0")
                .activation("relu")
                .conv2d(mid_channels, 3, 3, stride, stride, 1, 1, False)
                .batchnorm(1e-3, 0.1, True, "bn0")
                .activation("relu")
                .conv2d(out_channels, 1, 1, 1, 1, 0, 0, False)
                .batchnorm(1e-3, 0.1, True, "bn0")
                .build())
        short = []
        if stride != 1 or in_channels != out_channels:
            short = (LayerBuilder().input(shape).conv2d(out_channels, 1, 1, stride, stride, 0, 0, False)
                     .batchnorm(1e-3, 0.1, True, "bn0").build())
        return self._add(ResidualBlock(main, short, "relu", name))

    def build(self) -> Sequential:
        if not hasattr(self, "_shape"):
            raise RuntimeError("Input shape must be set before building model. Use .input() method.")
        self.model.input_shape = list(self._shape[1:])
        return self.model
