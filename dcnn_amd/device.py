"""Device runtime: Device / DeviceManager / Flow (stream) / Task (event).

MI355X-native replacement for the reference's L2 device runtime
(`include/device/device.hpp:12`, `include/device/device_manager.hpp:9`,
`include/device/flow.hpp:11`, `include/device/task.hpp:26`).

The GPU side is a thin Python layer over the native HIP runtime of the kernel library
(``_kernels.rt``, csrc/kernels/runtime.cpp):

  * memory: ``Device.allocate`` draws from a per-device stream-ordered caching pool
    (``hipMallocFromPoolAsync`` on the caller's flow, release threshold "keep everything") and
    hands the buffer to PyTorch zero-copy through DLPack — the framework's flat parameter /
    gradient / optimizer arenas live there; ``allocator_stats()`` shows reuse (steady-state
    training allocates without growing the reservation) instead of the reference's cudaMalloc
    per tensor;
  * a ``Flow`` is a native HIP stream (non-blocking, optional priority); the "default" flow wraps
    PyTorch's *current* stream handle, so captured hipGraphs and user-set streams are honoured,
    and ``Flow.stream`` exposes any flow to PyTorch as an external stream;
  * a ``Task`` is a native HIP event recorded on a flow — ``sync()`` waits for that event only,
    it never device-synchronises;
  * every call honours the device it is made on (``GPU:i``), there is no global "GPU 0"
    (reference defect G6).
CPU devices keep host semantics (synchronous flows, no events).
"""
from __future__ import annotations

import enum
import threading
from typing import Dict, List, Optional

import torch


def _rt():
    from .ops._ext import kernels
    return kernels().rt


_DLPACK_CODES = {torch.float32: (2, 32), torch.float64: (2, 64), torch.float16: (2, 16), torch.bfloat16: (4, 16),
                 torch.int32: (0, 32), torch.int64: (0, 64), torch.int16: (0, 16), torch.int8: (0, 8),
                 torch.uint8: (1, 8)}


class DeviceType(enum.Enum):
    CPU = 0
    GPU = 1


class Device:
    """A compute device: `CPU:0` or `GPU:i` (one MI355X)."""

    def __init__(self, dtype: DeviceType, index: int = 0):
        self.device_type = dtype
        self.index = index
        self._flows: Dict[str, "Flow"] = {}
        self._lock = threading.Lock()

    # --- identity -------------------------------------------------------------------
    @property
    def id(self) -> str:
        return f"{'CPU' if self.device_type == DeviceType.CPU else 'GPU'}:{self.index}"

    @property
    def torch_device(self) -> torch.device:
        if self.device_type == DeviceType.CPU:
            return torch.device("cpu")
        return torch.device("cuda", self.index)

    def is_gpu(self) -> bool:
        return self.device_type == DeviceType.GPU

    def __repr__(self) -> str:
        return f"Device({self.id})"

    def __eq__(self, other) -> bool:
        return isinstance(other, Device) and other.id == self.id

    def __hash__(self) -> int:
        return hash(self.id)

    # --- memory ---------------------------------------------------------------------
    def name(self) -> str:
        if self.device_type == DeviceType.CPU:
            try:
                from .utils.hardware import cpu_model_name
                return cpu_model_name()
            except Exception:
                return "CPU"
        return _rt().device_properties(self.index)["name"]

    def properties(self) -> dict:
        """Native device properties (name, gfx arch, memory, CU count, LDS, L2, ...)."""
        if self.device_type == DeviceType.CPU:
            return {"name": self.name()}
        return dict(_rt().device_properties(self.index))

    def get_total_memory(self) -> int:
        if self.device_type == DeviceType.CPU:
            from .utils.hardware import total_memory_bytes
            return total_memory_bytes()
        return int(_rt().mem_info(self.index)[1])

    def get_available_memory(self) -> int:
        if self.device_type == DeviceType.CPU:
            from .utils.hardware import available_memory_bytes
            return available_memory_bytes()
        return int(_rt().mem_info(self.index)[0])

    def allocate(self, numel, dtype=torch.float32, zero: bool = False, flow: str = "default") -> torch.Tensor:
        """A buffer of ``numel`` (int or shape) elements. GPU: from the native stream-ordered pool
        on ``flow`` (zero-copy PyTorch tensor via DLPack); CPU: host memory."""
        shape = [int(numel)] if isinstance(numel, int) else [int(s) for s in numel]
        if self.device_type == DeviceType.CPU:
            return torch.zeros(shape, dtype=dtype) if zero else torch.empty(shape, dtype=dtype)
        code, bits = _DLPACK_CODES[dtype]
        cap = _rt().alloc_dlpack(self.index, shape, code, bits, self.get_flow(flow).native, zero)
        return torch.from_dlpack(cap)

    def allocator_stats(self) -> dict:
        if self.device_type == DeviceType.CPU:
            return {}
        d = dict(_rt().Allocator.get(self.index).stats())
        from .runtime.arena import device_stats
        d.update(device_stats(self.index))  # the per-step activation arenas' share of in_use_bytes
        return d

    def copy_to_device(self, dst: torch.Tensor, src: torch.Tensor, flow: str = "default") -> None:
        """dst <- src, asynchronous on ``flow`` for GPU copies of dense same-dtype tensors."""
        if (self.device_type == DeviceType.GPU and dst.dtype == src.dtype and dst.numel() == src.numel()
                and dst.is_contiguous() and src.is_contiguous() and (dst.is_cuda or src.is_cuda)):
            kind = 2 if (dst.is_cuda and src.is_cuda) else (0 if dst.is_cuda else 1)
            _rt().memcpy_async(dst.data_ptr(), src.data_ptr(), dst.numel() * dst.element_size(), kind,
                               self.get_flow(flow).native)
            return
        dst.copy_(src, non_blocking=True)

    def synchronize(self) -> None:
        """Device-wide synchronize; also returns buffers released since the last allocation to
        the native pool (their frees are deferred: see runtime.cpp Allocator::defer_free)."""
        if self.device_type == DeviceType.GPU:
            _rt().device_synchronize(self.index)
            _rt().Allocator.get(self.index).release_deferred()

    # --- flows ----------------------------------------------------------------------
    def get_flow(self, name: str = "default") -> "Flow":
        with self._lock:
            fl = self._flows.get(name)
            if fl is None:
                fl = Flow(self, name)
                self._flows[name] = fl
            return fl


class Flow:
    """Named execution queue. CPU flows are synchronous; GPU flows are native HIP streams.

    The "default" GPU flow wraps PyTorch's *current* stream handle (looked up at every use) so
    that captured hipGraphs and user-set streams are honoured; other names own dedicated
    non-blocking streams (e.g. "comm", "h2d"); ``priority`` < 0 is a high-priority stream.
    """

    def __init__(self, device: Device, name: str, priority: int = 0):
        self.device = device
        self.name = name
        self._native = None
        if device.is_gpu() and name != "default":
            self._native = _rt().Flow(device.index, int(priority))
        self._torch_stream = None

    @property
    def native(self):
        """The native ``rt.Flow`` (for the default flow: a wrapper of the current stream)."""
        if self._native is not None:
            return self._native
        h = torch.cuda.current_stream(self.device.torch_device).cuda_stream
        return _rt().Flow.wrap(self.device.index, int(h))

    @property
    def stream(self):
        """This flow as a PyTorch stream (``with torch.cuda.stream(flow.stream): ...``)."""
        if not self.device.is_gpu():
            return None
        if self._native is None:
            return torch.cuda.current_stream(self.device.torch_device)
        if self._torch_stream is None:
            self._torch_stream = torch.cuda.ExternalStream(self._native.handle, device=self.device.torch_device)
        return self._torch_stream

    def synchronize(self) -> None:
        if self.device.is_gpu():
            self.native.synchronize()

    def wait(self, task: "Task") -> None:
        if self.device.is_gpu() and task.native is not None:
            self.native.wait(task.native)

    def query(self) -> bool:
        return True if not self.device.is_gpu() else bool(self.native.query())


class Task:
    """Completion handle of asynchronously launched work (a native HIP event on the flow)."""

    def __init__(self, flow: Optional[Flow] = None, timing: bool = False):
        self.flow = flow
        self.native = None
        if flow is not None and flow.device.is_gpu():
            self.native = _rt().Task(flow.device.index, bool(timing))
            self.native.record(flow.native)

    def sync(self) -> None:
        if self.native is not None:
            self.native.sync()

    def is_ready(self) -> bool:
        return True if self.native is None else bool(self.native.is_ready())

    def elapsed_ms(self, end: "Task") -> float:
        return float(self.native.elapsed_ms(end.native))


def task_sync_all(tasks: List[Task]) -> None:
    for t in tasks:
        t.sync()


class DeviceManager:
    """Singleton registry: CPU:0 plus every visible MI355X as GPU:i (`src/device/device_manager.cpp:16`)."""

    _instance: Optional["DeviceManager"] = None

    def __init__(self):
        self._devices: Dict[str, Device] = {}
        cpu = Device(DeviceType.CPU, 0)
        self._devices[cpu.id] = cpu
        n = torch.cuda.device_count()  # counting does not initialise HIP
        for i in range(n):
            d = Device(DeviceType.GPU, i)
            self._devices[d.id] = d
        self._default = cpu

    @classmethod
    def instance(cls) -> "DeviceManager":
        if cls._instance is None:
            cls._instance = DeviceManager()
        return cls._instance

    def get_device(self, device_id) -> Device:
        if isinstance(device_id, Device):
            return device_id
        if isinstance(device_id, DeviceType):
            return self.get_cpu() if device_id == DeviceType.CPU else self.get_gpu(0)
        if isinstance(device_id, torch.device):
            return self.get_cpu() if device_id.type == "cpu" else self.get_gpu(device_id.index or 0)
        s = str(device_id).upper()
        if s in ("CPU", "CPU:0"):
            return self.get_cpu()
        if s in ("GPU", "CUDA"):
            return self.get_gpu(0)
        if s.startswith("CUDA:"):
            s = "GPU:" + s.split(":")[1]
        if s not in self._devices:
            raise KeyError(f"unknown device {device_id!r}; available: {list(self._devices)}")
        return self._devices[s]

    def get_cpu(self) -> Device:
        return self._devices["CPU:0"]

    def get_gpu(self, index: int = 0) -> Device:
        key = f"GPU:{index}"
        if key not in self._devices:
            raise RuntimeError(f"{key} not available ({torch.cuda.device_count()} GPUs visible)")
        return self._devices[key]

    def get_device_ids(self) -> List[str]:
        return list(self._devices)

    def has_device(self, device_id: str) -> bool:
        return device_id.upper() in self._devices

    def get_devices_by_type(self, t: DeviceType) -> List[Device]:
        return [d for d in self._devices.values() if d.device_type == t]

    def set_default_device(self, device_id) -> None:
        self._default = self.get_device(device_id)

    def get_default_device(self) -> Device:
        return self._default


def get_cpu() -> Device:
    return DeviceManager.instance().get_cpu()


def get_gpu(index: int = 0) -> Device:
    return DeviceManager.instance().get_gpu(index)


def get_device(device_id) -> Device:
    return DeviceManager.instance().get_device(device_id)


def create_task(device: Device, flow: str = "default", timing: bool = False) -> Task:
    return Task(device.get_flow(flow), timing)
