"""Device runtime: Device / DeviceManager / Flow (stream) / Task (event).

MI355X-native replacement for the reference's L2 device runtime
(`include/device/device.hpp:12`, `include/device/device_manager.hpp:9`,
`include/device/flow.hpp:11`, `include/device/task.hpp:26`).

Design differences (intentional):
  * memory comes from PyTorch-ROCm's stream-ordered caching allocator
    (`hipMallocAsync`-style pools) instead of raw `cudaMalloc` per tensor;
  * a `Flow` is a real HIP stream (`torch.cuda.Stream`), and several flows per
    device are used (compute / comm / h2d) instead of a single "default" one;
  * a `Task` is a HIP event recorded on the flow — `sync()` waits for that
    event only, it never device-synchronises;
  * every call honours the tensor's own device (`GPU:i`), there is no global
    "GPU 0" (reference defect G6).
"""
from __future__ import annotations

import enum
import threading
from typing import Dict, List, Optional

import torch


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
        return torch.cuda.get_device_name(self.index)

    def get_total_memory(self) -> int:
        if self.device_type == DeviceType.CPU:
            from .utils.hardware import total_memory_bytes
            return total_memory_bytes()
        return torch.cuda.get_device_properties(self.index).total_memory

    def get_available_memory(self) -> int:
        if self.device_type == DeviceType.CPU:
            from .utils.hardware import available_memory_bytes
            return available_memory_bytes()
        free, _ = torch.cuda.mem_get_info(self.index)
        return free

    def allocate(self, numel: int, dtype=torch.float32) -> torch.Tensor:
        return torch.empty(numel, dtype=dtype, device=self.torch_device)

    def copy_to_device(self, dst: torch.Tensor, src: torch.Tensor) -> None:
        dst.copy_(src, non_blocking=True)

    # --- flows ----------------------------------------------------------------------
    def get_flow(self, name: str = "default") -> "Flow":
        with self._lock:
            fl = self._flows.get(name)
            if fl is None:
                fl = Flow(self, name)
                self._flows[name] = fl
            return fl


class Flow:
    """Named execution queue. CPU flows are synchronous; GPU flows own a HIP stream.

    The "default" GPU flow maps to PyTorch's *current* stream so that captured hipGraphs and
    user-set streams are honoured; other names get dedicated non-blocking streams (e.g. "comm").
    """

    def __init__(self, device: Device, name: str):
        self.device = device
        self.name = name
        self._stream: Optional[torch.cuda.Stream] = None
        if device.is_gpu() and name != "default":
            self._stream = torch.cuda.Stream(device=device.torch_device)

    @property
    def stream(self):
        if not self.device.is_gpu():
            return None
        if self._stream is None:
            return torch.cuda.current_stream(self.device.torch_device)
        return self._stream

    def synchronize(self) -> None:
        if self.device.is_gpu():
            self.stream.synchronize()

    def wait(self, task: "Task") -> None:
        if self.device.is_gpu() and task.event is not None:
            self.stream.wait_event(task.event)


class Task:
    """Completion handle of asynchronously launched work (a recorded HIP event)."""

    def __init__(self, flow: Optional[Flow] = None):
        self.flow = flow
        self.event = None
        if flow is not None and flow.device.is_gpu():
            self.event = torch.cuda.Event()
            self.event.record(flow.stream)

    def sync(self) -> None:
        if self.event is not None:
            self.event.synchronize()

    def is_ready(self) -> bool:
        return True if self.event is None else self.event.query()


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


def create_task(device: Device, flow: str = "default") -> Task:
    return Task(device.get_flow(flow))
