"""Utilities: environment/config, hardware info, memory, profiling."""
from .env import get_env, load_env_file  # noqa: F401
from .hardware import HardwareInfo, gpu_info, xgmi_topology  # noqa: F401
from .memory import device_memory, format_bytes, get_memory_usage_kb  # noqa: F401
from .profiling import DeviceTimer, ProfilerType, benchmark, roctx_range  # noqa: F401
