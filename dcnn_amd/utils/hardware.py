"""Host + GPU hardware information.

Host side comes from the native C++ runtime (``_native.read_cpu_info`` etc., counterpart of
the reference's ``HardwareInfo`` in src/utils/hardware_info.cpp:55-818: /proc/cpuinfo,
/proc/meminfo, cgroup limits, /proc/stat utilisation, thermal zones, P/E-core split).  The
GPU side (absent in the reference) reports each visible MI355X: name, gfx arch, CU count,
HBM capacity and — when ``rocm-smi`` is on PATH — the xGMI hop/link matrix that decides how
pipeline stages and DP rings are placed.
"""
from __future__ import annotations

import os
import shutil
import subprocess
from dataclasses import dataclass, field
from typing import Dict, List, Optional

from ..ops._ext import native


def _meminfo_kb(key: str) -> int:
    try:
        with open("/proc/meminfo") as f:
            for line in f:
                if line.startswith(key + ":"):
                    return int(line.split()[1])
    except OSError:
        pass
    return 0


def total_memory_bytes() -> int:
    return _meminfo_kb("MemTotal") * 1024


def available_memory_bytes() -> int:
    return _meminfo_kb("MemAvailable") * 1024


def cpu_model_name() -> str:
    try:
        return native().read_cpu_info()["model_name"] or "CPU"
    except Exception:  # pragma: no cover - native lib missing
        return "CPU"


@dataclass
class GpuInfo:
    index: int
    name: str
    arch: str
    compute_units: int
    total_memory: int
    xgmi_links: Dict[int, str] = field(default_factory=dict)  # peer -> link type


@dataclass
class HardwareInfo:
    """Snapshot of the host (static) + dynamic utilisation (``update_dynamic_info``)."""
    cpu: dict = field(default_factory=dict)
    gpus: List[GpuInfo] = field(default_factory=list)
    cpu_util_total: float = 0.0
    cpu_util_per_core: List[float] = field(default_factory=list)
    rss_kb: int = 0
    thermal: List = field(default_factory=list)

    @classmethod
    def initialize(cls, with_gpus: bool = True) -> "HardwareInfo":
        hw = cls(cpu=dict(native().read_cpu_info()))
        if with_gpus:
            hw.gpus = gpu_info()
        return hw

    def update_dynamic_info(self, sample_ms: int = 100) -> None:
        n = native()
        self.cpu_util_per_core = list(n.cpu_utilization(sample_ms))
        self.cpu_util_total = (sum(self.cpu_util_per_core) / len(self.cpu_util_per_core)
                               if self.cpu_util_per_core else 0.0)
        self.rss_kb = int(n.process_rss_kb())
        self.thermal = list(n.thermal_zones())

    def summary(self) -> str:
        c = self.cpu
        lines = [f"CPU: {c.get('model_name', '?')} ({c.get('vendor', '?')}), {c.get('physical_cores')} physical / "
                 f"{c.get('logical_cores')} logical cores, {c.get('sockets')} socket(s)",
                 f"RAM: {c.get('total_mem_kb', 0) / 2**20:.1f} GiB total, {c.get('avail_mem_kb', 0) / 2**20:.1f} GiB "
                 f"available"]
        if c.get("pcores") and c.get("ecores"):
            lines.append(f"P-cores {c['pcores']}  E-cores {c['ecores']}")
        for g in self.gpus:
            lines.append(f"GPU {g.index}: {g.name} [{g.arch}] {g.compute_units} CUs, {g.total_memory / 2**30:.0f} GiB")
        if self.cpu_util_per_core:
            lines.append(f"CPU utilisation {self.cpu_util_total:.1f}%  RSS {self.rss_kb / 1024:.1f} MiB")
        return "\n".join(lines)


def gpu_info() -> List[GpuInfo]:
    import torch
    out: List[GpuInfo] = []
    if not torch.cuda.is_available():
        return out
    links = xgmi_topology()
    for i in range(torch.cuda.device_count()):
        p = torch.cuda.get_device_properties(i)
        out.append(GpuInfo(i, p.name, getattr(p, "gcnArchName", "gfx950"), p.multi_processor_count, p.total_memory,
                           links.get(i, {})))
    return out


def xgmi_topology() -> Dict[int, Dict[int, str]]:
    """Parse ``rocm-smi --showtopotype`` into {gpu: {peer: 'XGMI'|'PCIE'}} (empty if unavailable)."""
    exe = shutil.which("rocm-smi")
    if exe is None:
        return {}
    try:
        txt = subprocess.run([exe, "--showtopotype"], capture_output=True, text=True, timeout=20).stdout
    except Exception:
        return {}
    topo: Dict[int, Dict[int, str]] = {}
    for line in txt.splitlines():
        parts = line.split()
        if len(parts) > 2 and parts[0] == "GPU" and parts[1].isdigit():
            row = int(parts[1])
            kinds = [p for p in parts[2:] if p in ("XGMI", "PCIE", "0")]
            topo[row] = {j: k for j, k in enumerate(kinds) if k != "0" and j != row}
    return topo


def process_rss_kb() -> int:
    try:
        return int(native().process_rss_kb())
    except Exception:
        return 0


def num_threads_default() -> int:
    return int(os.environ.get("NUM_THREADS", "0")) or (os.cpu_count() or 1)
