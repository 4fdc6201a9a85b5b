"""Memory usage helpers (reference include/utils/memory.hpp:10 get_memory_usage_kb), plus device
memory for a GPU (HBM3E, 288 GB per MI355X)."""
from __future__ import annotations

from typing import Dict

import torch

from .hardware import process_rss_kb


def get_memory_usage_kb() -> int:
    return process_rss_kb()


def device_memory(device: int = 0) -> Dict[str, int]:
    if not torch.cuda.is_available():
        return {}
    free, total = torch.cuda.mem_get_info(device)
    return {"free": free, "total": total, "allocated": torch.cuda.memory_allocated(device),
            "reserved": torch.cuda.memory_reserved(device), "peak": torch.cuda.max_memory_allocated(device)}


def format_bytes(n: float) -> str:
    for unit in ("B", "KiB", "MiB", "GiB", "TiB"):
        if abs(n) < 1024 or unit == "TiB":
            return f"{n:.1f} {unit}" if unit != "B" else f"{int(n)} B"
        n /= 1024
    return f"{n:.1f} TiB"
