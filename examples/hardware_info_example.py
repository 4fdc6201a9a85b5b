#!/usr/bin/env python3
"""Host + GPU hardware report with periodic CPU utilisation logging to ./logs/cpu_status.csv
(reference examples/hardware_info_example.cpp)."""
import csv
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dcnn_amd.utils import HardwareInfo  # noqa: E402

hw = HardwareInfo.initialize()
print(hw.summary())
os.makedirs("logs", exist_ok=True)
samples = int(sys.argv[1]) if len(sys.argv) > 1 else 5
with open("logs/cpu_status.csv", "w", newline="") as f:
    w = csv.writer(f)
    w.writerow(["t", "cpu_util_total", "rss_mb"] + [f"core{i}" for i in range(hw.cpu.get("logical_cores", 0))])
    t0 = time.time()
    for _ in range(samples):
        hw.update_dynamic_info(200)
        w.writerow([round(time.time() - t0, 2), round(hw.cpu_util_total, 1), round(hw.rss_kb / 1024, 1)]
                   + [round(u, 1) for u in hw.cpu_util_per_core])
print("CPU status data written to ./logs/cpu_status.csv")
