#!/usr/bin/env python3
"""Device discovery, flows (HIP streams) and tasks (HIP events) (reference
examples/device_manager_example.cpp)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from dcnn_amd import DeviceManager, Task  # noqa: E402

dm = DeviceManager.instance()
for did in dm.get_device_ids():
    d = dm.get_device(did)
    print(f"{did}: {d.name()}  total {d.get_total_memory() / 2**30:.1f} GiB, "
          f"available {d.get_available_memory() / 2**30:.1f} GiB")
x = torch.arange(8, dtype=torch.float32)
if torch.cuda.is_available():
    gpu = dm.get_device("GPU:0")
    flow = gpu.get_flow("copy")          # dedicated HIP stream
    with torch.cuda.stream(flow.stream):
        y = x.to(gpu.torch_device, non_blocking=True) * 2
    task = Task(flow)                    # HIP event recorded on the flow
    task.sync()
    print("GPU result:", y.cpu().tolist())
else:
    print("no GPU visible; CPU device:", dm.get_cpu().id)
