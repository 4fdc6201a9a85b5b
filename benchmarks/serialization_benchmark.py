#!/usr/bin/env python3
"""Serialization / control-plane benchmark (reference benchmarks/serialization_benchmark.cpp,
1 GiB tensor): native message encode/decode and a TCP loopback round trip."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dcnn_amd.ops._ext import native  # noqa: E402

c = native().comm
mb = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
arr = np.ones(mb * 2**20 // 4, dtype=np.float32)
m = c.Message("peer", 1)
t0 = time.perf_counter()
m.set_tensor(0, arr, legacy=True)
t1 = time.perf_counter()
b = c.serialize(m)
t2 = time.perf_counter()
r = c.deserialize(b)
t3 = time.perf_counter()
print(f"{mb} MiB: set_tensor {mb / 1024 / (t1 - t0):.2f} GiB/s, serialize {mb / 1024 / (t2 - t1):.2f} GiB/s, "
      f"deserialize {mb / 1024 / (t3 - t2):.2f} GiB/s")
del b, r
srv = c.TcpCommunicator("srv", "127.0.0.1", 0)
cli = c.TcpCommunicator("cli", "127.0.0.1", 0)
cli.connect("srv", "127.0.0.1", srv.port, 5000)
srv.wait_for_peer("cli", 5000)
m = c.Message("srv", 1)
m.set_tensor(0, arr)
t0 = time.perf_counter()
cli.send(m)
got = srv.recv(120000)
t1 = time.perf_counter()
print(f"TCP loopback {mb} MiB: {mb / 1024 / (t1 - t0):.2f} GiB/s ({got.nbytes} bytes)")
cli.close()
srv.close()
