#!/usr/bin/env python3
"""Payload compression benchmark (reference benchmarks/compression_benchmark.cpp: zstd level 3)."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dcnn_amd.ops._ext import native  # noqa: E402

c = native().comm
rng = np.random.default_rng(0)
relu_act = np.maximum(rng.normal(size=16 * 2**20 // 4).astype(np.float32), 0)  # activations: ~50% zeros
data = {"relu activations": relu_act.tobytes(), "random": rng.random(16 * 2**20 // 4).astype(np.float32).tobytes()}
for name, raw in data.items():
    for codec, cname in ((2, "zstd"), (1, "zlib")):
        if codec == 2 and not c.zstd_available():
            continue
        t0 = time.perf_counter()
        z = c.compress(raw, codec, 3)
        t1 = time.perf_counter()
        back = c.decompress(z, codec, len(raw))
        t2 = time.perf_counter()
        assert back == raw
        print(f"{name:<17}{cname:<5} ratio {len(raw) / len(z):5.2f}  compress {len(raw) / 2**20 / (t1 - t0):8.1f} MiB/s"
              f"  decompress {len(raw) / 2**20 / (t2 - t1):8.1f} MiB/s")
