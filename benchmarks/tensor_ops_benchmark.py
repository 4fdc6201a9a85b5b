#!/usr/bin/env python3
"""Tensor-op benchmark (reference benchmarks/tensor_ops_benchmark.cpp): im2col / col2im,
NCHW<->CNHW, pad, transpose, reductions on the GPU kernels vs the CPU path (GB/s)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dcnn_amd.ops import generic as G  # noqa: E402
from dcnn_amd.tensor import ops as T  # noqa: E402


def timeit(fn, dev, iters=10):
    fn()
    if dev == "cuda":
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    if dev == "cuda":
        torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters


def main():
    devs = ["cpu"] + (["cuda"] if torch.cuda.is_available() else [])
    for dev in devs:
        x = torch.randn(128, 64, 32, 32, device=dev)
        nb = x.numel() * 4
        rows = [
            ("im2col 3x3", lambda: T.im2col(x, 3, 3, 1, 1, 1, 1), nb * 10),
            ("nchw->cnhw", lambda: G.nchw_to_cnhw(x), nb * 2),
            ("pad 2", lambda: T.pad(x, 2, 2), nb * 2),
            ("transpose", lambda: G.transpose_2d(x.reshape(-1), 128 * 64, 1024), nb * 2),
            ("sum", lambda: G.sum(x.reshape(-1)), nb),
            ("axpy", lambda: G.axpy(0.5, x.reshape(-1), x.reshape(-1)), nb * 3),
        ]
        for name, fn, bytes_moved in rows:
            t = timeit(fn, dev)
            print(f"{dev:<5}{name:<14}{t * 1e6:10.1f} us {bytes_moved / t / 1e9:9.1f} GB/s")


if __name__ == "__main__":
    main()
