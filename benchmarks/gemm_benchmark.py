#!/usr/bin/env python3
"""GEMM benchmark (reference benchmarks/gemm_benchmark.cpp: SGEMM NN/NT/TN vs MKL).
Our MFMA gathered-GEMM kernels on plain dense shapes vs PyTorch's hipBLASLt matmul, bf16 and
fp32, on the GPU; CPU: PyTorch SGEMM.  Prints TFLOP/s per shape.

    python benchmarks/gemm_benchmark.py [--sizes 4096x4096x4096,8192x8192x8192]
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def bench(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e-3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="4096x4096x4096,8192x8192x8192,256x4096x4096,131072x64x576")
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    if not torch.cuda.is_available():
        for s in a.sizes.split(","):
            M, N, K = map(int, s.split("x"))
            x, w = torch.randn(M, K), torch.randn(N, K)
            t0 = time.perf_counter()
            x @ w.t()
            dt = time.perf_counter() - t0
            print(f"CPU sgemm {s}: {2 * M * N * K / dt / 1e12:.3f} TFLOP/s")
        return
    from dcnn_amd.ops import hip
    print(f"{'M x N x K':<22}{'dtype':<6}{'dcnn MFMA':>12}{'hipBLASLt':>12}  (TFLOP/s)")
    for s in a.sizes.split(","):
        M, N, K = map(int, s.split("x"))
        for dt in (torch.bfloat16, torch.float32):
            x = torch.randn(M, K, device="cuda").to(dt)
            w = torch.randn(N, K, device="cuda").to(dt)
            f = 2.0 * M * N * K
            ours = bench(lambda: hip.dense_fwd(x, w, None), a.iters)
            ref = bench(lambda: x @ w.t(), a.iters)
            print(f"{s:<22}{str(dt).split('.')[-1][:4]:<6}{f / ours / 1e12:12.1f}{f / ref / 1e12:12.1f}")


if __name__ == "__main__":
    main()
