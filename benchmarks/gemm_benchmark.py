#!/usr/bin/env python3
"""GEMM benchmark (reference benchmarks/gemm_benchmark.cpp: SGEMM NN/NT/TN vs MKL).
GPU: our MFMA gathered-GEMM kernels on plain dense shapes vs PyTorch's hipBLASLt matmul, bf16
and fp32. CPU (``--cpu``, or no GPU): the native blocked SGEMM/DGEMM (csrc/native/cpu_gemm.cpp,
through ``Matrix`` / ``ops.cpu.gemm``) in the NN / NT / TN forms vs PyTorch's CPU BLAS (the
reference compares its SGEMM with MKL).  Prints GFLOP/s or TFLOP/s per shape.

    python benchmarks/gemm_benchmark.py [--sizes 4096x4096x4096,8192x8192x8192]
    python benchmarks/gemm_benchmark.py --cpu --sizes 1024x1024x1024 --dtype fp64
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


def cpu_bench(fn, iters):
    fn()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    return (time.perf_counter() - t0) / iters


def cpu_main(a):
    from dcnn_amd.ops import cpu
    dt = torch.float64 if a.dtype == "fp64" else torch.float32
    sizes = a.sizes if a.sizes != DEFAULT_SIZES else "512x512x512,1024x1024x1024,2048x2048x2048,4096x64x576"
    iters = max(1, min(a.iters, 5))
    print(f"CPU {a.dtype}, {cpu.get_num_threads()} threads  (GFLOP/s)")
    print(f"{'M x N x K':<20}{'form':<6}{'native':>10}{'torch':>10}")
    for s in sizes.split(","):
        M, N, K = map(int, s.split("x"))
        f = 2.0 * M * N * K
        for form in ("NN", "NT", "TN"):
            ta, tb = form[0] == "T", form[1] == "T"
            x = torch.randn((K, M) if ta else (M, K), dtype=dt)
            w = torch.randn((N, K) if tb else (K, N), dtype=dt)
            out = torch.empty((M, N), dtype=dt)
            ours = cpu_bench(lambda: cpu.gemm(x, w, ta, tb, out=out), iters)
            xa, wb = (x.t() if ta else x), (w.t() if tb else w)
            ref = cpu_bench(lambda: torch.matmul(xa, wb, out=out), iters)
            err = (cpu.gemm(x, w, ta, tb) - xa @ wb).abs().max().item()
            print(f"{s:<20}{form:<6}{f / ours / 1e9:10.1f}{f / ref / 1e9:10.1f}   max|diff| {err:.1e}")


DEFAULT_SIZES = "4096x4096x4096,8192x8192x8192,256x4096x4096,131072x64x576"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default=DEFAULT_SIZES)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--cpu", action="store_true")
    ap.add_argument("--dtype", default="fp32", choices=["fp32", "fp64"])
    a = ap.parse_args()
    if a.cpu or not torch.cuda.is_available():
        cpu_main(a)
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
