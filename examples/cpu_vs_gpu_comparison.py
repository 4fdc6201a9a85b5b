#!/usr/bin/env python3
"""CPU vs GPU kernel comparison (reference examples/cuda_vs_avx2_comparison.cpp).

The reference times its multithreaded AVX2 kernels against its CUDA kernels on large float
arrays (add, mul, add_scalar, sqrt, ...), reports the host memory bandwidth as the CPU's
ceiling, checks that both devices produce the same values, and prints the speedups. Here the CPU
side is the framework's native C++ backend (``ops.cpu``: AVX-512/AVX2 kernels on the native
thread pool) and the GPU side the HIP kernels of ``ops.hip`` on an MI355X, both reached through
the device-dispatching ``ops.generic`` API; host<->device copies go through the native runtime
(``Device.copy_to_device``). GPU times are HIP-event times of the kernels alone (data already
resident), as in the reference; the transfer rows show what moving the data would cost.

    python examples/cpu_vs_gpu_comparison.py [--size 16777216] [--iters 10]
"""
import argparse
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from dcnn_amd.device import get_cpu, get_gpu  # noqa: E402
from dcnn_amd.ops import cpu as native_cpu  # noqa: E402
from dcnn_amd.ops import generic as G  # noqa: E402


def host_bandwidth(mb: int = 512) -> float:
    src = np.ones(mb * (1 << 20) // 4, dtype=np.float32)
    dst = np.empty_like(src)
    np.copyto(dst, src)
    t0 = time.perf_counter()
    np.copyto(dst, src)
    dt = time.perf_counter() - t0
    return src.nbytes * 2 / dt / 1e9  # read + write


def time_cpu(fn, iters):
    fn()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    return (time.perf_counter() - t0) / iters * 1e3


def time_gpu(fn, iters):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


OPS = {
    "add": (lambda a, b, c: G.add(a, b, out=c), 3),
    "mul": (lambda a, b, c: G.mul(a, b, out=c), 3),
    "add_scalar": (lambda a, b, c: G.add_scalar(a, 2.5, out=c), 2),
    "mul_scalar": (lambda a, b, c: G.mul_scalar(a, 0.75, out=c), 2),
    "sqrt": (lambda a, b, c: G.sqrt(a, out=c), 2),
    "fmadd": (lambda a, b, c: G.fmadd(a, b, c), 4),
}


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=1 << 24, help="elements per array (reference: 100M)")
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args(argv)
    n = a.size
    print(f"Available CPU threads: {native_cpu.get_num_threads()}")
    bw = host_bandwidth()
    print(f"System memory bandwidth (memcpy, read + write): {bw:.1f} GB/s")
    cpu = get_cpu()
    print(f"Using CPU device: {cpu.name()}")
    gpu = get_gpu(0) if torch.cuda.is_available() else None
    print(f"Using GPU device: {gpu.name() if gpu else '(none: CPU rows only)'}")
    print(f"Test size: {n} elements ({n * 4 >> 20} MB per array), iterations: {a.iters}\n")

    ha = torch.rand(n) + 0.5
    hb = torch.rand(n) + 0.5
    hc = torch.empty(n)
    if gpu is not None:
        da, db, dc = (gpu.allocate(n) for _ in range(3))
        t0 = time.perf_counter()
        gpu.copy_to_device(da, ha)
        gpu.copy_to_device(db, hb)
        gpu.synchronize()
        h2d = 2 * n * 4 / (time.perf_counter() - t0) / 1e9
        print(f"host -> device copy: {h2d:.1f} GB/s (pageable)")
    print(f"\n{'op':<12}{'CPU ms':>10}{'CPU GB/s':>10}{'GPU ms':>10}{'GPU GB/s':>10}{'speedup':>10}  check")
    for name, (fn, arrays) in OPS.items():
        nbytes = arrays * n * 4
        hc.fill_(1.0)
        tc = time_cpu(lambda: fn(ha, hb, hc), a.iters)
        row = f"{name:<12}{tc:10.3f}{nbytes / tc / 1e6:10.1f}"
        if gpu is not None:
            dc.fill_(1.0)
            tg = time_gpu(lambda: fn(da, db, dc), a.iters)
            # same op once more from a known state on both devices, then compare
            hc.fill_(1.0)
            dc.fill_(1.0)
            fn(ha, hb, hc)
            fn(da, db, dc)
            err = (dc.cpu() - hc).abs().max().item()
            row += f"{tg:10.3f}{nbytes / tg / 1e6:10.1f}{tc / tg:9.1f}x  {'OK' if err <= 1e-5 else f'MISMATCH {err:.2e}'}"
        print(row)
    s_cpu = float(G.sum(ha))
    line = f"\nsum reduction: CPU {s_cpu:.6e}"
    if gpu is not None:
        s_gpu = float(G.sum(da))
        line += f"  GPU {s_gpu:.6e}  rel diff {abs(s_gpu - s_cpu) / abs(s_cpu):.1e}"
    print(line)
    return 0


if __name__ == "__main__":
    sys.exit(main())
