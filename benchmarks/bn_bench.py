#!/usr/bin/env python3
"""BatchNorm apply-pass micro-benchmark at the ResNet-18-tiny activation shapes (bf16 NHWC).

Times the forward apply (scale/shift, + residual + ReLU as in a block tail) and the backward
apply (norm.hip) with the vectorised kernels on and off, reports device us per call and the
achieved HBM bandwidth, and checks the two kernel generations agree.

  python benchmarks/bn_bench.py --batch 256
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = [("l1", 64, 32), ("l2", 128, 16), ("l3", 256, 8), ("l4", 512, 4)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=50)
    a = ap.parse_args()
    from dcnn_amd.ops import hip
    from dcnn_amd.ops._ext import kernels
    K = kernels()
    dev = torch.device("cuda")
    g = torch.Generator(device="cpu").manual_seed(0)
    rows = []

    def timed(fn):
        # device time: the calls are captured in a hipGraph and replayed (no Python launch cost)
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr):
            for _ in range(a.iters):
                fn()
        gr.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            gr.replay()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / (5 * a.iters)

    for nm, C, HW in SHAPES:
        N = a.batch
        R = N * HW * HW
        mk = lambda: torch.randn(N, C, HW, HW, generator=g).to(dev).to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        x, res, dy = mk(), mk(), mk()
        # statistics as the conv epilogue leaves them after bn_stat_reduce: 8 partials on l1
        parts = 8 if C == 64 else 1
        part = torch.empty(parts, 3, C, device=dev)
        part[:, 0] = R / parts
        part[:, 1] = torch.randn(parts, C, generator=g).to(dev) * 0.1
        part[:, 2] = (R / parts) * (1 + torch.rand(parts, C, generator=g).to(dev))
        stats = hip.Stats(part, parts, 0) if parts > 1 else torch.cat([part[0, 1], part[0, 2] / part[0, 0]])
        gamma = (1 + 0.1 * torch.randn(C, generator=g)).to(dev)
        beta = (0.1 * torch.randn(C, generator=g)).to(dev)
        mean = (0.1 * torch.randn(C, generator=g)).to(dev)
        istd = (1 + 0.1 * torch.rand(C, generator=g)).to(dev)
        bsums = torch.randn(2 * C, generator=g).to(dev) * R * 0.01
        out = {}
        for vec in (0, 1):
            K.bn_set_vectorised(vec)
            fa = lambda: hip.bn_apply(x, stats, R, gamma, beta, 1e-5, relu=True)
            fr = lambda: hip.bn_apply(x, stats, R, gamma, beta, 1e-5, residual=res, relu=True)
            dx = torch.empty_like(x)
            def fb():
                st = hip.stream_ptr()
                K.bn_bwd_apply(1, dy.data_ptr(), 0, x.data_ptr(), dx.data_ptr(), R, C, mean.data_ptr(),
                               istd.data_ptr(), gamma.data_ptr(), bsums.data_ptr(), 1, float(R), 0, 0, 0, st)
            t = {"apply": timed(fa), "apply_res": timed(fr), "bwd_apply": timed(fb)}
            out[vec] = (fa().float(), fr().float(), (fb(), dx.float().clone())[1], t)
        K.bn_set_vectorised(1)
        nbytes = {"apply": 2, "apply_res": 3, "bwd_apply": 3}
        for k, i in (("apply", 0), ("apply_res", 1), ("bwd_apply", 2)):
            err = (out[0][i] - out[1][i]).abs().max().item()
            scale = out[0][i].abs().max().item()
            t0, t1 = out[0][3][k], out[1][3][k]
            gb = nbytes[k] * x.numel() * 2 / 1e9
            rows.append(dict(shape=nm, op=k, us_old=round(t0, 2), us_new=round(t1, 2),
                             tbps_old=round(gb / t0 * 1e3 / 1e3 * 1e3, 2), tbps_new=round(gb / t1 * 1e3 / 1e3 * 1e3, 2),
                             max_abs_diff=err, max_abs=scale))
            print(json.dumps(rows[-1]), flush=True)
    tot0 = sum(r["us_old"] for r in rows)
    tot1 = sum(r["us_new"] for r in rows)
    print(json.dumps({"total_us_old": round(tot0, 1), "total_us_new": round(tot1, 1)}))


if __name__ == "__main__":
    main()
