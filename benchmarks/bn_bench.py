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

SHAPES = {
    "resnet18": [("l1", 64, 32), ("l2", 128, 16), ("l3", 256, 8), ("l4", 512, 4)],
    # ResNet-50-tiny: each stage's widest (4x expansion) tensor and its bottleneck width
    "resnet50": [("l1.w", 256, 32), ("l1.b", 64, 32), ("l2.w", 512, 16), ("l2.b", 128, 16), ("l3.w", 1024, 8),
                 ("l3.b", 256, 8), ("l4.w", 2048, 4), ("l4.b", 512, 4)],
}
HBM_TBPS = 8.0  # MI355X HBM3E peak


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--model", choices=sorted(SHAPES), default="resnet18")
    ap.add_argument("--vec-only", action="store_true", help="the production (vectorised) kernels only, plus the "
                    "dual-branch passes: bytes moved and achieved bandwidth vs HBM peak")
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

    if a.vec_only:
        return bandwidth_table(a, K, hip, dev, g, timed)
    for nm, C, HW in SHAPES[a.model]:
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


def bandwidth_table(a, K, hip, dev, g, timed):
    """Production BatchNorm passes (vectorised kernels): forward apply (+ReLU), the block tail
    (+ residual + ReLU), the dual tail (two BatchNorms + add + ReLU: projection blocks), the
    backward apply and its dual form; minimum bytes each pass must move (bf16 tensors; the
    per-channel vectors are negligible) and the achieved fraction of HBM peak."""
    K.bn_set_vectorised(1)
    rows = []
    print(f"| shape | C x HW x HW | op | tensors | MB | us | TB/s | % of {HBM_TBPS:.0f} TB/s |")
    print("|---|---|---|---:|---:|---:|---:|---:|")
    for nm, C, HW in SHAPES[a.model]:
        N = a.batch
        R = N * HW * HW
        mk = lambda: torch.randn(N, C, HW, HW, generator=g).to(dev).to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        x, x2, res, dy = mk(), mk(), mk(), mk()
        stats = torch.cat([0.1 * torch.randn(C, generator=g), 1 + torch.rand(C, generator=g)]).to(dev)
        gamma = (1 + 0.1 * torch.randn(C, generator=g)).to(dev)
        beta = (0.1 * torch.randn(C, generator=g)).to(dev)
        mean = (0.1 * torch.randn(C, generator=g)).to(dev)
        istd = (1 + 0.1 * torch.rand(C, generator=g)).to(dev)
        bsums = torch.randn(2 * C, generator=g).to(dev) * R * 0.01
        other = hip.BnDeferred(x2, stats, R, gamma, beta, 1e-5, None, None, 0.1, False)
        dx, dx2 = torch.empty_like(x), torch.empty_like(x)
        dg, db = torch.zeros(C, device=dev), torch.zeros(C, device=dev)

        def fb():
            K.bn_bwd_apply(1, dy.data_ptr(), 0, x.data_ptr(), dx.data_ptr(), R, C, mean.data_ptr(), istd.data_ptr(),
                           gamma.data_ptr(), bsums.data_ptr(), 1, float(R), 0, 0, 0, hip.stream_ptr())

        def fbd():
            side = lambda xx, d: (xx.data_ptr(), d.data_ptr(), mean.data_ptr(), istd.data_ptr(), gamma.data_ptr(),
                                  bsums.data_ptr(), 1, float(R), dg.data_ptr(), db.data_ptr())
            K.bn_bwd_apply_dual(dy.data_ptr(), side(x, dx), side(x2, dx2), R, C, hip.stream_ptr())

        cp = torch.empty_like(x)
        ops = [("copy (reference)", 2, lambda: cp.copy_(x)),
               ("apply+relu", 2, lambda: hip.bn_apply(x, stats, R, gamma, beta, 1e-5, relu=True)),
               ("apply+res+relu", 3, lambda: hip.bn_apply(x, stats, R, gamma, beta, 1e-5, residual=res, relu=True)),
               ("bwd_apply", 3, fb)]
        if hip.bn_dual_ok(x):
            ops.append(("dual apply+relu", 3, lambda: hip.bn_apply_dual(x, stats, R, gamma, beta, 1e-5, other,
                                                                        relu=True)))
        if K.bn_apply_dual_supported(R, C):
            ops.append(("bwd_apply_dual", 5, fbd))
        for op, nt, fn in ops:
            us = timed(fn)
            mb = nt * x.numel() * 2 / 1e6
            tbps = mb / us  # MB/us = TB/s
            rows.append(dict(shape=nm, C=C, HW=HW, op=op, tensors=nt, MB=round(mb, 1), us=round(us, 2),
                             tbps=round(tbps, 2), pct_peak=round(100 * tbps / HBM_TBPS, 1)))
            print(f"| {nm} | {C} x {HW} x {HW} | {op} | {nt} | {mb:.1f} | {us:.2f} | {tbps:.2f} | "
                  f"{100 * tbps / HBM_TBPS:.0f}% |", flush=True)
    big = [r for r in rows if r["MB"] >= 64 and not r["op"].startswith("copy")]
    if big:
        print(json.dumps({"model": a.model, "batch": a.batch, "passes": len(rows),
                          "mean_pct_peak_ge64MB": round(sum(r["pct_peak"] for r in big) / len(big), 1)}))
    return rows


if __name__ == "__main__":
    main()
