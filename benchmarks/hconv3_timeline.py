#!/usr/bin/env python3
"""Per-wave phase timeline of the hconv3 kernel (diagnostic s_memtime stamps, hconv3_set_stamps):
prologue (halo + first weight stages landed), first chunk, remaining K loop, epilogue stores,
statistics — medians over waves, in shader cycles, plus dispatch skew and the span of the grid.

  python benchmarks/hconv3_timeline.py --batch 256 --shapes l1.c,l2.c
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = {"l1.c": (64, 32, 32, 64), "l2.c": (128, 16, 16, 128), "l3.c": (256, 8, 8, 256), "l4.c": (512, 4, 4, 512)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--shapes", default="l1.c,l2.c,l3.c,l4.c")
    ap.add_argument("--op", default="fwd", choices=["fwd", "dgrad"])
    ap.add_argument("--stagger", type=int, default=-1)
    a = ap.parse_args()
    from dcnn_amd.ops import hip
    K = hip.kernels()
    if a.stagger >= 0:
        K.hconv3_set_stagger(a.stagger)
    CL = torch.channels_last
    N = a.batch
    for nm in a.shapes.split(","):
        C, H, W, Co = SHAPES[nm]
        x = torch.randn(N, C, H, W, device="cuda").bfloat16().contiguous(memory_format=CL)
        w = (torch.randn(Co, C, 3, 3, device="cuda") * 0.05).bfloat16().contiguous(memory_format=CL)
        dy = torch.randn(N, Co, H, W, device="cuda").bfloat16().contiguous(memory_format=CL)
        wt = hip.conv_weight_t(w)
        if a.op == "fwd":
            fn = lambda: hip.conv2d_fwd(x, w, None, (1, 1), (1, 1), stats=True)
            grid = K.hconv_tiles(N, H, W, C, Co, 9) * K.hconv_splits(N, H, W, C, Co, 9)
        else:
            fn = lambda: hip.conv2d_dgrad(dy, wt, x.shape, (1, 1), (1, 1))
            grid = K.hconv_tiles(N, H, W, Co, C, 9) * K.hconv_splits(N, H, W, Co, C, 9)
        buf = torch.zeros(grid * 8 * 8, dtype=torch.int64, device="cuda")
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        K.hconv3_set_stamps(buf.data_ptr())
        fn()
        torch.cuda.synchronize()
        K.hconv3_set_stamps(0)
        raw = buf.view(grid, 8, 8).cpu()
        arr = raw[:, 0, 6]
        if int(arr.abs().sum()) != 0:
            # stagger diagnostics: workgroups per hardware CU key, arrival index histogram
            keys = (arr >> 8).tolist()
            olds = (arr & 0xff).tolist()
            per = {}
            for kk in keys:
                per[kk] = per.get(kk, 0) + 1
            hist = {}
            for o in olds:
                hist[o] = hist.get(o, 0) + 1
            print(f"   stagger: {len(per)} CU keys, workgroups/key min {min(per.values())} max {max(per.values())}, "
                  f"arrival index histogram {dict(sorted(hist.items()))}")
            raw[:, 0, 6] = 0
        t = raw.view(grid * 8, 8).double()
        live = t[:, 0] > 0
        t = t[live]
        t0 = t[:, 0].min()
        ph = {"prologue": t[:, 1] - t[:, 0], "chunk0": t[:, 2] - t[:, 1], "kloop_rest": t[:, 3] - t[:, 2],
              "epilogue": t[:, 4] - t[:, 3], "stats": t[:, 5] - t[:, 4], "wave_total": t[:, 5] - t[:, 0]}
        print(f"{nm} {a.op} batch {N}: grid {grid}, waves stamped {int(live.sum())}, "
              f"span {float(t[:, 5].max() - t0):.0f} cyc, start skew p50/p90/max "
              f"{float((t[:, 0] - t0).median()):.0f}/{float((t[:, 0] - t0).quantile(0.9)):.0f}/"
              f"{float((t[:, 0] - t0).max()):.0f}")
        print("   " + "  ".join(f"{k} {float(v.median()):.0f}" for k, v in ph.items()))


if __name__ == "__main__":
    main()
