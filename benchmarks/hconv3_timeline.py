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
    ap.add_argument("--shapes", default="l1.c,l2.c")
    ap.add_argument("--op", default="fwd", choices=["fwd", "dgrad"])
    a = ap.parse_args()
    from dcnn_amd.ops import hip
    K = hip.kernels()
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
            items = K.hconv_tiles(N, H, W, C, Co, 9) * K.hconv_splits(N, H, W, C, Co, 9)
        else:
            fn = lambda: hip.conv2d_dgrad(dy, wt, x.shape, (1, 1), (1, 1))
            items = K.hconv_tiles(N, H, W, Co, C, 9) * K.hconv_splits(N, H, W, Co, C, 9)
        # per item u and wave: [0] item start, [1] first chunk done, [2] K loop done, [3] epilogue
        # computed + stored, [4] item end (statistics merged); [5] workgroup start (first item)
        buf = torch.zeros(items * 4 * 8, dtype=torch.int64, device="cuda")
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        K.hconv3_set_stamps(buf.data_ptr())
        fn()
        torch.cuda.synchronize()
        K.hconv3_set_stamps(0)
        t = buf.view(items, 4, 8).double().cpu()
        t0 = t[:, :, 0][t[:, :, 0] > 0].min()
        kloop = (t[:, :, 2] - t[:, :, 0]).sum()
        epi = (t[:, :, 4] - t[:, :, 2]).sum()
        first = t[:, :, 5] > 0
        # a wave's life: from its workgroup's start to its last item's end; items of one workgroup
        # are the ones whose start stamp falls inside it (grid-strided), summed over all waves
        life_end = t[:, :, 4].max()
        per_item = {"kloop": t[:, :, 2] - t[:, :, 0], "chunk0": t[:, :, 1] - t[:, :, 0],
                    "epilogue": t[:, :, 3] - t[:, :, 2], "stats": t[:, :, 4] - t[:, :, 3]}
        prologue = (t[:, :, 0] - t[:, :, 5])[first]
        span = float(life_end - t0)
        wg = int(first.sum()) // 4
        print(f"{nm} {a.op} batch {N}: {items} items on {wg} workgroups, span {span:.0f} cyc; "
              f"K loop share of item time {float(kloop / (kloop + epi)) * 100:.1f}%, "
              f"of wave life {float(kloop / ((t[:, :, 4].max() - t0) * 4 * wg)) * 100:.1f}%")
        print("   medians per item: " + "  ".join(f"{k} {float(v.median()):.0f}" for k, v in per_item.items())
              + f"  prologue {float(prologue.median()):.0f}")


if __name__ == "__main__":
    main()
