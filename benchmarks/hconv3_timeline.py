#!/usr/bin/env python3
"""Per-wave phase timeline of the hconv3 kernel (diagnostic s_memtime stamps, hconv3_set_stamps):
prologue (halo + first weight stages landed), first chunk, remaining K loop, epilogue stores,
statistics — medians over waves, in shader cycles, and the K loop's share of each wave's life
(s_memtime counts per XCD, so only same-wave stamp differences are used).

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
        buf = torch.zeros(items * 4 * 16, dtype=torch.int64, device="cuda")
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        K.hconv3_set_stamps(buf.data_ptr())
        fn()
        torch.cuda.synchronize()
        K.hconv3_set_stamps(0)
        t = buf.view(items, 4, 16).double().cpu()
        # s_memtime is a per-XCD counter: only differences of stamps taken by the SAME wave are
        # meaningful (cross-workgroup spans mix clocks). Split-K items that are not their tile's
        # last arriver skip the epilogue stamps (3, 4): those phases use only the items that ran it.
        ok = lambda *ks: torch.stack([t[:, :, k] > 0 for k in ks]).all(0)
        per_item = {}
        for name, a_, b_ in (("kloop", 0, 2), ("chunk0", 0, 1), ("epilogue", 2, 3), ("stats", 3, 4)):
            m = ok(a_, b_)
            per_item[name] = (t[:, :, b_] - t[:, :, a_])[m]
        first = t[:, :, 5] > 0
        G = int(first[:, 0].sum())  # workgroups (each stamps 5 once, at its first item)
        # prologue split. 16 x 16+ maps (l1-l3): [5] -> [8] arguments, [8] -> [10] weight table,
        # [10] -> [9] weight addresses + W(0, 0) DMA issue + halo table, [9] -> [6] halo addresses,
        # [6] -> [11] halo / W(0, 1) issue + fragment addresses, [11] -> [7] first DMA landing
        # (vmcnt), [7] -> [0] first barrier. The 4 x 4-map gutter layout (l4) keeps the older order
        # [5] args [8] halo table [9] weight table [10] fragment addresses [11] addresses [6] DMA [7].
        seq = ((("args", 5, 8), ("w_tab", 8, 10), ("w_dma+halo_tab", 10, 9), ("addrs_h", 9, 6),
                ("issue+frag", 6, 11), ("dma", 11, 7), ("barrier", 7, 0)) if H > 4 else
               (("args", 5, 8), ("halo_tab", 8, 9), ("w_tab", 9, 10), ("frag", 10, 11), ("addrs", 11, 6),
                ("dma", 6, 7), ("barrier", 7, 0)))
        pro = {nm_: (t[:, :, b_] - t[:, :, a_])[first & ok(a_, b_)] for nm_, a_, b_ in seq}
        lives, kl, prol = [], [], []
        for u0 in torch.nonzero(first[:, 0]).flatten().tolist():
            us = list(range(u0, items, G))
            for w in range(4):
                start_ = t[u0, w, 5]
                ends = [t[u, w, 4] if t[u, w, 4] > 0 else t[u, w, 2] for u in us]
                lives.append(max(ends) - start_)
                kl.append(sum(t[u, w, 2] - t[u, w, 0] for u in us))
                prol.append(t[u0, w, 0] - start_)
        lives, kl, prol = torch.tensor(lives), torch.tensor(kl), torch.tensor(prol)
        kloop_sum = float(per_item["kloop"].sum())
        epi_sum = float(per_item["epilogue"].sum() + per_item["stats"].sum())
        print(f"{nm} {a.op} batch {N}: {items} items on {G} workgroups; median wave life {float(lives.median()):.0f} cyc; "
              f"K loop share of wave life {100 * float(kl.sum() / lives.sum()):.1f}%, "
              f"of item time (items with an epilogue) {100 * kloop_sum / max(kloop_sum + epi_sum, 1):.1f}%")
        print("   medians per item: " + "  ".join(f"{k} {float(v.median()):.0f}" if v.numel() else f"{k} -"
                                               for k, v in per_item.items())
              + f"  prologue {float(prol.median()):.0f} (" + "  ".join(
                  f"{k} {float(v.median()):.0f}" for k, v in pro.items() if v.numel()) + ")")

if __name__ == "__main__":
    main()
