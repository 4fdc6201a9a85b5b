#!/usr/bin/env python3
"""Per-shape microbenchmark of the implicit-GEMM conv kernels (fwd / dgrad / wgrad) on the
ResNet-18-tiny layer shapes. Reports device time per call and achieved TFLOP/s.

  python benchmarks/conv_bench.py --batch 256 [--only fwd|dgrad|wgrad] [--iters 20]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# (name, Ci, H, W, Co, k, s, p)
SHAPES = [
    ("stem", 3, 64, 64, 32, 3, 1, 1),
    ("l1.b1c1", 32, 32, 32, 64, 3, 1, 1),
    ("l1.c", 64, 32, 32, 64, 3, 1, 1),
    ("l1.proj", 32, 32, 32, 64, 1, 1, 0),
    ("l2.b1c1", 64, 32, 32, 128, 3, 2, 1),
    ("l2.c", 128, 16, 16, 128, 3, 1, 1),
    ("l2.proj", 64, 32, 32, 128, 1, 2, 0),
    ("l3.b1c1", 128, 16, 16, 256, 3, 2, 1),
    ("l3.c", 256, 8, 8, 256, 3, 1, 1),
    ("l3.proj", 128, 16, 16, 256, 1, 2, 0),
    ("l4.b1c1", 256, 8, 8, 512, 3, 2, 1),
    ("l4.c", 512, 4, 4, 512, 3, 1, 1),
    ("l4.proj", 256, 8, 8, 512, 1, 2, 0),
]

# ResNet-50-tiny bottleneck shapes (64x64 input, stride-2 max-pool stem: layer 1 at 32x32);
# --set r50 (include/nn/example_models.hpp:369-402 block structure)
SHAPES_R50 = [
    ("r1.c1a", 64, 32, 32, 64, 1, 1, 0),     # layer1_block1 1x1 reduce (64 in)
    ("r1.c1", 256, 32, 32, 64, 1, 1, 0),     # layer1 1x1 reduce
    ("r1.c2", 64, 32, 32, 64, 3, 1, 1),      # layer1 3x3
    ("r1.c3", 64, 32, 32, 256, 1, 1, 0),     # layer1 1x1 expand
    ("r2.c1", 512, 16, 16, 128, 1, 1, 0),
    ("r2.c2", 128, 16, 16, 128, 3, 1, 1),
    ("r2.c3", 128, 16, 16, 512, 1, 1, 0),
    ("r2.s2", 128, 32, 32, 128, 3, 2, 1),    # layer2_block1 strided 3x3
    ("r2.proj", 256, 32, 32, 512, 1, 2, 0),
    ("r3.c1", 1024, 8, 8, 256, 1, 1, 0),
    ("r3.c2", 256, 8, 8, 256, 3, 1, 1),
    ("r3.c3", 256, 8, 8, 1024, 1, 1, 0),
    ("r4.c1", 2048, 4, 4, 512, 1, 1, 0),
    ("r4.c2", 512, 4, 4, 512, 3, 1, 1),
    ("r4.c3", 512, 4, 4, 2048, 1, 1, 0),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--only", default="")
    ap.add_argument("--shapes", default="", help="comma-separated shape names (default: all)")
    ap.add_argument("--set", default="r18", choices=["r18", "r50"], help="ResNet-18-tiny or ResNet-50-tiny shapes")
    ap.add_argument("--v3", type=int, default=1, help="third-generation 3x3 halo conv (hconv3.hip) on/off")
    ap.add_argument("--eager", action="store_true", help="time eager launches instead of one hipGraph replay")
    ap.add_argument("--halo-1x1", type=int, default=1, help="K >= 1024 1x1 convs on the halo kernel (ops/fusion.py)")
    ap.add_argument("--torch-mm", action="store_true",
                    help="also time the 1x1 shapes' plain GEMMs on torch.mm (hipBLASLt; no fused statistics)")
    ap.add_argument("--hwgrad-s2", type=int, default=None, help="3x3 stride-2 wgrad on the stride-2 halo kernel (ops/fusion.py)")
    ap.add_argument("--split-target", type=int, default=None, help="hconv split-K workgroup target (tuning hook)")
    ap.add_argument("--split-min-work", type=int, default=None, help="hconv least taps x chunks per split")
    ap.add_argument("--bnb", action="store_true",
                    help="dgrad with the production epilogue: the consuming BatchNorm's ReLU mask (y) and "
                         "backward statistics (x, mean, istd) fused in (BnbRequest)")
    ap.add_argument("--no-group", action="store_true", help="strided dgrad phases as separate launches")
    a = ap.parse_args()
    from dcnn_amd.ops import hip, fusion
    if a.split_target is not None:
        hip.kernels().hconv_set_split_target(a.split_target)
    if a.split_min_work is not None:
        hip.kernels().hconv_set_split_min_work(a.split_min_work)
    hip.kernels().hconv3_enable(a.v3)
    fusion.HCONV_1X1 = bool(a.halo_1x1)
    if a.no_group:
        fusion.G2_GROUP = False
    if a.hwgrad_s2 is not None:
        fusion.HWGRAD_S2 = bool(a.hwgrad_s2)
    CL = torch.channels_last
    N = a.batch
    tot = {"fwd": 0.0, "dgrad": 0.0, "wgrad": 0.0}
    print(f"{'shape':<10}{'op':<7}{'us':>9}{'TFLOP/s':>9}{'TB/s':>7}")
    keep = set(a.shapes.split(",")) if a.shapes else None
    for (nm, Ci, H, W, Co, k, s, p) in (SHAPES_R50 if a.set == "r50" else SHAPES):
        if keep is not None and nm not in keep:
            continue
        x = torch.randn(N, Ci, H, W, device="cuda").bfloat16().contiguous(memory_format=CL)
        w = (torch.randn(Co, Ci, k, k, device="cuda") * 0.05).bfloat16().contiguous(memory_format=CL)
        wf = w
        if Ci < 8:  # the RGB stem runs channel-padded to 8 (as Conv2D does)
            x = hip.to_act_padded(x.float().contiguous(), 8)
            wf = hip.pad_weight_channels(w, 8)
        OH, OW = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
        dy = torch.randn(N, Co, OH, OW, device="cuda").bfloat16().contiguous(memory_format=CL)
        gw = torch.zeros(Co, Ci, k, k, device="cuda").contiguous(memory_format=CL)
        wt = hip.conv_weight_t(w)
        flops = 2.0 * N * OH * OW * Co * Ci * k * k
        # compulsory HBM bytes (bf16 operands read once, result written once; wgrad: fp32 result)
        hbm = {"fwd": 2.0 * (N * H * W * Ci + N * OH * OW * Co + Co * Ci * k * k),
               "dgrad": 2.0 * (N * H * W * Ci + N * OH * OW * Co + Co * Ci * k * k),
               "wgrad": 2.0 * (N * H * W * Ci + N * OH * OW * Co) + 4.0 * Co * Ci * k * k}
        bnb = None
        if a.bnb and Ci >= 8:
            # the BatchNorm that produced x: ReLU output y (mask), input xb, saved statistics
            from dcnn_amd.ops.hip_base import BnbRequest
            xb = torch.randn_like(x)
            bnb = BnbRequest(None, torch.relu(xb), xb, torch.zeros(Ci, device="cuda"),
                             torch.ones(Ci, device="cuda"))
            hbm["dgrad"] += 4.0 * N * H * W * Ci  # y and x read in the epilogue
        ops = {
            "fwd": lambda: hip.conv2d_fwd(x, wf, None, (s, s), (p, p), stats=True),
            "dgrad": lambda: hip.conv2d_dgrad(dy, wt, x.shape, (s, s), (p, p), bnb=bnb),
            "wgrad": lambda: hip.conv2d_wgrad(dy, x, w.shape, (s, s), (p, p), gw, None),
        }
        if a.torch_mm and k == 1 and s == 1:
            xm, dym = x.permute(0, 2, 3, 1).reshape(-1, Ci), dy.permute(0, 2, 3, 1).reshape(-1, Co)  # NHWC rows (views)
            w2 = w.reshape(Co, Ci)
            ops["mm_fwd"] = lambda: torch.mm(xm, w2.t())
            ops["mm_dgrad"] = lambda: torch.mm(dym, w2)
            ops["mm_wgrad"] = lambda: torch.mm(dym.t(), xm)
            for o in ("mm_fwd", "mm_dgrad", "mm_wgrad"):
                hbm[o] = hbm[o[3:]]
                tot.setdefault(o, 0.0)
        for op, fn in ops.items():
            if a.only and op.replace("mm_", "") != a.only:
                continue
            if op == "dgrad" and nm == "stem":
                continue
            for _ in range(3):
                fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            if a.eager:
                e0.record()
                for _ in range(a.iters):
                    fn()
                e1.record()
            else:
                # device time without host launch overhead: the calls captured into one graph
                g = torch.cuda.CUDAGraph()
                s_ = torch.cuda.Stream()
                s_.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(s_):
                    with torch.cuda.graph(g, stream=s_):
                        for _ in range(a.iters):
                            fn()
                torch.cuda.current_stream().wait_stream(s_)
                g.replay()
                torch.cuda.synchronize()
                e0.record()
                g.replay()
                e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1000 / a.iters
            tot[op] += us
            print(f"{nm:<10}{op:<7}{us:9.1f}{flops / us / 1e6:9.1f}{hbm[op] / us / 1e6:7.2f}")
    print("totals (us, one pass over the shapes):", {k: round(v, 1) for k, v in tot.items()})


if __name__ == "__main__":
    main()
