#!/usr/bin/env python3
"""BatchNorm-fold experiment: what folding a BatchNorm + ReLU apply into the consuming 3x3 conv
costs in the conv and what it saves.

The fold variant of hconv3 (``hconv3_set_input_affine``, the AIN instance) reads the stored BN
input y and applies relu(scale * y + shift) to each halo chunk in LDS, in the lanes that DMA'd it,
before the chunk is published; the unfused path is bn_apply (writes a = relu(bn(y))) + hconv3 on a.
Per ResNet-18 3x3 shape, batch 256, hipGraph replays of 20 launches each:

  conv          hconv3 forward with BN statistics on a stored activation
  conv+fold     the same launch reading y and applying the affine + ReLU in LDS
  bn_apply      the apply pass the fold removes (reads y, writes a)

and the numerical check conv+fold(y) == conv(relu(scale * y + shift)) (bf16 rounding of a).

  python benchmarks/bn_fold_probe.py --shapes l1.c,l2.c,l3.c
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = {"l1.c": (64, 32, 32), "l2.c": (128, 16, 16), "l3.c": (256, 8, 8)}


def timed(fn, reps=20):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()  # (warm: instances, workspaces)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(3):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / (3 * reps)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--shapes", default="l1.c,l2.c,l3.c")
    a = ap.parse_args()
    from dcnn_amd.ops import hip
    K = hip.kernels()
    CL = torch.channels_last
    N = a.batch
    rows = []
    for nm in a.shapes.split(","):
        C, H, W = SHAPES[nm]
        g = torch.Generator(device="cuda").manual_seed(0)
        y = torch.randn(N, C, H, W, device="cuda", generator=g).bfloat16().contiguous(memory_format=CL)
        w = (torch.randn(C, C, 3, 3, device="cuda", generator=g) * 0.05).bfloat16().contiguous(memory_format=CL)
        scale = (torch.rand(C, device="cuda", generator=g) + 0.5)
        shift = torch.randn(C, device="cuda", generator=g) * 0.2
        aff = torch.cat([scale, shift]).float().contiguous()
        act = torch.relu(y.float() * scale.view(1, C, 1, 1) + shift.view(1, C, 1, 1)).bfloat16().contiguous(memory_format=CL)
        mean = -shift / scale  # bn_apply with gamma = 1, beta = 0, var chosen so istd = scale
        var = 1.0 / (scale * scale) - 1e-5
        sums = torch.cat([mean, var]).float().contiguous()

        t_conv = timed(lambda: hip.conv2d_fwd(act, w, None, (1, 1), (1, 1), stats=True))
        ref, _ = hip.conv2d_fwd(act, w, None, (1, 1), (1, 1), stats=True)
        K.hconv3_set_input_affine(aff.data_ptr())
        try:
            t_fold = timed(lambda: hip.conv2d_fwd(y, w, None, (1, 1), (1, 1), stats=True))
            out, _ = hip.conv2d_fwd(y, w, None, (1, 1), (1, 1), stats=True)
            torch.cuda.synchronize()
        finally:
            K.hconv3_set_input_affine(0)
        t_apply = timed(lambda: hip.bn_apply(y, sums, N * H * W, None, None, 1e-5, relu=True))
        err = float((out.float() - ref.float()).abs().max() / ref.float().abs().max())
        rows.append(dict(shape=nm, conv_us=round(t_conv, 2), conv_fold_us=round(t_fold, 2),
                         fold_cost_us=round(t_fold - t_conv, 2), bn_apply_us=round(t_apply, 2),
                         net_saving_us=round(t_apply - (t_fold - t_conv), 2), max_rel_err=err))
        print(json.dumps(rows[-1]), flush=True)


if __name__ == "__main__":
    main()
