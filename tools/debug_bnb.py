#!/usr/bin/env python3
"""Debug helper: whole-model gradients with the backward-BN epilogue fusion on vs off, reported
per parameter tensor (last layer first) so the first diverging layer is visible."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from dcnn_amd.models import INPUT_SHAPES, NUM_CLASSES, create_model
    from dcnn_amd.nn import LossFactory
    from dcnn_amd.nn.sequential import _leaf_param_layers
    from dcnn_amd.ops import hip
    name = sys.argv[1] if len(sys.argv) > 1 else "resnet18_tiny_imagenet"
    torch.manual_seed(4)
    C, H, W = INPUT_SHAPES[name]
    x = torch.randn(16, C, H, W, device="cuda")
    y = torch.randint(0, NUM_CLASSES[name], (16,), device="cuda")
    lf = LossFactory.create("softmax_crossentropy")
    res = {}
    names = []
    for fuse in ("off", "off2", "on", "on2"):
        hip._BNB = fuse.startswith("on")
        m = create_model(name)
        m.set_seed(11)
        m.set_device("GPU:0")
        m.initialize()
        out = m.forward(x, return_on_input_device=False)
        _, g, _ = lf.loss_and_grad(out, y)
        m.backward(g)
        torch.cuda.synchronize()
        res[fuse] = [t.float().cpu().clone() for t in m.gradients()]
        if not names:
            for l in _leaf_param_layers(m.layers):
                for s in l.param_specs():
                    names.append(f"{l.name}.{s.name}")
    for j in range(len(res["off"]) - 1, -1, -1):
        a, b, c, d = res["off"][j], res["on"][j], res["off2"][j], res["on2"][j]
        n = max(a.norm().item(), 1e-12)
        e, e0, e1 = (a - b).norm().item() / n, (a - c).norm().item() / n, (b - d).norm().item() / n
        print(f"{j:3d} {names[j] if j < len(names) else '?':40s} |g|={a.norm().item():10.4e} "
              f"fused-vs-unfused={e:.3e} unfused-vs-unfused={e0:.3e} fused-vs-fused={e1:.3e}")


if __name__ == "__main__":
    main()
