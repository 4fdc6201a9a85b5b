"""Teacher-forced per-layer GPU vs bf16-emulated CPU comparison: every GPU layer gets the CPU
reference's input activation and output gradient, so errors do not compound across layers."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from test_gpu_model import bf16_emulate  # noqa: E402

from dcnn_amd.models import INPUT_SHAPES, NUM_CLASSES, create_model  # noqa: E402
from dcnn_amd.nn import LossFactory  # noqa: E402


def rel(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


name = sys.argv[1] if len(sys.argv) > 1 else "resnet18_tiny_imagenet"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 16
torch.manual_seed(0)
C, H, W = INPUT_SHAPES[name]
x = torch.randn(B, C, H, W)
y = torch.randint(0, NUM_CLASSES[name], (B,))
cpu = create_model(name)
cpu.set_seed(3)
cpu.initialize()
gpu = create_model(name)
gpu.set_seed(3)
gpu.set_device("GPU:0")
gpu.initialize()
bf16_emulate(cpu)
acts = [x]
for l in cpu.layers:
    acts.append(l.forward(acts[-1]))
lf = LossFactory.create("softmax_crossentropy")
_, g, _ = lf.loss_and_grad(acts[-1], y)
grads = [None] * len(cpu.layers)
for i in range(len(cpu.layers) - 1, -1, -1):
    grads[i] = g  # gradient wrt output of layer i
    g = cpu.layers[i].backward(g)
# re-run CPU per layer to get reference param grads per layer (fresh grads)
cpu.clear_gradients()
ref = []
for i, l in enumerate(cpu.layers):
    l.forward(acts[i])
    dx = l.backward(grads[i])
    ref.append((dx, [p.clone() for p in l.gradients()]))
for i, l in enumerate(gpu.layers):
    out = l.forward(acts[i].cuda())
    dx = l.backward(grads[i].cuda())
    dxr, pr = ref[i]
    pe = [f"{rel(b, a):.3f}" for a, b in zip(pr, l.gradients())]
    fwd = rel(out, acts[i + 1]) if not (hasattr(l, "fuse_relu") and l.fuse_relu) else rel(out, torch.relu(acts[i + 1]))
    print(f"{i:2d} {l.name:<16} fwd={fwd:.4f} dx={rel(dx, dxr) if dx is not None else -1:.4f} params {pe}")
