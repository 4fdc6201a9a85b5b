"""Per-layer teacher-forced GPU-vs-CPU errors of the PYTHON front end against a plain fp32 CPU
reference (no bf16 emulation): the bf16 noise floor of a block's input gradient, to compare with
the C++ engine's numbers (host_api_parity blocks)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from dcnn_amd.models import INPUT_SHAPES, NUM_CLASSES, create_model
from dcnn_amd.nn import LossFactory
from dcnn_amd.nn.layers import Activation, BatchNorm

def rel(a, b):
    a, b = a.double().cpu().reshape(-1), b.double().cpu().reshape(-1)
    return float((a - b).norm() / b.norm().clamp_min(1e-30))

name = sys.argv[1] if len(sys.argv) > 1 else "resnet18_tiny_imagenet"
torch.manual_seed(0)
C, H, W = INPUT_SHAPES[name]
B = int(sys.argv[2]) if len(sys.argv) > 2 else 64
x = torch.randn(B, C, H, W)
y = torch.randint(0, NUM_CLASSES[name], (B,))
cpu = create_model(name); cpu.set_seed(3); cpu.initialize()
gpu = create_model(name); gpu.set_seed(3); gpu.set_device("GPU:0"); gpu.initialize()
for l in gpu.layers:
    if isinstance(l, BatchNorm):
        l.fuse_pool = None
acts = [x]
for l in cpu.layers:
    acts.append(l.forward(acts[-1]))
_, g, _ = LossFactory.create("softmax_crossentropy").loss_and_grad(acts[-1], y)
grads = [None] * len(cpu.layers)
for i in range(len(cpu.layers) - 1, -1, -1):
    grads[i] = g
    g = cpu.layers[i].backward(g)
for i, (lc, lg) in enumerate(zip(cpu.layers, gpu.layers)):
    if isinstance(lg, Activation) and lg.passthrough:
        continue
    nxt_relu = isinstance(lg, BatchNorm) and lg.fuse_relu
    lc.forward(acts[i])
    dxc = lc.backward(grads[i] * (acts[i + 1] > 0) if nxt_relu else grads[i])
    out = lg.forward(acts[i].cuda())
    dxg = lg.backward(grads[i].cuda())
    ref = torch.relu(acts[i + 1]) if nxt_relu else acts[i + 1]
    e_dx = rel(dxg, dxc) if (dxc is not None and dxg is not None) else float("nan")
    print(f"{lg.name:16s} fwd {rel(out, ref):.4f} dx {e_dx:.4f}", flush=True)
