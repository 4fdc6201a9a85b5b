"""Run-to-run determinism on one GPU: logits of two forwards and first-step gradients of two
identical eager steps, bf16 and fp32 compute."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dcnn_amd.models import zoo  # noqa: E402
from dcnn_amd.nn import LossFactory  # noqa: E402


def make(dtype):
    m = zoo.create_model("resnet18_tiny_imagenet")
    m.set_seed(5)
    m.set_device("GPU:0")
    if dtype == "fp32":
        m.set_compute_dtype(torch.float32)
    m.initialize()
    m.set_first_layer_input_grad(False)
    return m


torch.cuda.set_device(0)
g = torch.Generator().manual_seed(11)
x = torch.randn(32, 3, 64, 64, generator=g).cuda()
y = torch.randint(0, 200, (32,), generator=g).cuda()
lf = LossFactory.create("softmax_crossentropy")
for dtype in ("bf16", "fp32"):
    m = make(dtype)
    m2 = make(dtype)
    print(dtype, "init params equal:", torch.equal(m.arena.data, m2.arena.data), flush=True)
    o1 = m.forward(x).float().clone()
    o2 = m.forward(x).float().clone()
    print(dtype, "logits rerun max diff", float((o1 - o2).abs().max()), "scale", float(o1.abs().max()), flush=True)
    grads = []
    for k in range(3):
        m.arena.zero_grad()
        out = m.forward(x)
        loss, grad, _ = lf.loss_and_grad(out, y)
        m.backward(grad)
        torch.cuda.synchronize()
        grads.append(m.arena.grad.cpu().clone())
        print(dtype, f"run {k} loss {float(loss):.7f}", flush=True)
    a = m.arena
    for k, s in enumerate(a.specs):
        n = torch.Size(s.shape).numel()
        lo = a.offsets[k]
        r, t, u = grads[0][lo:lo + n], grads[1][lo:lo + n], grads[2][lo:lo + n]
        print(dtype, f"spec {k} {s.name} {tuple(s.shape)} |g|={float(r.norm()):.3e} "
              f"d01={float((r - t).norm() / r.norm().clamp_min(1e-30)):.2e} d02={float((r - u).norm() / r.norm().clamp_min(1e-30)):.2e}",
              flush=True)
