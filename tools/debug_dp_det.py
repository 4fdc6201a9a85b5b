"""Gradient determinism / DP-segment check on one GPU: first-step gradients of ResNet-18-tiny
from graph/eager runs with and without an RCCL world-1 process group, compared per arena spec."""
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dcnn_amd.models import zoo  # noqa: E402
from dcnn_amd.nn import Adam, LossFactory  # noqa: E402
from dcnn_amd.parallel.dp import DataParallel  # noqa: E402
from dcnn_amd.runtime.step import TrainStep  # noqa: E402


def run(graph, bucket_mb=4.0):
    m = zoo.create_model("resnet18_tiny_imagenet")
    m.set_seed(5)
    m.set_device("GPU:0")
    m.initialize()
    m.set_first_layer_input_grad(False)
    dp = DataParallel(m, bucket_mb=bucket_mb)
    opt = Adam(1e-3)
    opt.attach(m)
    st = TrainStep(dp, LossFactory.create("softmax_crossentropy"), opt, use_graph=graph)
    g = torch.Generator().manual_seed(11)
    x = torch.randn(32, 3, 64, 64, generator=g).cuda()
    y = torch.randint(0, 200, (32,), generator=g).cuda()
    loss = float(st(x, y))
    torch.cuda.synchronize()
    return m, m.arena.grad.cpu().clone(), loss


def report(name, ref_m, ref, g, loss):
    a = ref_m.arena
    worst = []
    for k, s in enumerate(a.specs):
        n = torch.Size(s.shape).numel()
        if n < 4096:
            continue
        lo = a.offsets[k]
        r, t = ref[lo:lo + n], g[lo:lo + n]
        worst.append((float((r - t).norm() / r.norm().clamp_min(1e-30)), k, tuple(s.shape)))
    worst.sort(reverse=True)
    print(f"{name}: loss={loss:.6f} rel-norm diff per weight spec (top 8): "
          + ", ".join(f"#{k}{sh}={rel:.2e}" for rel, k, sh in worst[:8]), flush=True)


torch.cuda.set_device(0)
mA, A, lA = run(False)
print(f"A eager nopg loss={lA:.6f}", flush=True)
for name, graph in (("B eager nopg", False), ("C graph nopg", True), ("C2 graph nopg", True)):
    _, g, l = run(graph)
    report(name, mA, A, g, l)
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29541")
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
for name, graph in (("D graph pg", True), ("E eager pg", False), ("F graph pg 1000MB", True)):
    _, g, l = run(graph, 1000.0 if "1000" in name else 4.0)
    report(name, mA, A, g, l)
dist.destroy_process_group()
