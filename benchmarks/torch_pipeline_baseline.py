#!/usr/bin/env python3
"""Same-box PyTorch comparison for the pipeline BASELINE configs (ResNet-50 Tiny-ImageNet, 4-stage
sync / 8-stage semi-async, 8 micro-batches of 32).

Reference: the reference repo's own PyTorch pipeline scripts (torch/resnet18_pipeline.py:16-130:
model cut into sequential stages placed on devices, micro-batches pushed through stage by stage,
gradients accumulated, one optimizer step per batch; torch/coordinator_tiny_mp.py). This is a
re-statement of that pattern for the ResNet-50-tiny layer stack of `create_resnet50_tiny_imagenet`
with stock PyTorch-ROCm (MIOpen / hipBLASLt kernels, autograd):

* ``--schedule gpipe``: all micro-batch forwards stage by stage, then all backwards (autograd
  retains each micro-batch's graph), one Adam step;
* ``--schedule 1f1b``: the same work with each micro-batch's backward issued right after its
  forward (PyTorch eager has no stage concurrency on one device, so this is the activation-memory
  form of the schedule, not a speed trick);
* stages go round-robin on the visible GPUs (one GPU: every stage on cuda:0, exactly like
  benchmarks/pipeline_bench.py) and activations hop devices with ``.to()``.

Synthetic 64x64 inputs, random labels, random init; ``--mode bf16`` uses autocast + channels_last
(PyTorch's best eager configuration), ``--mode fp32`` the scripts' default precision.

    python benchmarks/torch_pipeline_baseline.py --stages 4 --schedule gpipe --mode bf16
"""
import argparse
import json
import time

import torch
import torch.nn as nn


class Bottleneck(nn.Module):
    def __init__(self, cin, mid, cout, stride):
        super().__init__()
        self.c1, self.b1 = nn.Conv2d(cin, mid, 1, bias=False), nn.BatchNorm2d(mid, eps=1e-3)
        self.c2, self.b2 = nn.Conv2d(mid, mid, 3, stride, 1, bias=False), nn.BatchNorm2d(mid, eps=1e-3)
        self.c3, self.b3 = nn.Conv2d(mid, cout, 1, bias=False), nn.BatchNorm2d(cout, eps=1e-3)
        self.proj = None
        if stride != 1 or cin != cout:
            self.proj = nn.Sequential(nn.Conv2d(cin, cout, 1, stride, bias=False), nn.BatchNorm2d(cout, eps=1e-3))

    def forward(self, x):
        h = torch.relu(self.b1(self.c1(x)))
        h = torch.relu(self.b2(self.c2(h)))
        h = self.b3(self.c3(h))
        return torch.relu(h + (self.proj(x) if self.proj is not None else x))


def resnet50_tiny_layers(ncls=200):
    """The layer list of create_resnet50_tiny_imagenet (units the partitioner may cut between)."""
    layers = [nn.Sequential(nn.Conv2d(3, 64, 3, 1, 1), nn.BatchNorm2d(64), nn.ReLU(), nn.MaxPool2d(3, 2, 1))]
    spec = [(64, 64, 256, 1)] + [(256, 64, 256, 1)] * 2 + [(256, 128, 512, 2)] + [(512, 128, 512, 1)] * 3 \
        + [(512, 256, 1024, 2)] + [(1024, 256, 1024, 1)] * 5 + [(1024, 512, 2048, 2)] + [(2048, 512, 2048, 1)] * 2
    layers += [Bottleneck(*s) for s in spec]
    layers.append(nn.Sequential(nn.AvgPool2d(4, 1), nn.Flatten(), nn.Linear(2048, ncls)))
    return layers


def partition(layers, stages):
    """Contiguous, near-equal layer counts (the reference's naive partitioner)."""
    n = len(layers)
    base, rem = divmod(n, stages)
    out, s = [], 0
    for i in range(stages):
        e = s + base + (1 if i < rem else 0)
        out.append(nn.Sequential(*layers[s:e]))
        s = e
    return out


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--stages", type=int, default=4)
    ap.add_argument("--schedule", default="gpipe", choices=["gpipe", "1f1b"])
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--microbatches", type=int, default=8)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--mode", choices=["fp32", "bf16"], default="bf16")
    a = ap.parse_args(argv)
    torch.backends.cudnn.benchmark = True
    ngpu = torch.cuda.device_count()
    devs = [torch.device("cuda", i % ngpu) for i in range(a.stages)]
    mf = torch.channels_last if a.mode == "bf16" else torch.contiguous_format
    stages = [st.to(d).to(memory_format=mf) for st, d in zip(partition(resnet50_tiny_layers(), a.stages), devs)]
    params = [p for st in stages for p in st.parameters()]
    opt = torch.optim.Adam(params, 1e-3)
    lossf = nn.CrossEntropyLoss()
    x = torch.randn(a.batch, 3, 64, 64, device=devs[0]).to(memory_format=mf)
    y = torch.randint(0, 200, (a.batch,), device=devs[-1])
    xs, ys = x.chunk(a.microbatches), y.chunk(a.microbatches)

    def fwd(mb):
        h = xs[mb]
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=a.mode == "bf16"):
            for st, d in zip(stages, devs):
                h = st(h.to(d, non_blocking=True))
            return lossf(h.float(), ys[mb]) / a.microbatches

    def step():
        opt.zero_grad(set_to_none=True)
        total = 0.0
        if a.schedule == "gpipe":
            losses = [fwd(i) for i in range(a.microbatches)]
            for l in losses:
                l.backward()
            total = sum(l.detach() for l in losses)
        else:
            for i in range(a.microbatches):
                l = fwd(i)
                l.backward()
                total = total + l.detach()
        opt.step()
        return total

    for _ in range(a.warmup):
        step()
    for d in set(devs):
        torch.cuda.synchronize(d)
    t0 = time.perf_counter()
    for _ in range(a.steps):
        loss = step()
    for d in set(devs):
        torch.cuda.synchronize(d)
    dt = time.perf_counter() - t0
    res = {"framework": "pytorch-rocm " + torch.__version__, "metric": "pipeline images/sec resnet50_tiny_imagenet",
           "value": round(a.batch * a.steps / dt, 1), "unit": "images/sec", "stages": a.stages,
           "gpus": ngpu, "schedule": a.schedule, "microbatches": a.microbatches, "batch": a.batch,
           "ms_per_step": round(dt / a.steps * 1e3, 3), "mode": a.mode, "data": "synthetic",
           "loss": round(float(loss), 4)}
    print(json.dumps(res), flush=True)
    return res


if __name__ == "__main__":
    main()
