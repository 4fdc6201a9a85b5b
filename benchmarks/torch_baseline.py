#!/usr/bin/env python3
"""Comparison point from BASELINE.md: the reference repo's own PyTorch ResNet-18-tiny training
script architecture (torch/torch_tiny_imagenet_trainer.py:111, same layer stack as
create_resnet18_tiny_imagenet) run with stock PyTorch-ROCm (MIOpen/hipBLASLt kernels) on the
same MI355X, synthetic data, Adam, cross-entropy. Modes: fp32 NCHW (the script's default) and
bf16 autocast + channels_last (PyTorch's best eager configuration).

``--model resnet9_cifar10`` runs the same comparison for the CIFAR-10 ResNet-9 BASELINE config
(the layer stack of create_resnet9_cifar10, reference examples/cifar10_resnet9.cpp:20-79).

  python benchmarks/torch_baseline.py --batch 256 --steps 20 --warmup 5 --mode bf16
  python benchmarks/torch_baseline.py --model resnet9_cifar10 --batch 128 --mode fp32
"""
import argparse
import json
import time

import torch
import torch.nn as nn


class Block(nn.Module):
    def __init__(self, cin, cout, stride):
        super().__init__()
        self.c1 = nn.Conv2d(cin, cout, 3, stride, 1, bias=True)
        self.b1 = nn.BatchNorm2d(cout)
        self.c2 = nn.Conv2d(cout, cout, 3, 1, 1, bias=True)
        self.b2 = nn.BatchNorm2d(cout)
        self.proj = None
        if stride != 1 or cin != cout:
            self.proj = nn.Sequential(nn.Conv2d(cin, cout, 1, stride, 0, bias=False), nn.BatchNorm2d(cout))

    def forward(self, x):
        h = torch.relu(self.b1(self.c1(x)))
        h = self.b2(self.c2(h))
        return torch.relu(h + (self.proj(x) if self.proj is not None else x))


class ResNet18Tiny(nn.Module):
    def __init__(self, ncls=200):
        super().__init__()
        self.stem = nn.Sequential(nn.Conv2d(3, 32, 3, 1, 1, bias=False), nn.BatchNorm2d(32, eps=1e-3), nn.ReLU(),
                                  nn.MaxPool2d(2, 2))
        chans = [(32, 64, 1), (64, 64, 1), (64, 128, 2), (128, 128, 1), (128, 256, 2), (256, 256, 1), (256, 512, 2),
                 (512, 512, 1)]
        self.blocks = nn.Sequential(*[Block(a, b, s) for a, b, s in chans])
        self.pool = nn.AvgPool2d(4, 1)
        self.fc = nn.Linear(512, ncls)

    def forward(self, x):
        return self.fc(torch.flatten(self.pool(self.blocks(self.stem(x))), 1))


class ResBlock(nn.Module):
    """Basic residual block with identity shortcut (cin == cout, stride 1)."""

    def __init__(self, c):
        super().__init__()
        self.c1, self.b1 = nn.Conv2d(c, c, 3, 1, 1), nn.BatchNorm2d(c)
        self.c2, self.b2 = nn.Conv2d(c, c, 3, 1, 1), nn.BatchNorm2d(c)

    def forward(self, x):
        h = torch.relu(self.b1(self.c1(x)))
        return torch.relu(self.b2(self.c2(h)) + x)


def _cbr(cin, cout):
    return [nn.Conv2d(cin, cout, 3, 1, 1), nn.BatchNorm2d(cout), nn.ReLU()]


class ResNet9Cifar(nn.Module):
    def __init__(self, ncls=10):
        super().__init__()
        self.body = nn.Sequential(*_cbr(3, 64), *_cbr(64, 128), nn.MaxPool2d(2, 2), ResBlock(128), ResBlock(128),
                                  *_cbr(128, 256), nn.MaxPool2d(2, 2), ResBlock(256), ResBlock(256),
                                  *_cbr(256, 512), nn.MaxPool2d(2, 2), ResBlock(512), nn.AvgPool2d(4, 1))
        self.fc = nn.Linear(512, ncls)

    def forward(self, x):
        return self.fc(torch.flatten(self.body(x), 1))


MODELS = {"resnet18_tiny_imagenet": (ResNet18Tiny, (3, 64, 64), 200), "resnet9_cifar10": (ResNet9Cifar, (3, 32, 32), 10)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--mode", choices=["fp32", "bf16"], default="bf16")
    ap.add_argument("--model", choices=sorted(MODELS), default="resnet18_tiny_imagenet")
    a = ap.parse_args()
    torch.backends.cudnn.benchmark = True
    dev = torch.device("cuda")
    cls, shape, ncls = MODELS[a.model]
    m = cls().to(dev)
    mf = torch.channels_last if a.mode == "bf16" else torch.contiguous_format
    m = m.to(memory_format=mf)
    opt = torch.optim.Adam(m.parameters(), 1e-3)
    lossf = nn.CrossEntropyLoss()
    xs = [torch.randn(a.batch, *shape, device=dev).to(memory_format=mf) for _ in range(4)]
    ys = [torch.randint(0, ncls, (a.batch,), device=dev) for _ in range(4)]

    def step(i):
        opt.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=a.mode == "bf16"):
            loss = lossf(m(xs[i % 4]), ys[i % 4])
        loss.backward()
        opt.step()
        return loss

    for i in range(a.warmup):
        step(i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(a.steps):
        loss = step(i)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    print(json.dumps({"framework": "pytorch-rocm " + torch.__version__, "model": a.model, "mode": a.mode, "batch": a.batch,
                      "images_per_sec": round(a.batch * a.steps / el, 1), "ms_per_step": round(el / a.steps * 1e3, 3),
                      "loss": round(float(loss), 4)}))


if __name__ == "__main__":
    main()
