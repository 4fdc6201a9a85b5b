"""Shared plumbing of the example trainers (reference examples/*.cpp): .env + TrainingConfig,
device selection, dataset loaders with a synthetic fallback when the dataset directory is
absent (this environment has no network; real data is used whenever it is present)."""
from __future__ import annotations

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from dcnn_amd.data import (SyntheticDataLoader, create_cifar10_loaders, create_cifar100_loaders,  # noqa: E402
                           create_mnist_loaders, create_tiny_image_loader)
from dcnn_amd.nn import TrainingConfig  # noqa: E402
from dcnn_amd.utils import get_env, load_env_file  # noqa: E402

SHAPES = {"mnist": ((1, 28, 28), 10), "cifar10": ((3, 32, 32), 10), "cifar100": ((3, 32, 32), 100),
          "tiny": ((3, 64, 64), 200)}


def parse(description: str, extra=None):
    ap = argparse.ArgumentParser(description=description)
    ap.add_argument("--data", default="./data")
    ap.add_argument("--device", default=None, help="CPU | GPU | GPU:i (default: DEVICE_TYPE env)")
    ap.add_argument("--epochs", type=int, default=None)
    ap.add_argument("--batch-size", type=int, default=None)
    ap.add_argument("--max-batches", type=int, default=0, help="limit batches per epoch (smoke runs)")
    ap.add_argument("--synthetic", type=int, default=0, help="force N synthetic samples instead of the dataset")
    ap.add_argument("--fp32", action="store_true", help="fp32 compute on the GPU (default bf16)")
    if extra:
        extra(ap)
    a = ap.parse_args()
    if load_env_file("./.env") < 0:
        print("No .env file found, using default training parameters.")
    cfg = TrainingConfig().load_from_env()
    if a.epochs is not None:
        cfg.epochs = a.epochs
    if a.batch_size is not None:
        cfg.batch_size = a.batch_size
    cfg.max_batches_per_epoch = a.max_batches
    dev = a.device or get_env("DEVICE_TYPE", "CPU")
    if dev.upper().startswith("GPU") and not torch.cuda.is_available():
        print("GPU requested but not available; using CPU")
        dev = "CPU"
    a.device = dev.upper()
    cfg.device_type = "GPU" if a.device.startswith("GPU") else "CPU"
    return a, cfg


def place(model, a):
    model.set_device(a.device)
    if a.fp32 and a.device.startswith("GPU"):
        model.set_compute_dtype(torch.float32)
    model.initialize()
    return model


def loaders(kind: str, a, cfg, **kw):
    shape, ncls = SHAPES[kind]
    try:
        if a.synthetic:
            raise FileNotFoundError
        if kind == "mnist":
            tr, te = create_mnist_loaders(os.path.join(a.data, "mnist"), **kw)
        elif kind == "cifar10":
            tr, te = create_cifar10_loaders(a.data, **kw)
        elif kind == "cifar100":
            tr, te = create_cifar100_loaders(a.data, **kw)
        else:
            tr, te = create_tiny_image_loader(os.path.join(a.data, "tiny-imagenet-200"), **kw)
        print(f"Loaded {kind}: {tr.size()} train / {te.size()} test samples")
    except (FileNotFoundError, RuntimeError, OSError):
        n = a.synthetic or 2048
        print(f"{kind} dataset not found under {a.data}: using {n} synthetic samples of shape {shape}")
        tr = SyntheticDataLoader(n, shape, ncls, seed=1, shuffle=True, **kw)
        te = SyntheticDataLoader(max(n // 4, 64), shape, ncls, seed=2, **kw)
    return tr, te
