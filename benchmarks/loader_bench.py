#!/usr/bin/env python3
"""Real-data feeding at GPU speed: decode, host loader, HBM-resident loader and end-to-end training.

Builds a synthetic Tiny-ImageNet directory (PIL-written 64x64 JPEGs in the reference's layout:
wnids.txt, words.txt, train/<wnid>/images/*.JPEG, val/images + val_annotations.txt), then times:

1. ``decode``: the native JPEG decoder over the directory (``TinyImageNetDataLoader.load_data``,
   all host threads) — images/s and images/s per host core;
2. ``host_loader``: the host path — native gather + host augmentation (crop + flip + normalise) +
   pinned staging + H2D on a side stream (``BaseDataLoader`` with ``device="cuda"``);
3. ``device_loader``: the HBM-resident path — one ``augment_batch`` launch per batch
   (``DeviceDataLoader``), timed with device synchronisation;
4. ``train``: ResNet-18-tiny training steps (hipGraph, Adam) fed by the device loader, against the
   same steps on a fixed synthetic batch (``bench.py``'s loop) — the ratio is the share of the
   GPU step rate that real data keeps.

  python benchmarks/loader_bench.py --images-per-class 50 --batch 256 --steps 40
Reference: include/data_loading/tiny_imagenet_data_loader.hpp:278-560, include/nn/train.hpp:108-147.
"""
import argparse
import io
import json
import os
import sys
import tempfile
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def make_dataset(root, classes, per_class, val_per_class, seed=0):
    from PIL import Image
    g = np.random.default_rng(seed)
    wnids = [f"n{10000000 + i:08d}" for i in range(classes)]
    os.makedirs(root, exist_ok=True)
    with open(os.path.join(root, "wnids.txt"), "w") as f:
        f.write("\n".join(wnids) + "\n")
    with open(os.path.join(root, "words.txt"), "w") as f:
        f.write("\n".join(f"{w}\tclass {i}" for i, w in enumerate(wnids)) + "\n")
    base = g.integers(0, 256, (classes, 8, 8, 3))

    def img(c):
        # a class-coloured smooth pattern + noise (compressible like a photo, not like white noise)
        up = np.kron(base[c], np.ones((8, 8, 1)))
        return np.clip(up + g.normal(0, 20, up.shape), 0, 255).astype(np.uint8)

    for c, w in enumerate(wnids):
        d = os.path.join(root, "train", w, "images")
        os.makedirs(d, exist_ok=True)
        for i in range(per_class):
            Image.fromarray(img(c)).save(os.path.join(d, f"{w}_{i}.JPEG"), "JPEG", quality=90)
    vd = os.path.join(root, "val", "images")
    os.makedirs(vd, exist_ok=True)
    with open(os.path.join(root, "val", "val_annotations.txt"), "w") as f:
        k = 0
        for c, w in enumerate(wnids):
            for i in range(val_per_class):
                name = f"val_{k}.JPEG"
                Image.fromarray(img(c)).save(os.path.join(vd, name), "JPEG", quality=90)
                f.write(f"{name}\t{w}\t0\t0\t63\t63\n")
                k += 1
    return classes * per_class


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--classes", type=int, default=200)
    ap.add_argument("--images-per-class", type=int, default=50)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--root", default="")
    a = ap.parse_args()
    from dcnn_amd.data import AugmentationBuilder, TinyImageNetDataLoader, to_device_loader
    cores = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    root = a.root or tempfile.mkdtemp(prefix="tinyimg_")
    t0 = time.perf_counter()
    n = make_dataset(root, a.classes, a.images_per_class, 2)
    print(json.dumps({"phase": "make_dataset", "images": n, "s": round(time.perf_counter() - t0, 2)}), flush=True)

    tr = TinyImageNetDataLoader(batch_size=a.batch, shuffle=True, seed=1, device="cuda")
    t0 = time.perf_counter()
    tr.load_data(root, True)
    dt = time.perf_counter() - t0
    print(json.dumps({"phase": "decode", "images": tr.size(), "images_per_sec": round(tr.size() / dt),
                      "host_cores": cores, "images_per_sec_per_core": round(tr.size() / dt / cores),
                      "failures": tr.decode_failures}), flush=True)
    aug = AugmentationBuilder().random_crop(0.5, 4).horizontal_flip(0.5).normalize().build()
    tr.set_augmentation(aug)

    def time_loader(ld, batches):
        ld.reset()
        got = 0
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(batches):
            b = ld.get_next_batch()
            if b is None:
                ld.reset()
                b = ld.get_next_batch()
            got += b[0].shape[0]
        torch.cuda.synchronize()
        return got / (time.perf_counter() - t)

    nb = max(4, min(a.steps, tr.num_batches() - 1))
    ips = time_loader(tr, nb)
    print(json.dumps({"phase": "host_loader", "images_per_sec": round(ips), "host_cores": cores,
                      "images_per_sec_per_core": round(ips / cores),
                      "path": "native gather + host augmentation + pinned staging + H2D"}), flush=True)
    dl = to_device_loader(tr)
    ips_d = time_loader(dl, nb)
    print(json.dumps({"phase": "device_loader", "images_per_sec": round(ips_d), "storage": dl.storage,
                      "device_bytes": dl._data.numel() * dl._data.element_size(),
                      "path": "HBM-resident uint8 + augment_batch kernel"}), flush=True)

    # ---- end to end: training steps fed by the device loader vs a fixed synthetic batch
    from dcnn_amd.models import create_model
    from dcnn_amd.nn import Adam, LossFactory
    from dcnn_amd.runtime.step import TrainStep
    m = create_model("resnet18_tiny_imagenet")
    m.set_seed(1)
    m.set_device("GPU:0")
    m.initialize()
    m.set_first_layer_input_grad(False)
    opt = Adam(1e-3)
    opt.attach(m)
    st = TrainStep(m, LossFactory.create("softmax_crossentropy"), opt, use_graph=True)
    dl.drop_last = True
    dl.reset()

    def batch():
        b = dl.get_next_batch()
        if b is None:
            dl.reset()
            b = dl.get_next_batch()
        return b

    for _ in range(5):
        st(*batch())
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(a.steps):
        st(*batch())
    torch.cuda.synchronize()
    real = a.batch * a.steps / (time.perf_counter() - t)
    x0, y0 = batch()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(a.steps):
        st(x0, y0)
    torch.cuda.synchronize()
    synth = a.batch * a.steps / (time.perf_counter() - t)
    print(json.dumps({"phase": "train", "model": "resnet18_tiny_imagenet", "batch": a.batch,
                      "images_per_sec_device_loader": round(real), "images_per_sec_fixed_batch": round(synth),
                      "ratio": round(real / synth, 3), "final_loss": round(float(st.last_loss), 4)}), flush=True)


if __name__ == "__main__":
    main()
