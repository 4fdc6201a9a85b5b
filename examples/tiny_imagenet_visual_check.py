#!/usr/bin/env python3
"""Tiny-ImageNet visual inspection tool (reference examples/tiny_imagenet_visual_check.cpp:143-260).

Loads the train and val splits through the framework's loader (native JPEG decoder on a thread
pool, ``data/datasets.py``), prints the dataset and class-name summary, draws a few training
samples, and for each one saves a PNG, prints per-channel statistics (min / max / mean / std in
the loader's [0, 1] scale) and an 8x8 ASCII grayscale preview — the checks the reference uses to
confirm that decoding, channel order and normalisation are right before training.

No dataset in this environment (no network): ``--synthetic`` (or a missing directory) draws
random images instead so the tool runs end to end; point ``--root`` at a real
``tiny-imagenet-200`` directory to inspect real data.

    python examples/tiny_imagenet_visual_check.py --root data/tiny-imagenet-200 --samples 5 --out visual_check
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from dcnn_amd.data import SyntheticDataLoader, TinyImageNetDataLoader  # noqa: E402

RAMP = " .:-=+*#%@"


def save_png(path: str, img_chw: np.ndarray) -> None:
    """[3,H,W] float in [0,1] -> 8-bit RGB PNG."""
    from PIL import Image
    hwc = (np.clip(img_chw.transpose(1, 2, 0), 0.0, 1.0) * 255.0 + 0.5).astype(np.uint8)
    Image.fromarray(hwc, "RGB").save(path)


def channel_stats(img_chw: np.ndarray):
    return [(float(c.min()), float(c.max()), float(c.mean()), float(c.std())) for c in img_chw]


def ascii_preview(img_chw: np.ndarray, n: int = 8) -> str:
    gray = 0.299 * img_chw[0] + 0.587 * img_chw[1] + 0.114 * img_chw[2]
    rows = []
    for y in range(min(n, gray.shape[0])):
        rows.append(" ".join(RAMP[min(len(RAMP) - 1, int(v * len(RAMP)))] for v in gray[y, :n]))
    bar = "--" * n
    return "\n".join(["  " + bar] + ["  " + r for r in rows] + ["  " + bar])


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--root", default="data/tiny-imagenet-200")
    ap.add_argument("--samples", type=int, default=5)
    ap.add_argument("--out", default="visual_check")
    ap.add_argument("--max-per-class", type=int, default=0, help="decode at most this many train images per class")
    ap.add_argument("--synthetic", action="store_true")
    ap.add_argument("--seed", type=int, default=0)
    a = ap.parse_args(argv)
    print("=== Tiny ImageNet Visual Inspection Tool ===")
    real = not a.synthetic and os.path.isdir(a.root)
    if real:
        print("\n--- Loading Training Data ---")
        tr = TinyImageNetDataLoader()
        tr.load_data(a.root, True, threads=0, max_per_class=a.max_per_class)
        print(f"Loaded {tr.size()} training samples ({tr.decode_failures} decode failures)")
        print("\n--- Loading Validation Data ---")
        va = TinyImageNetDataLoader()
        va.load_data(a.root, False)
        print(f"Loaded {va.size()} validation samples")
        print("\n=== Dataset Information ===")
        print(f"Classes: {len(tr.wnids)}   image shape: {tr.get_data_shape()}")
        print("\n--- Sample Class Names (first 10) ---")
        for i, w in enumerate(tr.wnids[:10]):
            print(f"  {i}: {w} - {tr.class_names.get(w, w)}")
        names = [tr.class_names.get(w, w) for w in tr.wnids]
    else:
        print(f"\n(no dataset at {a.root!r}: using {max(a.samples, 8)} synthetic 3x64x64 images)")
        tr = SyntheticDataLoader(max(a.samples, 8), (3, 64, 64), 200, seed=a.seed)
        tr.load_data()
        names = [f"class_{i}" for i in range(200)]
    os.makedirs(a.out, exist_ok=True)
    print("\n=== Sampling Training Images ===")
    tr.shuffle()
    x, y = tr.get_batch(a.samples)
    x, y = x.numpy(), y.numpy()
    lab = y.argmax(1) if y.ndim == 2 else y
    print(f"\nBatch shape: {'x'.join(str(s) for s in x.shape)}")
    for i in range(len(x)):
        img = x[i].astype(np.float32)
        label = int(lab[i])
        print(f"\n--- Sample {i + 1} ---")
        print(f"\n  Image: {names[label] if label < len(names) else label} (label {label})")
        for ch, (lo, hi, mu, sd) in zip("RGB", channel_stats(img)):
            print(f"    {ch} channel: min={lo:.4f}  max={hi:.4f}  mean={mu:.4f}  std={sd:.4f}")
        if img.min() < 0.0 or img.max() > 1.0:
            print("    WARNING: values outside [0, 1] — the loader's normalisation is off")
        path = os.path.join(a.out, f"sample_{i + 1}_label{label}.png")
        save_png(path, img)
        print(f"  Saved: {path}")
        print("\n  ASCII preview (top-left 8x8, grayscale):")
        print(ascii_preview(img))
    return 0


if __name__ == "__main__":
    sys.exit(main())
