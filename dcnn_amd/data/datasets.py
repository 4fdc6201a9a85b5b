"""Dataset loaders on the native parsers (reference include/data_loading/*):

* MNIST CSV (label + 784 pixels, header line) -> [N,1,28,28] / 255   (mnist_data_loader.hpp:36-331)
* CIFAR-10 binary batches (1 label byte + 3072)  -> [N,3,32,32] / 255 (cifar10_data_loader.hpp:37-396)
* CIFAR-100 binary (coarse, fine label bytes)    -> fine or coarse labels (cifar100_data_loader.hpp)
* Tiny-ImageNet-200 directory (wnids.txt, train/<wnid>/images/*.JPEG, val_annotations.txt),
  JPEGs decoded by the native decoder on a thread pool -> [N,3,64,64] / 255
  (tiny_imagenet_data_loader.hpp:55-626).  A decoded copy can be cached as .npy
  (``cache=True``) so later runs memory-map it instead of decoding 100k files.
* UJI / UTS WiFi fingerprint CSV, regression or classification, with z-score normalisation
  fitted on the training split (wifi_data_loader.hpp:24-461).
"""
from __future__ import annotations

import os
from typing import List, Optional, Sequence, Tuple

import numpy as np

from ..ops._ext import native
from .loader import BaseDataLoader


def _d():
    return native().data


class MNISTDataLoader(BaseDataLoader):
    num_classes = 10

    def load_data(self, path: str, has_header: bool = True) -> bool:
        x, y = _d().load_mnist_csv(path, has_header)
        self.set_arrays(x, y)
        return len(x) > 0


class CIFAR10DataLoader(BaseDataLoader):
    num_classes = 10
    class_names = ["airplane", "automobile", "bird", "cat", "deer", "dog", "frog", "horse", "ship", "truck"]

    def load_data(self, path: str) -> bool:
        return self.load_multiple_files([path])

    def load_multiple_files(self, paths: Sequence[str]) -> bool:
        x, y = _d().load_cifar_bin(list(paths), 1, 0)
        self.set_arrays(x, y)
        return len(x) > 0


class CIFAR100DataLoader(BaseDataLoader):
    def __init__(self, use_coarse_labels: bool = False, **kw):
        super().__init__(**kw)
        self.use_coarse_labels = use_coarse_labels
        self.num_classes = 20 if use_coarse_labels else 100

    def load_data(self, path: str) -> bool:
        x, y = _d().load_cifar_bin([path], 2, 0 if self.use_coarse_labels else 1)
        self.set_arrays(x, y)
        return len(x) > 0


class TinyImageNetDataLoader(BaseDataLoader):
    num_classes = 200

    def __init__(self, **kw):
        super().__init__(**kw)
        self.wnids: List[str] = []
        self.class_names: dict = {}
        self.decode_failures = 0

    def load_data(self, root: str, train: bool = True, cache: bool = False, threads: int = 0,
                  max_per_class: int = 0) -> bool:
        split = "train" if train else "val"
        cpath = os.path.join(root, f".dcnn_cache_{split}_{max_per_class}.npz")
        if cache and os.path.exists(cpath):
            with np.load(cpath, allow_pickle=False) as z:
                x, y, wn = z["x"], z["y"], [str(s) for s in z["wnids"]]
            fails = 0
        else:
            x, y, wn, fails = _d().load_tiny_imagenet(root, split, threads, max_per_class)
            if cache:
                np.savez(cpath, x=x, y=y, wnids=np.array(wn))
        self.wnids = list(wn)
        self.decode_failures = int(fails)
        words = os.path.join(root, "words.txt")
        if os.path.exists(words):
            table = _d().read_tiny_imagenet_words(words)
            self.class_names = {w: table.get(w, w) for w in self.wnids}
        self.set_arrays(x, y)
        return len(x) > 0


class WiFiDataLoader(BaseDataLoader):
    """RSSI fingerprints -> coordinates (regression) or floor/building ids (classification)."""

    def __init__(self, is_regression: bool = True, **kw):
        super().__init__(**kw)
        self.is_regression = is_regression
        self.feature_mean = self.feature_std = None
        self.target_mean = self.target_std = None

    def load_data(self, path: str, feature_start: int = 0, feature_end: int = 520, target_start: int = 520,
                  target_end: int = 522, has_header: bool = True) -> bool:
        f, t = _d().load_wifi_csv(path, feature_start, feature_end, target_start, target_end, has_header)
        if not self.is_regression:
            t = t[:, 0].astype(np.int64)
            self.num_classes = int(t.max()) + 1 if len(t) else 0
        self.set_arrays(f, t)
        return len(f) > 0

    def normalize_data(self, stats_from: Optional["WiFiDataLoader"] = None) -> None:
        """Z-score features (and regression targets) with this split's or ``stats_from``'s stats."""
        src = stats_from or self
        if src.feature_mean is None:
            src.feature_mean = src.data.mean(0)
            s = src.data.std(0)
            src.feature_std = np.where(s < 1e-8, 1.0, s).astype(np.float32)
            if self.is_regression:
                src.target_mean = src.labels.mean(0)
                s = src.labels.std(0)
                src.target_std = np.where(s < 1e-8, 1.0, s).astype(np.float32)
        self.feature_mean, self.feature_std = src.feature_mean, src.feature_std
        self.data = np.ascontiguousarray((self.data - src.feature_mean) / src.feature_std, dtype=np.float32)
        if self.is_regression:
            self.target_mean, self.target_std = src.target_mean, src.target_std
            self.labels = np.ascontiguousarray((self.labels - src.target_mean) / src.target_std, dtype=np.float32)

    def denormalize_targets(self, t: np.ndarray) -> np.ndarray:
        return t * self.target_std + self.target_mean if self.target_std is not None else t


# ---------------------------------------------------------------- factories (reference create_* helpers)
def create_mnist_loaders(data_dir: str = "data/mnist", **kw) -> Tuple[MNISTDataLoader, MNISTDataLoader]:
    tr, te = MNISTDataLoader(**kw), MNISTDataLoader(**kw)
    tr.load_data(os.path.join(data_dir, "train.csv"))
    te.load_data(os.path.join(data_dir, "test.csv"))
    return tr, te


def create_cifar10_loaders(data_dir: str = "data", **kw):
    d = os.path.join(data_dir, "cifar-10-batches-bin")
    tr, te = CIFAR10DataLoader(**kw), CIFAR10DataLoader(**kw)
    tr.load_multiple_files([os.path.join(d, f"data_batch_{i}.bin") for i in range(1, 6)])
    te.load_data(os.path.join(d, "test_batch.bin"))
    return tr, te


def create_cifar100_loaders(data_dir: str = "data", use_coarse_labels: bool = False, **kw):
    d = os.path.join(data_dir, "cifar-100-binary")
    tr = CIFAR100DataLoader(use_coarse_labels, **kw)
    te = CIFAR100DataLoader(use_coarse_labels, **kw)
    tr.load_data(os.path.join(d, "train.bin"))
    te.load_data(os.path.join(d, "test.bin"))
    return tr, te


def create_tiny_image_loader(root: str = "data/tiny-imagenet-200", cache: bool = True, **kw):
    tr, va = TinyImageNetDataLoader(**kw), TinyImageNetDataLoader(**kw)
    tr.load_data(root, True, cache)
    va.load_data(root, False, cache)
    return tr, va
