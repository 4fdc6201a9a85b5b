"""HBM-resident data plane: the dataset lives in device memory, each batch is gathered and augmented
by one kernel launch (csrc/kernels/augment.hip).

The reference loads a dataset into host memory and, per batch, copies samples, augments them on
the host per sample and hands a host tensor to the trainer (include/data_loading/
tiny_imagenet_data_loader.hpp:481-560, include/data_augmentation/augmentation.hpp:114,
include/nn/train.hpp:108-147). At ~80k images/s per MI355X the host side of that path (gather,
per-sample augmentation, pinned staging, H2D) is the bottleneck of a real training run. With
288 GB of HBM per GPU the whole dataset fits on the device many times over (Tiny-ImageNet:
100k x 3 x 64 x 64 = 1.2 GB as uint8), so:

* ``DeviceDataLoader`` uploads the samples once — as uint8 when every value is k / 255 (decoded
  images: 4x smaller than fp32, exact), else fp32 — and the labels as int64;
* every epoch's sample order is a host permutation (the same rng as the host loaders, and
  ``nn.train._shard`` can restrict it to a rank's shard) uploaded once per epoch;
* ``get_next_batch`` launches ``augment_batch`` on the current stream: one workgroup per sample
  gathers it, runs the augmentation chain in LDS and writes the fp32 NCHW model input and its
  label. No host work per batch beyond the launch, no host sync, no H2D copy.

The augmentation ops and their order are the reference's (``AugmentationBuilder``); their random
draws come from a counter-based hash (``aug_uniform``), so :func:`reference_augment` below
reproduces a batch exactly on the host (tests/test_device_loader.py).
"""
from __future__ import annotations

from typing import Optional, Sequence

import numpy as np
import torch

from .augmentation import AugmentationStrategy
from .loader import BaseDataLoader

_KINDS = ("horizontal_flip", "vertical_flip", "rotation", "brightness", "contrast", "gaussian_noise",
          "random_crop", "cutout", "normalize")
_M64 = (1 << 64) - 1


def _mix(z: int) -> int:
    z = (z + 0x9E3779B97F4A7C15) & _M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & _M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & _M64
    return z ^ (z >> 31)


def aug_uniform(seed: int, sample: int, op: int, draw: int) -> np.float32:
    """The kernel's draw ``draw`` of op ``op`` for dataset sample ``sample`` (augment.hip)."""
    h = _mix(seed ^ _mix((sample * 0x100000001B3 + (op << 32) + draw) & _M64))
    return np.float32(h >> 40) * np.float32(1.0 / 16777216.0)


def _mix_np(z):
    z = z + np.uint64(0x9E3779B97F4A7C15)
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def _uniform_np(seed: int, sample: int, op: int, draws: np.ndarray) -> np.ndarray:
    base = np.uint64((sample * 0x100000001B3 + (op << 32)) & _M64)
    with np.errstate(over="ignore"):
        h = _mix_np(np.uint64(seed) ^ _mix_np(base + draws.astype(np.uint64)))
    return (h >> np.uint64(40)).astype(np.float32) * np.float32(1.0 / 16777216.0)


def device_ops(strategy: Optional[AugmentationStrategy], C: int):
    """AugmentationStrategy -> the kernel's op list [(kind, p, params)]; normalize gets its six
    (mean[3], std[3]) values with the host backend's channel rule (csrc/native/data.cpp)."""
    out = []
    for a in (strategy.augmentations if strategy is not None else []):
        name, p, args = a.op()
        if name not in _KINDS:
            raise ValueError(f"device augmentation: unknown op {name}")
        args = list(args)
        if name == "normalize":
            if len(args) >= 6 and C == 3:
                args = args[:6]
            else:
                m, s = args[0], args[len(args) // 2]
                args = [m, m, m, s, s, s]
        out.append((_KINDS.index(name), float(p), [float(v) for v in args]))
    if len(out) > 12:
        raise ValueError("device augmentation: at most 12 ops per chain")
    return out


def reference_augment(img: np.ndarray, sample: int, ops, seed: int) -> np.ndarray:
    """Host reference of one sample's chain with the kernel's draws ([C,H,W] float32 in [0, 1])."""
    x = img.astype(np.float32).copy()
    C, H, W = x.shape
    n = x.size
    for k, (kind, p, a) in enumerate(ops):
        name = _KINDS[kind]
        if name == "normalize":
            for c in range(C):
                cc = c if c < 3 else 0
                x[c] = (x[c] - np.float32(a[cc])) / np.float32(a[3 + cc])
            continue
        if aug_uniform(seed, sample, k, 0) >= np.float32(p):
            continue
        if name == "horizontal_flip":
            x = x[:, :, ::-1].copy()
        elif name == "vertical_flip":
            x = x[:, ::-1, :].copy()
        elif name == "brightness":
            f = np.float32(-a[0]) + np.float32(2 * a[0]) * aug_uniform(seed, sample, k, 1)
            x = np.clip(x + f, 0, 1)
        elif name == "contrast":
            f = np.float32(1 - a[0]) + np.float32(2 * a[0]) * aug_uniform(seed, sample, k, 1)
            x = np.clip(x * f, 0, 1)
        elif name == "gaussian_noise":
            i = np.arange(n, dtype=np.uint64)
            u1 = np.maximum(_uniform_np(seed, sample, k, 2 + 2 * i), np.float32(1e-7))
            u2 = _uniform_np(seed, sample, k, 3 + 2 * i)
            g = np.sqrt(-2 * np.log(u1)) * np.cos(np.float32(6.28318530717958647) * u2)
            x = np.clip(x + np.float32(a[0]) * g.reshape(x.shape).astype(np.float32), 0, 1)
        elif name == "random_crop":
            pad = int(a[0])
            span = 2 * pad + 1
            sx = min(int(aug_uniform(seed, sample, k, 1) * span), span - 1) - pad
            sy = min(int(aug_uniform(seed, sample, k, 2) * span), span - 1) - pad
            ys, xs = np.arange(H) + sy, np.arange(W) + sx
            valid = ((ys >= 0) & (ys < H))[:, None] & ((xs >= 0) & (xs < W))[None, :]
            src = x[:, np.clip(ys, 0, H - 1)][:, :, np.clip(xs, 0, W - 1)]
            x = np.where(valid[None], src, np.float32(0)).astype(np.float32)
        elif name == "cutout":
            sz = int(a[0])
            nx, ny = max(0, W - sz) + 1, max(0, H - sz) + 1
            x0 = min(int(aug_uniform(seed, sample, k, 1) * nx), nx - 1)
            y0 = min(int(aug_uniform(seed, sample, k, 2) * ny), ny - 1)
            x[:, y0:y0 + sz, x0:x0 + sz] = 0
        elif name == "rotation":
            ang = (np.float32(-a[0]) + np.float32(2 * a[0]) * aug_uniform(seed, sample, k, 1)) * np.float32(
                3.14159265358979) / np.float32(180)
            ca, sa = np.cos(ang), np.sin(ang)
            cx, cy = W / 2.0, H / 2.0
            yy, xx = np.meshgrid(np.arange(H), np.arange(W), indexing="ij")
            fx0 = (xx - cx) * ca - (yy - cy) * sa + cx
            fy0 = (xx - cx) * sa + (yy - cy) * ca + cy
            x1, y1 = np.floor(fx0).astype(int), np.floor(fy0).astype(int)
            fx, fy = fx0 - x1, fy0 - y1

            def at(q, a_, b_):
                ok = (a_ >= 0) & (a_ < H) & (b_ >= 0) & (b_ < W)
                return np.where(ok, q[np.clip(a_, 0, H - 1), np.clip(b_, 0, W - 1)], 0)
            x = np.stack([(1 - fx) * (1 - fy) * at(q, y1, x1) + fx * (1 - fy) * at(q, y1, x1 + 1)
                          + (1 - fx) * fy * at(q, y1 + 1, x1) + fx * fy * at(q, y1 + 1, x1 + 1) for q in x])
            x = x.astype(np.float32)
    return x


class DeviceDataLoader(BaseDataLoader):
    """Dataset resident in HBM; batches gathered + augmented on the GPU (module docstring).

    ``source``: a loaded :class:`BaseDataLoader` (its arrays, classes and augmentation are taken
    over) or None with ``data`` / ``labels`` arrays. ``storage``: "auto" (uint8 when exact),
    "u8" or "f32"."""

    def __init__(self, source: Optional[BaseDataLoader] = None, data: Optional[np.ndarray] = None,
                 labels: Optional[np.ndarray] = None, num_classes: int = 0, batch_size: int = 32,
                 shuffle: bool = False, seed: int = 0, one_hot: bool = False, drop_last: bool = False,
                 device: str = "cuda", storage: str = "auto"):
        super().__init__(batch_size=batch_size, shuffle=shuffle, seed=seed, one_hot=one_hot, drop_last=drop_last,
                         device=device, prefetch=False)
        self.seed0 = int(seed)
        if source is not None:
            data, labels = source.data, source.labels
            num_classes = num_classes or getattr(source, "num_classes", 0)
            if source.augmentation is not None:
                self.augmentation = source.augmentation
        if data is None or labels is None:
            raise ValueError("DeviceDataLoader needs a source loader or data + labels")
        if data.ndim != 4:
            raise ValueError("DeviceDataLoader: [N, C, H, W] image data")
        from ..ops._ext import kernels
        self._K = kernels()
        N, C, H, W = data.shape
        if not self._K.augment_batch_supported(C, H, W):
            raise ValueError(f"DeviceDataLoader: {C}x{H}x{W} images exceed the kernel's LDS staging")
        self.num_classes = num_classes
        self.data = None  # host copy not kept (the device holds it)
        self._shape = (C, H, W)
        self._n = N
        self.labels = np.ascontiguousarray(labels).astype(np.int64)
        self.order = np.arange(N, dtype=np.int64)
        self.current = 0
        self.dev = torch.device(device)
        u8 = storage == "u8" or (storage == "auto" and self._exact_u8(data))
        self.storage = "u8" if u8 else "f32"
        self._data = self._upload(data, u8)
        self._labels = torch.from_numpy(self.labels).to(self.dev)
        self._order_dev = None
        self._order_src = None
        self.epoch = 0

    @staticmethod
    def _exact_u8(data: np.ndarray, chunk: int = 4096) -> bool:
        for i in range(0, len(data), chunk):
            d = data[i:i + chunk]
            q = np.rint(d * np.float32(255))
            if q.min() < 0 or q.max() > 255 or not np.array_equal((q / np.float32(255)).astype(np.float32), d):
                return False
        return True

    def _upload(self, data: np.ndarray, u8: bool, chunk: int = 8192) -> torch.Tensor:
        N = len(data)
        per = int(np.prod(data.shape[1:]))
        out = torch.empty((N, per), dtype=torch.uint8 if u8 else torch.float32, device=self.dev)
        for i in range(0, N, chunk):
            d = np.ascontiguousarray(data[i:i + chunk]).reshape(-1, per)
            if u8:
                d = np.rint(d * np.float32(255)).astype(np.uint8)
            out[i:i + len(d)].copy_(torch.from_numpy(d))
        return out

    # ---- BaseDataLoader surface
    def size(self) -> int:
        return self._n

    __len__ = size

    def get_data_shape(self):
        return list(self._shape)

    def load_data(self, *a, **kw) -> bool:
        return True

    def shuffle(self) -> None:
        super().shuffle()  # (in place: the cached device copy of the order is stale)
        self._order_dev = None

    def reset(self) -> None:
        super().reset()
        self._order_dev = None
        self.epoch += 1

    def _device_order(self) -> torch.Tensor:
        if self._order_dev is None or self._order_src is not self.order:
            self._order_dev = torch.from_numpy(np.ascontiguousarray(self.order, dtype=np.int64)).to(self.dev)
            self._order_src = self.order
        return self._order_dev

    def get_batch(self, batch_size: int):
        n = len(self.order)
        if self.current >= n:
            return None
        e = min(self.current + batch_size, n)
        if self.drop_last and e - self.current < batch_size:
            return None
        order = self._device_order()
        idx = order[self.current:e]
        self.current = e
        C, H, W = self._shape
        x = torch.empty((len(idx), C, H, W), dtype=torch.float32, device=self.dev)
        y = torch.empty((len(idx),), dtype=torch.int64, device=self.dev)
        from ..ops._ext import stream_ptr
        self._K.augment_batch(self._data.data_ptr(), int(self.storage == "u8"), idx.data_ptr(),
                              self._labels.data_ptr(), y.data_ptr(), x.data_ptr(), len(idx), C, H, W,
                              self.seed_for_epoch(), device_ops(self.augmentation, C), stream_ptr(self.dev))
        if self.one_hot:
            y = torch.nn.functional.one_hot(y, self.num_classes).float().view(len(idx), self.num_classes, 1, 1)
        return x, y

    def seed_for_epoch(self) -> int:
        """The augmentation seed of the current epoch (the kernel's ``seed``): a function of the
        loader seed and the epoch counter, so a rerun reproduces every batch."""
        return _mix((self.seed0 * 0x2545F4914F6CDD1D + self.epoch) & _M64)

    def get_next_batch(self):
        return self.get_batch(self.batch_size)


def to_device_loader(loader: BaseDataLoader, **kw) -> DeviceDataLoader:
    """The HBM-resident twin of a loaded host loader (same arrays, classes, batch size, shuffling,
    augmentation chain)."""
    kw.setdefault("batch_size", loader.batch_size)
    kw.setdefault("shuffle", loader.shuffle_each_epoch)
    kw.setdefault("drop_last", loader.drop_last)
    kw.setdefault("one_hot", loader.one_hot)
    return DeviceDataLoader(source=loader, **kw)
