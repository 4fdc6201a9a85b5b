"""Data loaders (reference include/data_loading/data_loader.hpp:25-190).

``BaseDataLoader`` keeps the reference iterator API — ``load_data``, ``get_next_batch``,
``get_batch``, ``reset``, ``shuffle``, ``prepare_batches``, ``set_augmentation`` — over an
in-memory dataset.  Batches are gathered by the native runtime (GIL released), augmented
per batch, and returned as torch tensors; with ``device="cuda"`` a background thread
prepares batch *k+1* into pinned memory and issues its host-to-device copy on a side
stream while batch *k* trains.

Labels are class indices (int64) by default — the fused loss kernels take them directly —
or the reference's one-hot ``[N, C, 1, 1]`` float tensors with ``one_hot=True``.
Unlike the reference, ``prepare_batches`` does not materialise every augmented batch of the
epoch up front (memory); augmentation happens when a batch is produced, with the same
per-epoch randomness.
"""
from __future__ import annotations

import queue
import threading
from typing import Optional, Tuple

import numpy as np
import torch

from ..ops._ext import native
from .augmentation import AugmentationStrategy


class BaseDataLoader:
    num_classes: int = 0

    def __init__(self, batch_size: int = 32, shuffle: bool = False, seed: int = 0, one_hot: bool = False,
                 drop_last: bool = False, device: Optional[str] = None, prefetch: bool = True):
        self.data: Optional[np.ndarray] = None      # [N, ...] float32
        self.labels: Optional[np.ndarray] = None    # [N] int64 or [N, K] float32 (regression)
        self.batch_size = int(batch_size)
        self.shuffle_each_epoch = shuffle
        self.one_hot = one_hot
        self.drop_last = drop_last
        self.device = device
        self.prefetch = prefetch
        self.augmentation: Optional[AugmentationStrategy] = None
        self.rng = np.random.default_rng(seed)
        self.order: Optional[np.ndarray] = None
        self.current = 0
        self._q = None
        self._worker = None
        self._stream = None

    # ---- dataset
    def load_data(self, *a, **kw) -> bool:
        raise NotImplementedError

    def set_arrays(self, data: np.ndarray, labels: np.ndarray) -> "BaseDataLoader":
        self.data = np.ascontiguousarray(data, dtype=np.float32)
        self.labels = np.ascontiguousarray(labels)
        self.order = np.arange(len(self.data), dtype=np.int64)
        self.current = 0
        return self

    def size(self) -> int:
        return 0 if self.data is None else len(self.data)

    __len__ = size

    def get_data_shape(self):
        return list(self.data.shape[1:])

    def num_batches(self) -> int:
        n = self.size()
        return n // self.batch_size if self.drop_last else (n + self.batch_size - 1) // self.batch_size

    # ---- iteration
    def set_augmentation(self, strategy: Optional[AugmentationStrategy]) -> None:
        self.augmentation = strategy

    def shuffle(self) -> None:
        self.rng.shuffle(self.order)

    def prepare_batches(self, batch_size: int) -> None:
        self.batch_size = int(batch_size)
        self.reset()

    def reset(self) -> None:
        self._stop_worker()
        self.current = 0
        if self.shuffle_each_epoch:
            self.shuffle()

    def _make(self, idx: np.ndarray) -> Tuple[torch.Tensor, torch.Tensor]:
        x = np.empty((len(idx),) + self.data.shape[1:], dtype=np.float32)
        native().data.gather_rows(self.data, idx, x)
        if self.augmentation is not None and x.ndim == 4:
            self.augmentation.apply(x)
        y = self.labels[idx]
        xt = torch.from_numpy(x)
        yt = torch.from_numpy(np.ascontiguousarray(y))
        if self.one_hot and yt.dtype == torch.int64:
            yt = torch.nn.functional.one_hot(yt, self.num_classes).float().view(len(idx), self.num_classes, 1, 1)
        return xt, yt

    def _next_indices(self, batch_size: int) -> Optional[np.ndarray]:
        n = self.size()
        if self.current >= n:
            return None
        e = min(self.current + batch_size, n)
        if self.drop_last and e - self.current < batch_size:
            return None
        idx = self.order[self.current:e]
        self.current = e
        return idx

    def get_batch(self, batch_size: int):
        idx = self._next_indices(batch_size)
        if idx is None:
            return None
        x, y = self._make(idx)
        if self.device is not None:
            x, y = x.to(self.device), y.to(self.device)
        return x, y

    def get_next_batch(self):
        if self.device is None or not self.prefetch or not str(self.device).startswith("cuda"):
            return self.get_batch(self.batch_size)
        if self._worker is None:
            self._start_worker()
        item = self._q.get()
        if item is None:
            self._worker.join()
            self._worker = None
            return None
        x, y, ev = item
        torch.cuda.current_stream().wait_event(ev)
        x.record_stream(torch.cuda.current_stream())
        y.record_stream(torch.cuda.current_stream())
        return x, y

    def __iter__(self):
        self.reset()
        while True:
            b = self.get_next_batch()
            if b is None:
                return
            yield b

    # ---- background prefetch (pinned host buffer -> side-stream H2D copy)
    def _start_worker(self):
        self._q = queue.Queue(maxsize=2)
        self._stop = False
        if self._stream is None:
            self._stream = torch.cuda.Stream(device=self.device)

        def work():
            while not self._stop:
                idx = self._next_indices(self.batch_size)
                if idx is None:
                    break
                x, y = self._make(idx)
                x, y = x.pin_memory(), y.pin_memory()
                with torch.cuda.stream(self._stream):
                    xd = x.to(self.device, non_blocking=True)
                    yd = y.to(self.device, non_blocking=True)
                    ev = torch.cuda.Event()
                    ev.record(self._stream)
                self._q.put((xd, yd, ev))
            self._q.put(None)

        self._worker = threading.Thread(target=work, daemon=True)
        self._worker.start()

    def _stop_worker(self):
        if self._worker is not None:
            self._stop = True
            while self._worker.is_alive():
                try:
                    self._q.get(timeout=0.1)
                except queue.Empty:
                    pass
            self._worker.join()
            self._worker = None


class ArrayDataLoader(BaseDataLoader):
    """Loader over in-memory arrays."""

    def __init__(self, data, labels, num_classes: int = 0, **kw):
        super().__init__(**kw)
        self.num_classes = num_classes
        self.set_arrays(np.asarray(data), np.asarray(labels))

    def load_data(self, *a, **kw):
        return True


class SyntheticDataLoader(BaseDataLoader):
    """Deterministic random images + labels of a given shape (benchmarks, tests; the
    reference has no synthetic loader)."""

    def __init__(self, num_samples: int, shape, num_classes: int, seed: int = 0, **kw):
        super().__init__(seed=seed, **kw)
        self.num_classes = num_classes
        g = np.random.default_rng(seed)
        data = g.random((num_samples,) + tuple(shape), dtype=np.float32)
        labels = g.integers(0, num_classes, num_samples, dtype=np.int64)
        self.set_arrays(data, labels)

    def load_data(self, *a, **kw):
        return True
