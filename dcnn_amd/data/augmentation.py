"""Data augmentation (reference include/data_augmentation/augmentation.hpp:17-178 and the
per-transform headers).  The transforms are executed by the native runtime
(``_native.data.augment``) on whole host batches, multithreaded with the GIL released;
per-sample random streams depend only on (seed, sample index).

Semantics follow the reference: brightness adds U(-r, r) and clamps to [0,1]; contrast
multiplies by U(1-r, 1+r) and clamps; gaussian noise adds N(0, std) and clamps; random crop
zero-pads by ``padding`` and crops back at a uniform offset; cutout zeroes a square;
rotation is bilinear about the centre with zero fill; normalisation is (x - mean) / std per
channel and is always applied.
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import numpy as np

from ..ops._ext import native


class Augmentation:
    kind = ""

    def __init__(self, probability: float = 0.5, *args: float):
        self.probability = float(probability)
        self.args = [float(a) for a in args]

    def name(self) -> str:
        return type(self).__name__

    def op(self) -> Tuple[str, float, List[float]]:
        return (self.kind, self.probability, self.args)

    def clone(self):
        c = object.__new__(type(self))
        c.__dict__.update(self.__dict__)
        c.args = list(self.args)
        return c


class HorizontalFlip(Augmentation):
    kind = "horizontal_flip"


class VerticalFlip(Augmentation):
    kind = "vertical_flip"


class Rotation(Augmentation):
    kind = "rotation"

    def __init__(self, probability: float = 0.5, max_angle_degrees: float = 15.0):
        super().__init__(probability, max_angle_degrees)


class Brightness(Augmentation):
    kind = "brightness"

    def __init__(self, probability: float = 0.5, brightness_range: float = 0.2):
        super().__init__(probability, brightness_range)


class Contrast(Augmentation):
    kind = "contrast"

    def __init__(self, probability: float = 0.5, contrast_range: float = 0.2):
        super().__init__(probability, contrast_range)


class GaussianNoise(Augmentation):
    kind = "gaussian_noise"

    def __init__(self, probability: float = 0.3, noise_std: float = 0.05):
        super().__init__(probability, noise_std)


class RandomCrop(Augmentation):
    kind = "random_crop"

    def __init__(self, probability: float = 0.5, padding: int = 4):
        super().__init__(probability, padding)


class Cutout(Augmentation):
    kind = "cutout"

    def __init__(self, probability: float = 0.5, cutout_size: int = 8):
        super().__init__(probability, cutout_size)


class Normalization(Augmentation):
    kind = "normalize"

    def __init__(self, mean: Sequence[float] = (0.485, 0.456, 0.406), std: Sequence[float] = (0.229, 0.224, 0.225)):
        mean, std = list(mean), list(std)
        if len(mean) != len(std) or len(mean) not in (1, 3):
            raise ValueError("Normalization needs 1 or 3 per-channel means/stds")
        if len(mean) == 1:
            mean, std = mean * 3, std * 3
        super().__init__(1.0, *(mean + std))


class AugmentationStrategy:
    """Ordered pipeline of augmentations applied to a host batch in place."""

    def __init__(self, augs: Optional[Sequence[Augmentation]] = None, seed: int = 0):
        self.augmentations: List[Augmentation] = list(augs or [])
        self.seed = int(seed)
        self._calls = 0

    def add(self, a: Augmentation) -> "AugmentationStrategy":
        self.augmentations.append(a)
        return self

    def set_seed(self, seed: int) -> None:
        self.seed = int(seed)
        self._calls = 0

    def apply(self, batch: np.ndarray, labels=None) -> np.ndarray:
        """Augment ``batch`` ([N,C,H,W] float32, C-contiguous) in place; returns it."""
        if not self.augmentations:
            return batch
        if batch.dtype != np.float32 or not batch.flags.c_contiguous:
            raise ValueError("augment: expected a C-contiguous float32 [N,C,H,W] array")
        seed = (self.seed * 0x9E3779B97F4A7C15 + self._calls) & ((1 << 64) - 1)
        self._calls += 1
        native().data.augment(batch, [a.op() for a in self.augmentations], seed)
        return batch

    def clone(self) -> "AugmentationStrategy":
        return AugmentationStrategy([a.clone() for a in self.augmentations], self.seed)

    def __len__(self):
        return len(self.augmentations)


class AugmentationBuilder:
    """Fluent builder (reference augmentation.hpp AugmentationBuilder)."""

    def __init__(self):
        self._augs: List[Augmentation] = []

    def horizontal_flip(self, probability=0.5):
        self._augs.append(HorizontalFlip(probability))
        return self

    def vertical_flip(self, probability=0.5):
        self._augs.append(VerticalFlip(probability))
        return self

    def rotation(self, probability=0.5, max_angle_degrees=15.0):
        self._augs.append(Rotation(probability, max_angle_degrees))
        return self

    def brightness(self, probability=0.5, brightness_range=0.2):
        self._augs.append(Brightness(probability, brightness_range))
        return self

    def contrast(self, probability=0.5, contrast_range=0.2):
        self._augs.append(Contrast(probability, contrast_range))
        return self

    def gaussian_noise(self, probability=0.3, noise_std=0.05):
        self._augs.append(GaussianNoise(probability, noise_std))
        return self

    def random_crop(self, probability=0.5, padding=4):
        self._augs.append(RandomCrop(probability, padding))
        return self

    def cutout(self, probability=0.5, cutout_size=8):
        self._augs.append(Cutout(probability, cutout_size))
        return self

    def normalize(self, mean=(0.485, 0.456, 0.406), std=(0.229, 0.224, 0.225)):
        self._augs.append(Normalization(mean, std))
        return self

    def build(self, seed: int = 0) -> AugmentationStrategy:
        return AugmentationStrategy(self._augs, seed)
