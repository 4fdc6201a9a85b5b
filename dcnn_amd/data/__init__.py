"""Data loading and augmentation (native parsers / JPEG decoder / augmentation kernels)."""
from .augmentation import (Augmentation, AugmentationBuilder, AugmentationStrategy, Brightness, Contrast,  # noqa
                           Cutout, GaussianNoise, HorizontalFlip, Normalization, RandomCrop, Rotation, VerticalFlip)
from .datasets import (CIFAR10DataLoader, CIFAR100DataLoader, MNISTDataLoader, TinyImageNetDataLoader,  # noqa
                       WiFiDataLoader, create_cifar10_loaders, create_cifar100_loaders, create_mnist_loaders,
                       create_tiny_image_loader)
from .loader import ArrayDataLoader, BaseDataLoader, SyntheticDataLoader  # noqa: F401
from .device_loader import DeviceDataLoader, to_device_loader  # noqa: F401
