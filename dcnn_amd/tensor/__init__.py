"""Matrix and tensor ops (im2col/col2im, pad/unpad/crop, slicing, micro-batch split, channel softmax)."""
from .ops import apply_softmax, col2im, crop, im2col, pad, slice_batch, slice_channels, split, unpad  # noqa: F401
from .matrix import Matrix  # noqa: F401
