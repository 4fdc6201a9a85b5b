"""Loader for the in-tree native extensions.

The HIP kernel library (``dcnn_amd/_kernels*.so``) is REQUIRED for every GPU code path: a GPU
op never silently falls back to an eager PyTorch implementation.  ``kernels()`` raises a
clear error when the extension is missing (build it with ``python -m dcnn_amd._build``).
"""
from __future__ import annotations

import importlib
import os

import torch

_kernels = None
_native = None
_err = None


def kernels():
    """Return the compiled HIP kernel module or raise (never fall back)."""
    global _kernels, _err
    if _kernels is None:
        try:
            _kernels = importlib.import_module("dcnn_amd._kernels")
        except ImportError as e:  # pragma: no cover - exercised on a box without a build
            _err = e
            if os.environ.get("DCNN_AUTOBUILD", "1") == "1":
                from .. import _build
                _build.build_kernels()
                _kernels = importlib.import_module("dcnn_amd._kernels")
            else:
                raise RuntimeError(
                    "dcnn_amd HIP kernel library is not built; run `python -m dcnn_amd._build`") from e
    return _kernels


def native():
    """Return the host C++ runtime module (TCP control plane, loaders, hwinfo, ...)."""
    global _native
    if _native is None:
        try:
            _native = importlib.import_module("dcnn_amd._native")
        except ImportError:
            if os.environ.get("DCNN_AUTOBUILD", "1") == "1":
                from .. import _build
                _build.build_native()
                _native = importlib.import_module("dcnn_amd._native")
            else:
                raise
    return _native


def stream_ptr(device: torch.device | None = None) -> int:
    """hipStream_t of PyTorch's current stream (honours torch.cuda.graph capture streams)."""
    return torch.cuda.current_stream(device).cuda_stream


def ptr(t) -> int:
    return 0 if t is None else t.data_ptr()


def dt_code(dtype: torch.dtype) -> int:
    if dtype == torch.float32:
        return 0
    if dtype == torch.bfloat16:
        return 1
    raise TypeError(f"unsupported activation dtype {dtype} (expected float32 or bfloat16)")
