"""Matrix: a dense row-major 2-D array on a framework Device (reference include/matrix/matrix.hpp:22-221).

The reference's ``Matrix<T>`` is a thin owner of an aligned device buffer with elementwise
operators dispatched through ``ops::`` and a random fill; its GEMM benchmark builds on it. Here the
storage is a contiguous tensor from the framework device layer — CPU: 64-byte aligned host memory;
GPU: the native stream-ordered pool of ``_kernels.rt`` (``Device.allocate``) — and every operator
runs on the framework's own kernels: the native C++ backend on the CPU (float32/float64), the HIP
``ops.hip`` kernels on the GPU (float32), through ``ops.generic``. ``a @ b`` is a real GEMM
(native blocked SGEMM/DGEMM on the CPU, the MFMA f32 GEMM on the GPU). Deliberate difference: the
reference's ``operator*(Matrix)`` checks GEMM shapes but multiplies elementwise
(matrix.hpp:173-182); here ``*`` with a Matrix is the elementwise (Hadamard) product under
elementwise shape rules and ``@`` / :meth:`matmul` is the matrix product.
"""
from __future__ import annotations

import random
from typing import Optional, Union

import torch

from .. import ops as _ops_pkg  # noqa: F401  (package import order)
from ..device import Device, get_cpu, get_gpu
from ..ops import cpu as _cpu
from ..ops import generic as G

_ALIGN = 64  # bytes (the reference's MKL_ALIGNMENT)


def _alloc(rows: int, cols: int, dtype: torch.dtype, device: Device, zero: bool = False) -> torch.Tensor:
    n = rows * cols
    if device.is_gpu():
        t = device.allocate(max(n, 1), dtype=dtype, zero=zero)[:n]
    else:
        es = torch.empty((), dtype=dtype).element_size()
        pad = _ALIGN // es
        raw = torch.zeros(n + pad, dtype=dtype) if zero else torch.empty(n + pad, dtype=dtype)
        off = (-raw.data_ptr() // es) % pad  # first element on a 64-byte boundary
        t = raw[off:off + n]
    return t.view(rows, cols)


class Matrix:
    """rows x cols, row-major, float32 (GPU/CPU) or float64 (CPU)."""

    def __init__(self, rows: int = 0, cols: int = 0, data: Optional[torch.Tensor] = None,
                 device: Optional[Device] = None, dtype: torch.dtype = torch.float32):
        self.device = device or get_cpu()
        if self.device.is_gpu() and dtype != torch.float32:
            raise TypeError("GPU matrices are float32")
        self.dtype = dtype
        self._d = _alloc(rows, cols, dtype, self.device)
        if data is not None:
            src = data.reshape(-1)
            if src.numel() != rows * cols:
                raise ValueError("data size does not match rows x cols")
            self._d.view(-1).copy_(src.to(dtype))

    # ---- construction helpers
    @classmethod
    def _wrap(cls, t: torch.Tensor, device: Device) -> "Matrix":
        m = cls.__new__(cls)
        m.device, m.dtype, m._d = device, t.dtype, t
        return m

    @classmethod
    def from_tensor(cls, t: torch.Tensor, device: Optional[Device] = None) -> "Matrix":
        if t.dim() != 2:
            raise ValueError("Matrix.from_tensor takes a 2-D tensor")
        dev = device or (get_gpu(t.device.index or 0) if t.is_cuda else get_cpu())
        return cls(t.shape[0], t.shape[1], t, dev, t.dtype)

    def like(self) -> "Matrix":
        return Matrix._wrap(_alloc(self.rows, self.cols, self.dtype, self.device), self.device)

    # ---- shape / data
    @property
    def rows(self) -> int:
        return self._d.shape[0]

    @property
    def cols(self) -> int:
        return self._d.shape[1]

    def size(self) -> int:
        return self.rows * self.cols

    def data(self) -> torch.Tensor:
        """The backing [rows, cols] tensor (shares storage)."""
        return self._d

    def to_tensor(self) -> torch.Tensor:
        return self._d.detach().cpu().clone()

    def clone(self) -> "Matrix":
        out = self.like()
        out._d.copy_(self._d)
        return out

    def reshape(self, rows: int, cols: int) -> "Matrix":
        if rows * cols != self.size():
            raise ValueError("Total number of elements must remain the same for reshape.")
        out = Matrix._wrap(_alloc(rows, cols, self.dtype, self.device), self.device)
        out._d.view(-1).copy_(self._d.view(-1))
        return out

    def resize(self, rows: int, cols: int) -> None:
        """New shape; contents are undefined afterwards (as in the reference)."""
        if (rows, cols) != (self.rows, self.cols):
            self._d = _alloc(rows, cols, self.dtype, self.device)

    def to(self, device: Device) -> "Matrix":
        return Matrix(self.rows, self.cols, self._d.to(device.torch_device), device, self.dtype)

    # ---- fills
    def fill(self, value: float) -> "Matrix":
        self._d.fill_(value)
        return self

    def fill_random_uniform(self, rng: float, seed: Optional[int] = None) -> "Matrix":
        G.fill_random_uniform(self._d.view(-1), -rng, rng, random.getrandbits(62) if seed is None else seed)
        return self

    def fill_random_normal(self, mean: float, stddev: float, seed: Optional[int] = None) -> "Matrix":
        G.fill_random_normal(self._d.view(-1), mean, stddev, random.getrandbits(62) if seed is None else seed)
        return self

    # ---- elementwise
    def _check(self, o: "Matrix", what: str) -> None:
        if (self.rows, self.cols) != (o.rows, o.cols):
            raise ValueError(f"Matrix dimensions must match for {what}.")

    def _bin(self, o, fn, what, inplace=False):
        self._check(o, what)
        out = self if inplace else self.like()
        fn(self._d.view(-1), o._d.view(-1), out=out._d.view(-1))
        return out

    def __add__(self, o: "Matrix") -> "Matrix":
        return self._bin(o, G.add, "addition")

    def __iadd__(self, o: "Matrix") -> "Matrix":
        return self._bin(o, G.add, "addition", True)

    def __sub__(self, o: "Matrix") -> "Matrix":
        return self._bin(o, G.sub, "subtraction")

    def __isub__(self, o: "Matrix") -> "Matrix":
        return self._bin(o, G.sub, "subtraction", True)

    def __mul__(self, o: Union["Matrix", float]) -> "Matrix":
        if isinstance(o, Matrix):
            return self._bin(o, G.mul, "elementwise product")
        out = self.like()
        G.mul_scalar(self._d.view(-1), float(o), out=out._d.view(-1))
        return out

    __rmul__ = __mul__

    def __imul__(self, o: Union["Matrix", float]) -> "Matrix":
        if isinstance(o, Matrix):
            return self._bin(o, G.mul, "elementwise product", True)
        G.mul_scalar(self._d.view(-1), float(o), out=self._d.view(-1))
        return self

    def __truediv__(self, s: float) -> "Matrix":
        if s == 0:
            raise ZeroDivisionError("Division by zero.")
        out = self.like()
        G.div_scalar(self._d.view(-1), float(s), out=out._d.view(-1))
        return out

    def __itruediv__(self, s: float) -> "Matrix":
        if s == 0:
            raise ZeroDivisionError("Division by zero.")
        G.div_scalar(self._d.view(-1), float(s), out=self._d.view(-1))
        return self

    # ---- GEMM
    def matmul(self, o: "Matrix", alpha: float = 1.0) -> "Matrix":
        """alpha * self @ o on the framework GEMM of the matrices' device."""
        if self.cols != o.rows:
            raise ValueError("Matrix dimensions must match for multiplication.")
        if self.device.is_gpu():
            from ..ops import hip
            bt = G.transpose_2d(o._d.reshape(-1), o.rows, o.cols)  # [N][K] operand
            y = hip.dense_fwd(self._d, bt, None)
            if alpha != 1.0:
                G.mul_scalar(y.view(-1), alpha, out=y.view(-1))
            return Matrix._wrap(y, self.device)
        y = _cpu.gemm(self._d, o._d, alpha=alpha)
        return Matrix._wrap(y, self.device)

    __matmul__ = matmul

    def transpose(self) -> "Matrix":
        t = G.transpose_2d(self._d.reshape(-1), self.rows, self.cols)
        return Matrix._wrap(t.view(self.cols, self.rows), self.device)

    def sum(self) -> float:
        return float(G.sum(self._d.view(-1)))

    def __repr__(self) -> str:
        return f"Matrix({self.rows}x{self.cols}, {str(self.dtype).split('.')[-1]}, {self.device})"
