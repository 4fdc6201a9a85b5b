"""Matrix (reference include/matrix/matrix.hpp) on the native CPU backend and the HIP kernels."""
import pytest
import torch

from dcnn_amd.device import get_cpu, get_gpu
from dcnn_amd.tensor import Matrix


def _check_ops(dev, dtype, tol):
    a = Matrix(37, 53, device=dev, dtype=dtype).fill_random_uniform(1.0, seed=3)
    b = Matrix(53, 29, device=dev, dtype=dtype).fill_random_normal(0.0, 1.0, seed=4)
    A, B = a.data().double().cpu(), b.data().double().cpu()
    assert a.data().data_ptr() % 64 == 0 or dev.is_gpu()
    assert A.abs().max() <= 1.0 and A.std() > 0.3
    c = a @ b
    assert (c.rows, c.cols) == (37, 29)
    torch.testing.assert_close(c.data().double().cpu(), A @ B, rtol=tol, atol=tol)
    torch.testing.assert_close(a.matmul(b, alpha=0.5).data().double().cpu(), 0.5 * (A @ B), rtol=tol, atol=tol)
    s = a + a
    torch.testing.assert_close(s.data().double().cpu(), 2 * A)
    s -= a
    torch.testing.assert_close(s.data().double().cpu(), A)
    torch.testing.assert_close((a * a).data().double().cpu(), A * A, rtol=1e-6, atol=1e-7)
    torch.testing.assert_close((a * 3.0).data().double().cpu(), 3 * A, rtol=1e-6, atol=1e-7)
    torch.testing.assert_close((a / 4.0).data().double().cpu(), A / 4, rtol=1e-6, atol=1e-7)
    torch.testing.assert_close(a.transpose().data().double().cpu(), A.t())
    r = a.reshape(53, 37)
    torch.testing.assert_close(r.data().double().cpu().reshape(-1), A.reshape(-1))
    assert abs(a.sum() - float(A.sum())) < 1e-3
    cl = a.clone()
    cl *= 2.0
    torch.testing.assert_close(a.data().double().cpu(), A)  # clone is a deep copy
    with pytest.raises(ValueError):
        a + b
    with pytest.raises(ValueError):
        a @ a
    with pytest.raises(ZeroDivisionError):
        a / 0.0
    with pytest.raises(ValueError):
        a.reshape(5, 5)


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 1e-4), (torch.float64, 1e-12)])
def test_matrix_cpu(dtype, tol):
    _check_ops(get_cpu(), dtype, tol)


def test_matrix_random_fill_matches_across_devices_seeded():
    a = Matrix(8, 8).fill_random_uniform(2.0, seed=11)
    b = Matrix(8, 8).fill_random_uniform(2.0, seed=11)
    assert torch.equal(a.data(), b.data())


@pytest.mark.gpu
def test_matrix_gpu():
    dev = get_gpu(0)
    _check_ops(dev, torch.float32, 2e-3)
    m = Matrix(64, 64, device=dev).fill(1.0)
    assert m.data().is_cuda
    c = Matrix(8, 8).fill_random_uniform(1.0, seed=5)
    g = c.to(dev)
    torch.testing.assert_close(g.data().cpu(), c.data())
    # the same Philox stream on both devices
    torch.testing.assert_close(Matrix(8, 8, device=dev).fill_random_uniform(2.0, seed=11).data().cpu(),
                               Matrix(8, 8).fill_random_uniform(2.0, seed=11).data())
