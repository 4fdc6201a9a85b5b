"""Generic ops + tensor ops: CPU semantics (reference tensor_ops / ops tests) and GPU HIP
kernels against the CPU reference."""
import pytest
import torch

from dcnn_amd.ops import generic as G
from dcnn_amd.tensor import ops as T


def test_tensor_ops_cpu_semantics():
    x = torch.arange(2 * 3 * 4 * 5, dtype=torch.float32).view(2, 3, 4, 5)
    p = T.pad(x, 1, 2)
    assert p.shape == (2, 3, 6, 9) and torch.equal(p[:, :, 1:5, 2:7], x) and p[0, 0, 0, 0] == 0
    assert torch.equal(T.unpad(p, 1, 2), x)
    c = T.crop(x, 1, 1, 2, 3)
    assert torch.equal(c, x[:, :, 1:3, 1:4])
    with pytest.raises(ValueError):
        T.crop(x, 0, 0, 4, 1)
    parts = T.split(torch.arange(7.0).view(7, 1, 1, 1), 3)
    assert [q.shape[0] for q in parts] == [2, 2, 3]
    assert torch.equal(T.slice_channels(x, 1, 3), x[:, 1:3])
    col = T.im2col(x, 3, 3, 1, 1, 1, 1)
    assert col.shape == (3 * 9, 2 * 4 * 5)
    back = T.col2im(col, x.shape, 3, 3, 1, 1, 1, 1)
    ones = T.col2im(T.im2col(torch.ones_like(x), 3, 3, 1, 1, 1, 1), x.shape, 3, 3, 1, 1, 1, 1)
    torch.testing.assert_close(back, x * ones)
    s = T.apply_softmax(torch.randn(2, 5, 3, 3))
    torch.testing.assert_close(s.sum(1), torch.ones(2, 3, 3))


def test_generic_ops_cpu():
    a, b = torch.randn(10), torch.randn(10)
    torch.testing.assert_close(G.add(a, b), a + b)
    torch.testing.assert_close(G.sub_mul_scalar(a, 1.0, 2.0), (a - 1) * 2)
    c = b.clone()
    G.fmadd(a, b, c)
    torch.testing.assert_close(c, a * b + b)
    torch.testing.assert_close(G.dot_product(a, b), (a * b).sum().view(1))
    assert G.transpose_2d(torch.arange(6.0), 2, 3).tolist() == [[0, 3], [1, 4], [2, 5]]
    x = torch.randn(2, 3, 4, 4)
    assert torch.equal(G.cnhw_to_nchw(G.nchw_to_cnhw(x)), x)


@pytest.mark.gpu
def test_generic_ops_gpu_match_cpu():
    torch.manual_seed(0)
    n = 1000003
    a, b = torch.randn(n), torch.rand(n) + 0.5
    ag, bg = a.cuda(), b.cuda()
    for name in ["add", "sub", "mul", "div", "min", "max", "equal", "greater"]:
        torch.testing.assert_close(getattr(G, name)(ag, bg).cpu(), getattr(G, name)(a, b))
    for name in ["add_scalar", "mul_scalar", "div_scalar", "scalar_max"]:
        torch.testing.assert_close(getattr(G, name)(ag, 0.7).cpu(), getattr(G, name)(a, 0.7))
    for name in ["sqrt", "rsqrt", "rcp", "abs", "exp", "log", "copy"]:
        torch.testing.assert_close(getattr(G, name)(bg).cpu(), getattr(G, name)(b), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(G.clamp(ag, -0.5, 0.5).cpu(), a.clamp(-0.5, 0.5))
    c = bg.clone()
    G.fnmadd(ag, bg, c)
    torch.testing.assert_close(c.cpu(), b - a * b)
    y = bg.clone()
    G.axpy(0.3, ag, y)
    torch.testing.assert_close(y.cpu(), b + 0.3 * a)
    for name, ref in [("sum", a.sum()), ("norm_squared", (a * a).sum())]:
        torch.testing.assert_close(getattr(G, name)(ag).cpu()[0], ref, rtol=1e-4, atol=1e-2)
    torch.testing.assert_close(G.dot_product(ag, bg).cpu()[0], (a * b).sum(), rtol=1e-4, atol=1e-2)
    torch.testing.assert_close(G.sum_squared_diff(ag, bg).cpu()[0], ((a - b) ** 2).sum(), rtol=1e-4, atol=1e-2)
    u = G.fill_random_uniform(torch.empty(400000, device="cuda"), -2, 3, seed=5).cpu()
    assert u.min() >= -2 and u.max() < 3 and abs(u.mean() - 0.5) < 0.02
    v = G.fill_random_normal(torch.empty(400000, device="cuda"), 1.0, 2.0, seed=6).cpu()
    assert abs(v.mean() - 1.0) < 0.02 and abs(v.std() - 2.0) < 0.02
    m = torch.randn(3, 70, 130)
    torch.testing.assert_close(G.transpose_2d(m.cuda().reshape(-1), 70, 130, 3).cpu(), m.transpose(1, 2))
    x = torch.randn(3, 5, 7, 6)
    torch.testing.assert_close(G.nchw_to_cnhw(x.cuda()).cpu(), G.nchw_to_cnhw(x))
    torch.testing.assert_close(G.cnhw_to_nchw(G.nchw_to_cnhw(x.cuda())).cpu(), x)


@pytest.mark.gpu
def test_tensor_ops_gpu_match_cpu():
    x = torch.randn(2, 3, 9, 7)
    xg = x.cuda()
    torch.testing.assert_close(T.pad(xg, 2, 1, 0.5).cpu(), T.pad(x, 2, 1, 0.5))
    torch.testing.assert_close(T.unpad(xg, 2, 1).cpu(), T.unpad(x, 2, 1))
    torch.testing.assert_close(T.crop(xg, 1, 2, 6, 5).cpu(), T.crop(x, 1, 2, 6, 5))
    torch.testing.assert_close(T.im2col(xg, 3, 3, 2, 2, 1, 1).cpu(), T.im2col(x, 3, 3, 2, 2, 1, 1))
    s = torch.randn(2, 10, 3, 3)
    torch.testing.assert_close(T.apply_softmax(s.cuda()).cpu(), torch.softmax(s, 1), rtol=1e-5, atol=1e-6)
