"""Native CPU backend (csrc/native/cpu_ops.cpp, cpu_gemm.cpp) against ATen as the oracle, in
float32 (1e-4 relative) and float64 (1e-10): GEMM in every transpose combination, generic
elementwise/reduction ops, layout ops, conv fwd/bwd (incl. stride/padding/1x1), dense, batch and
group norm, pooling, activations, losses and optimizer steps; thread-count determinism."""
import pytest
import torch
import torch.nn.functional as F

from dcnn_amd.ops import cpu

DTYPES = [torch.float32, torch.float64]


def tol(dt):
    return dict(rtol=1e-4, atol=1e-5) if dt == torch.float32 else dict(rtol=1e-10, atol=1e-12)


def rnd(*shape, dt=torch.float32, seed=0):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(*shape, generator=g, dtype=torch.float64).to(dt)


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("ta,tb", [(False, False), (False, True), (True, False), (True, True)])
@pytest.mark.parametrize("mnk", [(1, 1, 1), (7, 13, 5), (70, 37, 300), (130, 250, 64)])
def test_gemm(dt, ta, tb, mnk):
    M, N, K = mnk
    a = rnd(*((K, M) if ta else (M, K)), dt=dt, seed=1)
    b = rnd(*((N, K) if tb else (K, N)), dt=dt, seed=2)
    c0 = rnd(M, N, dt=dt, seed=3)
    ref = 0.5 * (a.t() if ta else a) @ (b.t() if tb else b) + 2.0 * c0
    out = cpu.gemm(a, b, ta, tb, alpha=0.5, beta=2.0, out=c0.clone())
    torch.testing.assert_close(out, ref, **tol(dt))


def test_gemm_deterministic_across_thread_counts():
    a, b = rnd(300, 200, seed=4), rnd(200, 170, seed=5)
    prev = cpu.get_num_threads()
    try:
        cpu.set_num_threads(1)
        r1 = cpu.gemm(a, b)
        cpu.set_num_threads(max(2, prev))
        r2 = cpu.gemm(a, b)
    finally:
        cpu.set_num_threads(prev)
    assert torch.equal(r1, r2)


@pytest.mark.parametrize("dt", DTYPES)
def test_elementwise_and_reduce(dt):
    from dcnn_amd.ops import generic as G
    a = rnd(1000, dt=dt, seed=6).abs() + 0.1
    b = rnd(1000, dt=dt, seed=7).abs() + 0.1
    for name, fn in [("add", torch.add), ("sub", torch.sub), ("mul", torch.mul), ("div", torch.div),
                     ("min", torch.minimum), ("max", torch.maximum)]:
        torch.testing.assert_close(getattr(G, name)(a, b), fn(a, b), **tol(dt))
    for name, fn in [("sqrt", torch.sqrt), ("rsqrt", torch.rsqrt), ("exp", torch.exp), ("log", torch.log),
                     ("abs", torch.abs)]:
        torch.testing.assert_close(getattr(G, name)(a), fn(a), **tol(dt))
    torch.testing.assert_close(G.clamp(a, 0.5, 1.0), a.clamp(0.5, 1.0), **tol(dt))
    torch.testing.assert_close(G.mul_add_scalar(a, 2.0, 3.0), a * 2 + 3, **tol(dt))
    c = b.clone()
    G.fmadd(a, b, c)
    torch.testing.assert_close(c, a * b + b, **tol(dt))
    y = b.clone()
    G.axpy(0.25, a, y)
    torch.testing.assert_close(y, b + 0.25 * a, **tol(dt))
    torch.testing.assert_close(G.sum(a), a.sum().view(1), **tol(dt))
    torch.testing.assert_close(G.dot_product(a, b), (a * b).sum().view(1), **tol(dt))
    torch.testing.assert_close(G.sum_squared_diff(a, b), ((a - b) ** 2).sum().view(1), **tol(dt))


def test_random_fill_matches_gpu_philox_statistics():
    from dcnn_amd.ops import generic as G
    a = torch.empty(100003)
    G.fill_random_uniform(a, -1.0, 1.0, seed=9)
    assert -1.0 <= float(a.min()) and float(a.max()) < 1.0 and abs(float(a.mean())) < 0.02
    b = torch.empty(100003)
    G.fill_random_uniform(b, -1.0, 1.0, seed=9)
    assert torch.equal(a, b)
    n = torch.empty(200000)
    G.fill_random_normal(n, 1.0, 2.0, seed=3)
    assert abs(float(n.mean()) - 1.0) < 0.03 and abs(float(n.std()) - 2.0) < 0.03


@pytest.mark.parametrize("dt", DTYPES)
def test_layout_ops(dt):
    x = rnd(2, 3, 5, 7, dt=dt, seed=8)
    torch.testing.assert_close(cpu.transpose_2d(x, 6, 35), x.reshape(6, 35).t().contiguous())
    torch.testing.assert_close(cpu.swap01(x), x.permute(1, 0, 2, 3).contiguous())
    torch.testing.assert_close(cpu.pad2d(x, 2, 1, 0.5), F.pad(x, (1, 1, 2, 2), value=0.5))
    torch.testing.assert_close(cpu.crop2d(x, 1, 2, 3, 4), x[:, :, 1:4, 2:6].contiguous())
    col = cpu.im2col(x, 3, 3, 2, 1, 1, 1)
    ref = F.unfold(x, (3, 3), padding=(1, 1), stride=(2, 1))  # [N, C*9, L]
    torch.testing.assert_close(col, ref.permute(1, 0, 2).reshape(ref.shape[1], -1), **tol(dt))
    back = cpu.col2im(col, x.shape, 3, 3, 2, 1, 1, 1)
    refb = F.fold(ref, (5, 7), (3, 3), padding=(1, 1), stride=(2, 1))
    torch.testing.assert_close(back, refb, **tol(dt))


CONV_CASES = [
    # N, Ci, H, W, Co, K, stride, pad
    (4, 3, 9, 9, 8, 3, 1, 1),
    (3, 5, 10, 7, 6, 3, 2, 1),
    (2, 8, 6, 6, 16, 1, 1, 0),
    (20, 4, 5, 5, 3, 3, 1, 0),   # many samples: spread over the pool
    (1, 2, 11, 11, 4, 5, 2, 2),
]


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("case", CONV_CASES)
def test_conv2d(dt, case):
    N, Ci, H, W, Co, K, s, pd = case
    x = rnd(N, Ci, H, W, dt=dt, seed=10)
    w = rnd(Co, Ci, K, K, dt=dt, seed=11) * 0.3
    b = rnd(Co, dt=dt, seed=12)
    y = cpu.conv2d_fwd(x, w, b, (s, s), (pd, pd))
    torch.testing.assert_close(y, F.conv2d(x, w, b, s, pd), **tol(dt))
    dy = rnd(*y.shape, dt=dt, seed=13)
    gw = torch.ones_like(w)      # accumulates
    gb = torch.ones_like(b)
    dx = cpu.conv2d_bwd(x, w, dy, (s, s), (pd, pd), gw, gb)
    xr, wr = x.clone().requires_grad_(), w.clone().requires_grad_()
    F.conv2d(xr, wr, None, s, pd).backward(dy)
    torch.testing.assert_close(dx, xr.grad, **tol(dt))
    torch.testing.assert_close(gw, 1 + wr.grad, **tol(dt))
    torch.testing.assert_close(gb, 1 + dy.sum((0, 2, 3)), **tol(dt))


@pytest.mark.parametrize("dt", DTYPES)
def test_dense(dt):
    x, w, b = rnd(9, 17, dt=dt, seed=14), rnd(5, 17, dt=dt, seed=15), rnd(5, dt=dt, seed=16)
    torch.testing.assert_close(cpu.dense_fwd(x, w, b), F.linear(x, w, b), **tol(dt))
    dy = rnd(9, 5, dt=dt, seed=17)
    gw, gb = torch.zeros_like(w), torch.zeros_like(b)
    dx = cpu.dense_bwd(x, w, dy, gw, gb)
    torch.testing.assert_close(dx, dy @ w, **tol(dt))
    torch.testing.assert_close(gw, dy.t() @ x, **tol(dt))
    torch.testing.assert_close(gb, dy.sum(0), **tol(dt))


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("relu,res", [(False, False), (True, False), (True, True)])
def test_batchnorm(dt, relu, res):
    x = rnd(6, 4, 5, 5, dt=dt, seed=18) * 3 + 1
    g, be = rnd(4, dt=dt, seed=19), rnd(4, dt=dt, seed=20)
    r = rnd(*x.shape, dt=dt, seed=21) if res else None
    rm, rv = torch.zeros(4, dtype=dt), torch.ones(4, dtype=dt)
    y, mean, istd = cpu.batchnorm_fwd(x, g, be, 1e-5, True, rm, rv, 0.1, relu=relu, residual=r)
    xr = x.clone().requires_grad_()
    gr, br = g.clone().requires_grad_(), be.clone().requires_grad_()
    rm2, rv2 = torch.zeros(4, dtype=dt), torch.ones(4, dtype=dt)
    ref = F.batch_norm(xr, rm2, rv2, gr, br, True, 0.1, 1e-5)
    if r is not None:
        ref = ref + r
    if relu:
        ref = torch.relu(ref)
    torch.testing.assert_close(y, ref, **tol(dt))
    torch.testing.assert_close(rm, rm2, **tol(dt))
    torch.testing.assert_close(rv, rv2, **tol(dt))
    dy = rnd(*x.shape, dt=dt, seed=22)
    ref.backward(dy)
    dg, db = torch.zeros(4, dtype=dt), torch.zeros(4, dtype=dt)
    dx, masked = cpu.batchnorm_bwd(x, dy, y if relu else None, mean, istd, g, dg, db, True, want_masked=True)
    torch.testing.assert_close(dx, xr.grad, **tol(dt))
    torch.testing.assert_close(dg, gr.grad, **tol(dt))
    torch.testing.assert_close(db, br.grad, **tol(dt))
    if relu:
        torch.testing.assert_close(masked, dy * (y > 0), **tol(dt))


def test_batchnorm_large_mean_matches_fp64_variance():
    """Two-pass statistics: mean 1e3, std 1 inputs keep their variance to 1e-3 in float32."""
    x = (rnd(64, 3, 8, 8, seed=23) + 1000.0).float()
    _, mean, istd = cpu.batchnorm_fwd(x, None, None, 0.0, True, None, None, 0.1)
    var = 1.0 / istd.double() ** 2
    ref = x.double().var((0, 2, 3), unbiased=False)
    assert torch.allclose(var, ref, rtol=1e-3)


@pytest.mark.parametrize("dt", DTYPES)
def test_groupnorm(dt):
    x = rnd(3, 6, 4, 4, dt=dt, seed=24)
    g, be = rnd(6, dt=dt, seed=25), rnd(6, dt=dt, seed=26)
    y, mean, istd = cpu.groupnorm_fwd(x, 3, g, be, 1e-5)
    xr, gr, br = x.clone().requires_grad_(), g.clone().requires_grad_(), be.clone().requires_grad_()
    ref = F.group_norm(xr, 3, gr, br, 1e-5)
    torch.testing.assert_close(y, ref, **tol(dt))
    dy = rnd(*x.shape, dt=dt, seed=27)
    ref.backward(dy)
    dg, db = torch.zeros(6, dtype=dt), torch.zeros(6, dtype=dt)
    dx = cpu.groupnorm_bwd(x, dy, 3, g, mean, istd, dg, db)
    torch.testing.assert_close(dx, xr.grad, **tol(dt))
    torch.testing.assert_close(dg, gr.grad, **tol(dt))
    torch.testing.assert_close(db, br.grad, **tol(dt))


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("k,s,pd", [(2, 2, 0), (3, 2, 1), (3, 1, 1)])
def test_pools(dt, k, s, pd):
    x = rnd(2, 3, 9, 8, dt=dt, seed=28)
    y, idx = cpu.maxpool_fwd(x, (k, k), (s, s), (pd, pd))
    xr = x.clone().requires_grad_()
    ref = F.max_pool2d(xr, k, s, pd)
    torch.testing.assert_close(y, ref)
    dy = rnd(*y.shape, dt=dt, seed=29)
    ref.backward(dy)
    torch.testing.assert_close(cpu.maxpool_bwd(dy, idx, x.shape), xr.grad, **tol(dt))
    ya = cpu.avgpool_fwd(x, (k, k), (s, s), (pd, pd))
    xr2 = x.clone().requires_grad_()
    refa = F.avg_pool2d(xr2, k, s, pd)
    torch.testing.assert_close(ya, refa, **tol(dt))
    refa.backward(dy)
    torch.testing.assert_close(cpu.avgpool_bwd(dy, x.shape, (k, k), (s, s), (pd, pd)), xr2.grad, **tol(dt))


@pytest.mark.parametrize("dt", DTYPES)
def test_activations_and_softmax(dt):
    x = rnd(2, 5, 3, 3, dt=dt, seed=30)
    dy = rnd(2, 5, 3, 3, dt=dt, seed=31)
    for kind, fn in [("relu", torch.relu), ("leaky_relu", lambda t: F.leaky_relu(t, 0.01)),
                     ("elu", lambda t: F.elu(t, 1.0)), ("sigmoid", torch.sigmoid), ("tanh", torch.tanh)]:
        alpha = 0.01 if kind == "leaky_relu" else 1.0
        xr = x.clone().requires_grad_()
        ref = fn(xr)
        ref.backward(dy)
        torch.testing.assert_close(cpu.act_fwd(x, kind, alpha), ref.detach(), **tol(dt))
        torch.testing.assert_close(cpu.act_bwd(x, dy, kind, alpha), xr.grad, **tol(dt))
    xr = x.clone().requires_grad_()
    ref = torch.softmax(xr, 1)
    ref.backward(dy)
    y = cpu.softmax_channels(x)
    torch.testing.assert_close(y, ref.detach(), **tol(dt))
    torch.testing.assert_close(cpu.softmax_channels_bwd(y, dy), xr.grad, **tol(dt))


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("kind", ["softmax_crossentropy", "crossentropy", "mse", "mae", "huber"])
def test_losses(dt, kind):
    from dcnn_amd.nn.loss import LossFactory
    lf = LossFactory.create(kind)
    pred = rnd(8, 5, dt=dt, seed=32)
    if kind == "crossentropy":
        pred = torch.softmax(pred, 1)
    lab = torch.randint(0, 5, (8,), generator=torch.Generator().manual_seed(3))
    tgt = F.one_hot(lab, 5).to(dt)
    loss, grad, cor = cpu.loss_fused(pred, tgt, None, kind, lf.param)
    ref_l = lf._cpu_loss(pred.double(), tgt.double())
    ref_g = lf._cpu_grad(pred.double(), tgt.double())
    if kind == "softmax_crossentropy":  # (the oracle rounds this one through float32)
        ref_g = (torch.softmax(pred.double(), 1) - tgt.double()) / pred.shape[0]
    # (the oracle's loss is rounded to float32 for some kinds)
    torch.testing.assert_close(loss.double(), ref_l.view(1).double(), rtol=1e-6, atol=1e-7)
    torch.testing.assert_close(grad.double(), ref_g.double(), **tol(dt))
    assert int(cor) == int((pred.argmax(1) == lab).sum())
    l2, g2, c2 = cpu.loss_fused(pred, None, lab, kind, lf.param)
    assert torch.equal(l2, loss) and torch.equal(g2, grad) and int(c2) == int(cor)


@pytest.mark.parametrize("dt", DTYPES)
def test_optimizer_steps(dt):
    p0, g = rnd(100, dt=dt, seed=33), rnd(100, dt=dt, seed=34)
    p, v = p0.clone(), torch.zeros_like(p0)
    cpu.sgd_step(p, g, v, 0.1, 0.9)
    torch.testing.assert_close(p, p0 - 0.1 * g, **tol(dt))
    p, m, vv = p0.clone(), torch.zeros_like(p0), torch.zeros_like(p0)
    cpu.adam_step(p, g, m, vv, 1e-3, 0.9, 0.999, 1e-8, 0.1, 0.001, 0.0, 0)
    mh, vh = 0.1 * g / 0.1, 0.001 * g * g / 0.001
    torch.testing.assert_close(p, p0 - 1e-3 * mh / (vh.sqrt() + 1e-8), **tol(dt))


def _train_cpu(dtype, steps=3, adam=True):
    from dcnn_amd.models import zoo
    from dcnn_amd.nn import SGD, Adam, LossFactory
    m = zoo.create_model("mnist_cnn")
    m.set_seed(3)
    m.set_compute_dtype(dtype)
    m.initialize()
    opt = Adam(1e-3) if adam else SGD(0.05, 0.9)
    opt.attach(m)
    lf = LossFactory.create("softmax_crossentropy")
    g = torch.Generator().manual_seed(1)
    x = torch.randn(16, 1, 28, 28, generator=g)
    y = torch.randint(0, 10, (16,), generator=g)
    losses = []
    for _ in range(steps):
        opt.clear_gradients()
        out = m.forward(x)
        loss, grad, _ = lf.loss_and_grad(out, y)
        m.backward(grad)
        opt.update()
        losses.append(float(loss))
    return m, losses


def test_fp64_model_trains_and_tracks_fp32():
    """A float64 CPU model (double master weights, gradients and optimizer state, the reference's
    dkernels/dgemm path) trains and agrees with the float32 model to float32 precision (SGD: Adam's
    normalised step would amplify rounding on near-zero gradients)."""
    m64, l64 = _train_cpu(torch.float64, adam=False)
    m32, l32 = _train_cpu(torch.float32, adam=False)
    assert m64.arena.data.dtype == torch.float64 and m64.arena.grad.dtype == torch.float64
    assert l64[-1] < l64[0]
    for a, b in zip(l64, l32):
        assert abs(a - b) < 1e-4 * max(1.0, abs(a))
    for p64, p32 in zip(m64.parameters(), m32.parameters()):
        torch.testing.assert_close(p64.float(), p32, rtol=1e-3, atol=1e-5)


def test_cpu_training_is_deterministic_across_thread_counts():
    prev = cpu.get_num_threads()
    try:
        cpu.set_num_threads(1)
        m1, l1 = _train_cpu(torch.float32, 2)
        cpu.set_num_threads(max(2, prev))
        m2, l2 = _train_cpu(torch.float32, 2)
    finally:
        cpu.set_num_threads(prev)
    assert l1 == l2
    assert torch.equal(m1.arena.data, m2.arena.data)
