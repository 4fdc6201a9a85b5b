"""Losses, optimizers, LR schedulers, model zoo and checkpoint format (reference:
`unit_tests/cuda_loss_funcs_test.cpp:70-623`, `include/nn/optimizers.hpp`, `include/nn/schedulers.hpp`,
`include/nn/example_models.hpp`, `include/nn/sequential.hpp:832-915`). Loss semantics follow
`src/nn/loss_impl/cpu/loss_ops.cpp`: one-hot targets, batch-mean losses (MSE/MAE/Huber: mean over
all elements), gradients scaled by the same count."""
import json
import math
import struct

import pytest
import torch

from dcnn_amd.nn import (SGD, Adam, AdamW, LossFactory, OptimizerFactory, SequentialBuilder)
from dcnn_amd.nn.schedulers import SchedulerFactory

LOSSES = ["crossentropy", "softmax_crossentropy", "logsoftmax_crossentropy", "mse", "mae", "huber"]
ALIASES = {"ce": "crossentropy", "softmax_ce": "softmax_crossentropy", "logsoftmax_ce": "logsoftmax_crossentropy",
           "mean_squared_error": "mse", "mean_absolute_error": "mae"}


def _ref_loss_grad(kind, p, t):
    N = p.shape[0]
    if kind == "crossentropy":
        pc = p.clamp(1e-15, 1 - 1e-15)
        return -(t * torch.log(pc)).sum() / N, (p - t) / N
    if kind in ("softmax_crossentropy", "logsoftmax_crossentropy"):
        ls = torch.log_softmax(p.double(), 1).float()
        return -(t * ls).sum() / N, (torch.softmax(p.double(), 1).float() - t) / N
    d = p - t
    n = p.numel()
    if kind == "mse":
        return (d * d).sum() / n, 2 * d / n
    if kind == "mae":
        return d.abs().sum() / n, torch.where(d > 0, torch.ones_like(d), -torch.ones_like(d)) / n
    a = d.abs()
    l = torch.where(a <= 1.0, 0.5 * d * d, a - 0.5)
    return l.sum() / n, torch.where(a <= 1.0, d, torch.sign(d)) / n


def _inputs(kind, N=12, C=7, seed=0):
    g = torch.Generator().manual_seed(seed)
    labels = torch.randint(0, C, (N,), generator=g)
    t = torch.nn.functional.one_hot(labels, C).float()
    p = torch.randn(N, C, generator=g)
    if kind == "crossentropy":
        p = torch.softmax(p, 1)
    return p.view(N, C, 1, 1), t.view(N, C, 1, 1), labels


@pytest.mark.parametrize("kind", LOSSES)
def test_loss_cpu_matches_reference_math(kind):
    lf = LossFactory.create(kind)
    p, t, labels = _inputs(kind)
    loss, grad, correct = lf.loss_and_grad(p, t)
    rl, rg = _ref_loss_grad(kind, p.view(12, 7), t.view(12, 7))
    assert abs(loss.item() - rl.item()) < 1e-5 * max(1.0, abs(rl.item()))
    assert torch.allclose(grad.view(12, 7), rg, atol=1e-6)
    assert grad.shape == p.shape
    assert correct.item() == (p.view(12, 7).argmax(1) == labels).sum().item()
    assert abs(lf.compute_loss(p, t) - rl.item()) < 1e-5 * max(1.0, abs(rl.item()))


@pytest.mark.parametrize("kind", ["crossentropy", "softmax_crossentropy", "logsoftmax_crossentropy"])
def test_integer_labels_equal_one_hot(kind):
    lf = LossFactory.create(kind)
    p, t, labels = _inputs(kind, seed=3)
    l1, g1, c1 = lf.loss_and_grad(p, t)
    l2, g2, c2 = lf.loss_and_grad(p, labels)
    assert torch.allclose(l1, l2) and torch.allclose(g1, g2) and torch.equal(c1, c2)


def test_loss_factory_aliases_and_config():
    for alias, kind in ALIASES.items():
        assert LossFactory.create(alias).name() == kind
    h = LossFactory.create("huber", delta=2.5)
    again = LossFactory.create_from_config(h.get_config())
    assert again.name() == "huber" and again.param == 2.5
    with pytest.raises(ValueError):
        LossFactory.create("nope")


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("kind", LOSSES)
def test_loss_gpu_matches_cpu(kind, dtype):
    """Fused HIP loss kernel (loss + gradient + correct count in one pass) vs the CPU path."""
    lf = LossFactory.create(kind)
    p, t, labels = _inputs(kind, N=64, C=200, seed=5)
    lc, gc, cc = lf.loss_and_grad(p, t)
    pg = p.cuda().to(dtype)
    lg, gg, cg = lf.loss_and_grad(pg, t.cuda())
    lc2, gc2, _ = lf.loss_and_grad(pg.float().cpu(), t)  # same rounded inputs
    tol = 1e-5 if dtype == torch.float32 else 2e-2
    assert abs(lg.item() - lc2.item()) <= tol * max(1.0, abs(lc2.item())) + 1e-6
    assert (gg.float().cpu() - gc2).norm() <= tol * gc2.norm() + 1e-7
    assert cg.item() == (pg.float().cpu().view(64, 200).argmax(1) == labels).sum().item()
    if kind != "crossentropy":
        lgl, ggl, _ = lf.loss_and_grad(pg, labels.cuda()) if "entropy" in kind else (lg, gg, cg)
        assert abs(lgl.item() - lg.item()) < 1e-4 * max(1.0, abs(lg.item()))


# --------------------------------------------------------------------------------- optimizers
def _tiny_model(device=None, dtype=None):
    m = SequentialBuilder().input([4, 6, 6]).conv2d(8, 3, 3, 1, 1, 1, 1).batchnorm().activation("relu") \
        .flatten().dense(5).build()
    m.set_seed(3)
    if device:
        m.set_device(device)
        if dtype is not None:
            m.set_compute_dtype(dtype)
    m.initialize()
    return m


def _set_grads(m, seed):
    g = torch.Generator().manual_seed(seed)
    for gr in m.gradients():
        gr.copy_(torch.randn(gr.shape, generator=g))


@pytest.mark.parametrize("opt_name", ["sgd", "sgd_momentum", "adam", "adam_l2", "adamw"])
def test_optimizer_update_rules(opt_name):
    """Reference update rules (`src/nn/optimizers_impl/cpu/*_kernels.cpp`): SGD p -= lr g; momentum
    v = mu v - lr g, p += v; Adam bias-corrected with eps after the sqrt; weight decay lr*wd*p added
    to the UPDATE (reference L2 form, the moments see the raw gradient) or applied to p first
    (AdamW) — both give the same trajectory, as in the reference kernels."""
    m = _tiny_model()
    p0 = [p.clone() for p in m.parameters()]
    opt = {"sgd": SGD(0.1), "sgd_momentum": SGD(0.1, 0.9), "adam": Adam(0.01),
           "adam_l2": Adam(0.01, weight_decay=0.05), "adamw": AdamW(0.01, weight_decay=0.05)}[opt_name]
    opt.attach(m)
    ref = [p.clone() for p in p0]
    v = [torch.zeros_like(p) for p in p0]
    mm = [torch.zeros_like(p) for p in p0]
    vv = [torch.zeros_like(p) for p in p0]
    for step in range(1, 4):
        _set_grads(m, step)
        grads = [g.clone() for g in m.gradients()]
        opt.update()
        for i, (r, g) in enumerate(zip(ref, grads)):
            if opt_name == "sgd":
                r -= 0.1 * g
            elif opt_name == "sgd_momentum":
                v[i] = 0.9 * v[i] - 0.1 * g
                r += v[i]
            else:
                mm[i] = 0.9 * mm[i] + 0.1 * g
                vv[i] = 0.999 * vv[i] + 0.001 * g * g
                mh = mm[i] / (1 - 0.9 ** step)
                vh = vv[i] / (1 - 0.999 ** step)
                upd = mh / (vh.sqrt() + 1e-8)
                if opt_name == "adam":
                    r -= 0.01 * upd
                else:  # L2: decay added to the update (adam_kernels.cpp:44-51); AdamW: decoupled
                    r -= 0.01 * (upd + 0.05 * r)
        for p, r in zip(m.parameters(), ref):
            assert torch.allclose(p, r, atol=1e-6, rtol=1e-5), (opt_name, step)
    opt.clear_gradients()
    assert all((g == 0).all() for g in m.gradients())


def test_optimizer_factory_and_config():
    for cfg in ({"type": "sgd", "parameters": {"learning_rate": 0.2, "momentum": 0.5}},
                {"type": "adam", "parameters": {"learning_rate": 0.003}},
                {"type": "adamw", "parameters": {"learning_rate": 0.004, "weight_decay": 0.02}}):
        o = OptimizerFactory.create_from_config(cfg)
        assert abs(o.get_learning_rate() - cfg["parameters"]["learning_rate"]) < 1e-12
    o = SGD(0.3)
    o.set_learning_rate(0.05)
    assert o.get_learning_rate() == 0.05


@pytest.mark.gpu
@pytest.mark.parametrize("opt_name", ["sgd_momentum", "adam", "adamw"])
def test_optimizer_gpu_matches_cpu(opt_name):
    """Flat-arena fused optimizer kernels (one launch for all parameters, device-side step
    scalars) follow the CPU update rule and refresh the bf16 weight shadow."""
    mc = _tiny_model()
    mg = _tiny_model("GPU:0")
    mg.load_parameters([p.clone() for p in mc.parameters()])
    mk = {"sgd_momentum": lambda: SGD(0.1, 0.9), "adam": lambda: Adam(0.01), "adamw": lambda: AdamW(0.01, 0.9, 0.999,
                                                                                                   1e-8, 0.05)}
    oc, og = mk[opt_name](), mk[opt_name]()
    oc.attach(mc)
    og.attach(mg)
    for step in range(1, 4):
        _set_grads(mc, step)
        for a, b in zip(mg.gradients(), mc.gradients()):
            a.copy_(b)
        oc.update()
        og.update()
    for a, b in zip(mg.parameters(), mc.parameters()):
        assert torch.allclose(a.cpu(), b, atol=1e-5, rtol=1e-4)
    if mg.arena.shadow is not None:
        assert torch.allclose(mg.arena.shadow.float().cpu(), mg.arena.data.cpu(), atol=1e-2, rtol=1e-2)


# --------------------------------------------------------------------------------- schedulers
def _lrs(sched, n, metrics=None):
    out = []
    for i in range(n):
        sched.step(metrics[i]) if metrics is not None else sched.step()
        out.append(sched.get_lr())
    return out


@pytest.mark.parametrize("name,params,expect", [
    ("step_lr", {"step_size": 2, "gamma": 0.5}, lambda k: 0.1 * 0.5 ** (k // 2)),
    ("multi_step_lr", {"milestones": [2, 5], "gamma": 0.1}, lambda k: 0.1 * 0.1 ** ((k >= 2) + (k >= 5))),
    ("exponential_lr", {"gamma": 0.9}, lambda k: 0.1 * 0.9 ** k),
    ("cosine_annealing_lr", {"T_max": 10, "eta_min": 0.01},
     lambda k: 0.01 + 0.09 * (1 + math.cos(math.pi * (k % 10) / 10)) / 2),
    ("polynomial_lr", {"total_steps": 8, "power": 2.0, "end_lr": 0.001},
     lambda k: 0.099 * (1 - min(k / 8, 1)) ** 2 + 0.001),
    ("linear_warmup", {"warmup_steps": 4, "start_lr": 0.0}, lambda k: 0.1 * min(k, 4) / 4),
])
def test_scheduler_closed_forms(name, params, expect):
    opt = SGD(0.1)
    s = SchedulerFactory.create(name, opt, params)
    got = _lrs(s, 9)
    for k, g in enumerate(got, start=1):
        assert abs(g - expect(k)) < 1e-9, (name, k, g, expect(k))
    assert s.get_current_step() == 9
    again = SchedulerFactory.create_from_config(s.get_config(), SGD(0.1))
    assert type(again) is type(s)


def test_warm_restarts_onecycle_warmup_cosine_and_plateau():
    s = SchedulerFactory.create("cosine_annealing_warm_restarts", SGD(0.1), {"T_0": 3, "T_mult": 2})
    lrs = _lrs(s, 9)
    assert abs(lrs[2] - 0.1) < 1e-12 and lrs[1] < lrs[0]     # restart after 3 steps
    assert abs(lrs[8] - 0.1) < 1e-12                          # second period of 6 steps
    o = SchedulerFactory.create("one_cycle_lr", SGD(0.1), {"max_lr": 1.0, "total_steps": 10, "pct_start": 0.3})
    lrs = _lrs(o, 10)
    assert abs(lrs[2] - 1.0) < 1e-9 and lrs[-1] < 1e-3 and max(lrs) <= 1.0 + 1e-12
    w = SchedulerFactory.create("warmup_cosine_annealing", SGD(0.1), {"warmup_steps": 2, "total_steps": 6})
    lrs = _lrs(w, 6)
    assert abs(lrs[1] - 0.1) < 1e-12 and abs(lrs[-1]) < 1e-12
    p = SchedulerFactory.create("reduce_lr_on_plateau", SGD(0.1), {"patience": 2, "factor": 0.5})
    lrs = _lrs(p, 6, metrics=[1.0, 0.9, 0.95, 0.96, 0.97, 0.98])
    assert lrs[3] == pytest.approx(0.05) and lrs[5] == pytest.approx(0.025)
    p.reset()
    assert p.get_lr() == 0.1 and p.get_current_step() == 0


# --------------------------------------------------------------------------------- model zoo
ZOO_PARAMS = {  # reference builders (include/nn/example_models.hpp) — parameter counts of this build
    "resnet18_tiny_imagenet": (11.0e6, 11.5e6),
    "resnet50_tiny_imagenet": (23.0e6, 24.5e6),
    "resnet50_imagenet": (25.0e6, 26.5e6),
}


@pytest.mark.parametrize("name", ["mnist_cnn", "cifar10_cnn_v1", "cifar10_cnn_v2", "resnet9_cifar10", "resnet18_cifar10",
                                  "resnet20_cifar10", "resnet50_cifar10", "resnet9_tiny_imagenet",
                                  "cnn_tiny_imagenet", "resnet18_tiny_imagenet", "resnet34_tiny_imagenet",
                                  "resnet50_tiny_imagenet", "resnet50_imagenet"])
def test_model_zoo_shapes(name):
    from dcnn_amd.models import INPUT_SHAPES, NUM_CLASSES, create_model
    m = create_model(name)
    C, H, W = INPUT_SHAPES[name]
    assert m.compute_output_shape([2, C, H, W]) == [2, NUM_CLASSES[name], 1, 1]
    m.set_seed(1)
    m.initialize()
    n = m.num_parameters()
    if name in ZOO_PARAMS:
        lo, hi = ZOO_PARAMS[name]
        assert lo <= n <= hi, (name, n)
    if H <= 64 and n < 30e6:
        y = m.forward(torch.randn(2, C, H, W))
        assert y.shape == (2, NUM_CLASSES[name], 1, 1) and torch.isfinite(y).all()
    assert m.forward_flops([1, C, H, W]) > 0


# --------------------------------------------------------------------------------- checkpoint format
def test_checkpoint_bin_layout_and_roundtrip(tmp_path):
    """`.bin` = concatenation, in layer / parameters() order, of {u64 shape[4]; f32 data}; `.json`
    = {name, is_training, layers:[{type, name, parameters}]} (`include/nn/sequential.hpp:832-915`)."""
    from dcnn_amd.nn import Sequential
    m = _tiny_model()
    path = str(tmp_path / "model")
    m.save_to_file(path)
    cfg = json.load(open(path + ".json"))
    assert {"name", "layers"} <= set(cfg) and [l["type"] for l in cfg["layers"]][:2] == ["conv2d", "batchnorm"]
    raw = open(path + ".bin", "rb").read()
    off = 0
    for p in m.parameters():
        shape = struct.unpack_from("<4Q", raw, off)
        off += 32
        assert list(shape) == list(p.shape) + [1] * (4 - p.dim())
        n = p.numel()
        vals = torch.tensor(struct.unpack_from(f"<{n}f", raw, off))
        off += 4 * n
        assert torch.equal(vals, p.detach().reshape(-1))
    assert off == len(raw)
    m2 = Sequential.from_file(path)
    for a, b in zip(m.parameters(), m2.parameters()):
        assert torch.equal(a, b)
    x = torch.randn(3, 4, 6, 6)
    m.set_training(False)
    m2.set_training(False)
    assert torch.allclose(m.forward(x), m2.forward(x))
