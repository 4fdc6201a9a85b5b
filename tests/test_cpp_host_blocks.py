"""C++ host API beyond plain CNNs (csrc/host/nn.cpp, train.cpp; examples/cpp/host_api_parity.cpp,
tiny_imagenet_resnet18.cpp): residual blocks (basic / bottleneck builders), GroupNorm, Dropout,
softmax, the six losses, the ten schedulers and the model zoo — checked against the Python front
end on the same inputs (checkpoints cross in both directions), and the routed MFMA conv kernels on
the GPU against the C++ CPU backend."""
import os
import re
import subprocess
import sys

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "dcnn_amd", "bin")
NAMES = ("host_api_parity", "tiny_imagenet_resnet18")


@pytest.fixture(scope="module")
def bins():
    have = all(os.path.exists(os.path.join(BIN, n)) for n in NAMES)
    if not (have and torch.cuda.is_available()):
        from dcnn_amd import _build
        _build.build_host()
    return {n: os.path.join(BIN, n) for n in NAMES}


def _run(cmd, cwd, timeout=600):
    r = subprocess.run(cmd, cwd=cwd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=timeout)
    assert r.returncode == 0, r.stdout[-3000:]
    return r.stdout


def _lines(out):
    d = {}
    for l in out.splitlines():
        parts = l.split()
        if parts:
            d[parts[0]] = parts[1:]
    return d


SCHED = [("step_lr", dict(step_size=3, gamma=0.5)), ("multi_step_lr", dict(milestones=[2, 5, 9], gamma=0.3)),
         ("exponential_lr", dict(gamma=0.9)), ("cosine_annealing_lr", dict(T_max=7, eta_min=0.001)),
         ("cosine_annealing_warm_restarts", dict(T_0=3, T_mult=2, eta_min=0.0)),
         ("linear_warmup", dict(warmup_steps=4, start_lr=0.01)),
         ("warmup_cosine_annealing", dict(warmup_steps=3, total_steps=10, start_lr=0.0, eta_min=0.01)),
         ("reduce_lr_on_plateau", dict(mode="min", factor=0.5, patience=2, threshold=1e-4, min_lr=0.001)),
         ("polynomial_lr", dict(total_steps=8, power=2.0, end_lr=0.001)),
         ("one_cycle_lr", dict(max_lr=0.5, total_steps=10, pct_start=0.3, div_factor=25.0, final_div_factor=1e4))]


def test_cpp_schedulers_match_python(bins, tmp_path):
    from dcnn_amd.nn.optimizers import SGD
    from dcnn_amd.nn.schedulers import SchedulerFactory
    got = _lines(_run([bins["host_api_parity"], "schedulers"], tmp_path))
    metrics = [1.0, 0.9, 0.95, 0.95, 0.96, 0.97, 0.5, 0.6, 0.6, 0.6, 0.7, 0.8]
    assert len(got) == 10
    for name, params in SCHED:
        opt = SGD(0.1)
        s = SchedulerFactory.create(name, opt, params)
        ref = [opt.get_learning_rate()]
        for k in range(12):
            s.step(metrics[k]) if name == "reduce_lr_on_plateau" else s.step()
            ref.append(opt.get_learning_rate())
        # (the C++ optimizer keeps its learning rate in float32)
        np.testing.assert_allclose([float(v) for v in got[name]], ref, rtol=2e-6, atol=1e-9, err_msg=name)


def test_cpp_losses_match_python(bins, tmp_path):
    from dcnn_amd.nn.loss import LossFactory
    from dcnn_amd.nn.sequential import save_tensor
    torch.manual_seed(3)
    N, C = 6, 5
    pred = torch.rand(N, C) * 0.9 + 0.05  # valid probabilities-ish for the CE on probabilities too
    with open(tmp_path / "pred.bin", "wb") as f:
        save_tensor(f, pred.view(N, C, 1, 1))
    got = _lines(_run([bins["host_api_parity"], "losses", "pred.bin", str(C)], tmp_path))
    labels = torch.arange(N) % C
    for name in ("crossentropy", "softmax_crossentropy", "logsoftmax_crossentropy", "mse", "mae", "huber"):
        loss, grad, correct = LossFactory.create(name).loss_and_grad(pred.clone(), labels)
        vals = [float(v) for v in got[name]]
        assert vals[0] == pytest.approx(float(loss.reshape(-1)[0]), rel=1e-5), name
        assert int(vals[1]) == int(correct.reshape(-1)[0]), name
        np.testing.assert_allclose(vals[2:], grad.reshape(-1).numpy(), rtol=1e-5, atol=1e-7, err_msg=name)


@pytest.mark.parametrize("model_name,batch", [("resnet18_tiny_imagenet", 2), ("resnet50_tiny_imagenet", 1)])
def test_python_resnet_checkpoint_runs_in_cpp(bins, tmp_path, model_name, batch):
    """Python -> C++: a ResNet (residual_block records with JSON-string sub-layer paths, BN
    statistics after a training step) saved by the Python front end loads in C++ and gives the
    same eval-mode logits."""
    from dcnn_amd.models import create_model
    from dcnn_amd.nn import SGD, LossFactory
    from dcnn_amd.nn.sequential import save_tensor
    m = create_model(model_name)
    m.set_seed(4)
    m.initialize()
    opt = SGD(0.01)
    opt.attach(m)
    g = torch.Generator().manual_seed(9)
    x = torch.randn(batch, 3, 64, 64, generator=g)
    y = torch.randint(0, 200, (batch,), generator=g)
    lf = LossFactory.create("softmax_crossentropy")
    out = m.forward(x)
    _, grad, _ = lf.loss_and_grad(out, y)
    m.backward(grad)
    opt.update()  # moves the weights and the BN running statistics away from their init
    m.set_training(False)
    with torch.no_grad():
        ref = m.forward(x).reshape(batch, -1).double().numpy()
    m.save_to_file(str(tmp_path / "py" / "m"))
    with open(tmp_path / "x.bin", "wb") as f:
        save_tensor(f, x)
    got = _lines(_run([bins["host_api_parity"], "forward", "py/m", "x.bin"], tmp_path))
    assert int(got["params"][0]) == sum(p.numel() for p in m.parameters())
    logits = np.array([float(v) for v in got["logits"]]).reshape(batch, -1)
    rel = np.linalg.norm(logits - ref) / np.linalg.norm(ref)
    assert rel < 1e-4, rel


def test_cpp_resnet_trains_and_loads_in_python(bins, tmp_path):
    """C++ -> Python: ResNet-9 (basic residual blocks) trained by C++ Adam steps, saved, reloaded
    by the Python front end: the same eval-mode logits as the C++ model."""
    from dcnn_amd.nn.sequential import Sequential, save_tensor
    out = _lines(_run([bins["host_api_parity"], "train", "resnet9_cifar10", "4", "4", "snap/r9"], tmp_path))
    losses = [float(v) for v in out["losses"]]
    assert len(losses) == 4 and all(np.isfinite(losses))
    m = Sequential.from_file(str(tmp_path / "snap" / "r9"))
    assert [l.type() for l in m.layers].count("residual_block") == 5
    m.set_training(False)
    x = torch.randn(3, 3, 32, 32, generator=torch.Generator().manual_seed(1))
    with open(tmp_path / "x.bin", "wb") as f:
        save_tensor(f, x)
    got = _lines(_run([bins["host_api_parity"], "forward", "snap/r9", "x.bin"], tmp_path))
    with torch.no_grad():
        ref = m.forward(x).reshape(3, -1).double().numpy()
    cpp = np.array([float(v) for v in got["logits"]]).reshape(3, -1)
    assert np.linalg.norm(cpp - ref) / np.linalg.norm(ref) < 1e-4


def test_cpp_tiny_imagenet_trainer_cpu(bins, tmp_path):
    out = _run([bins["tiny_imagenet_resnet18"], "--device", "CPU", "--model", "resnet9_cifar10", "--batch", "8",
                "--steps", "3", "--epochs", "2", "--lr", "0.003", "--scheduler", "cosine_annealing_lr",
                "--loss", "logsoftmax_ce", "--save", "snap/r9"], tmp_path)
    ep = [float(m) for m in re.findall(r"train loss (\S+)", out)]
    assert len(ep) == 2 and all(np.isfinite(ep)), out
    assert os.path.exists(tmp_path / "snap" / "r9.bnstats")


@pytest.mark.gpu
def test_cpp_resnet_gpu_matches_cpu_backend(bins, tmp_path):
    """The GPU backend's routed conv kernels (halo 3x3 fwd/dgrad, halo wgrad, streaming 1x1,
    stride-phase-grouped gathered GEMM) through residual blocks: a C++-trained ResNet-18 checkpoint
    evaluated on the GPU (bf16) and on the CPU (fp32) agrees to bf16 accuracy."""
    out = _lines(_run([bins["host_api_parity"], "train", "resnet18_tiny_imagenet", "3", "16", "snap/r18",
                       "--device", "GPU"], tmp_path, timeout=300))
    losses = [float(v) for v in out["losses"]]
    assert all(np.isfinite(losses)), losses
    from dcnn_amd.nn.sequential import save_tensor
    x = torch.randn(4, 3, 64, 64, generator=torch.Generator().manual_seed(2))
    with open(tmp_path / "x.bin", "wb") as f:
        save_tensor(f, x)
    g = np.array([float(v) for v in _lines(_run([bins["host_api_parity"], "forward", "snap/r18", "x.bin", "--device",
                                                 "GPU"], tmp_path))["logits"]])
    c = np.array([float(v) for v in _lines(_run([bins["host_api_parity"], "forward", "snap/r18", "x.bin"],
                                                tmp_path))["logits"]])
    assert np.linalg.norm(g - c) / np.linalg.norm(c) < 5e-2


@pytest.mark.gpu
def test_cpp_tiny_imagenet_trainer_gpu_bench(bins, tmp_path):
    out = _run([bins["tiny_imagenet_resnet18"], "--device", "GPU", "--batch", "64", "--steps", "10", "--bench"],
               tmp_path, timeout=300)
    m = re.search(r"\"value\": (\S+),", out)
    assert m and float(m.group(1)) > 0, out
    print(out)


@pytest.mark.gpu
def test_cpp_resnet18_gpu_training_matches_cpu_backend(bins, tmp_path):
    """The GPU backend's fused training path — conv-epilogue BatchNorm statistics, BN + ReLU,
    residual-tail BN with the shortcut add and its masked branch gradient, the dgrad epilogue's
    BN-backward statistics, head-conv shortcut add, deferred weight-gradient reduce, parameter
    arena with the fused Adam step and batched weight transposes — against the CPU backend's
    plain fp32 ops: the same initial weights and batches give the same losses over 3 Adam steps
    to bf16 accuracy."""
    args = ["train", "resnet18_tiny_imagenet", "3", "8"]
    g = [float(v) for v in _lines(_run([bins["host_api_parity"], *args, "snap/g", "--device", "GPU"], tmp_path,
                                       timeout=300))["losses"]]
    c = [float(v) for v in _lines(_run([bins["host_api_parity"], *args, "snap/c"], tmp_path, timeout=600))["losses"]]
    assert len(g) == len(c) == 3
    # (smoke check only: the per-parameter gradient comparison is the test below; later steps
    # carry Adam's sign-sensitive updates of weights whose gradients are bf16 noise)
    np.testing.assert_allclose(g[:2], c[:2], rtol=5e-2)
    np.testing.assert_allclose(g[2], c[2], rtol=1.5e-1)


@pytest.mark.gpu
def test_cpp_resnet18_gpu_gradients_match_cpu_backend(bins, tmp_path):
    """Every parameter gradient of one ResNet-18 step on the C++ GPU backend's fused path (conv
    epilogue statistics, BN + ReLU, residual tails with the shortcut add and masked branch
    gradient, dgrad-epilogue BN-backward statistics, head-conv shortcut add, deferred split-K
    weight-gradient reduce) against the C++ CPU backend's plain fp32 ops on the same weights and
    batch, per parameter (relative L2 error and cosine).

    bf16 activations and gradients compound through 17 BatchNorm backwards of a random-init
    network, so the stem's gradient legitimately drifts from fp32 (cosine ~0.92 at batch 16). The
    yardstick is the Python front end's GPU path — validated layer by layer against fp32 by
    tests/test_gpu_model.py::test_gpu_vs_cpu_model_teacher_forced — run on the same weights and
    batch; the same fused GPU path in exact fp32 must match the CPU to 1e-2 (measured 4e-3: this
    random-init backward amplifies relative rounding ~1000x from the classifier to the stem, which
    is also why bf16 drifts by ~0.4 there — precision, not a fusion error). Per parameter the C++ GPU error may exceed the Python GPU error
    by at most 25% + 0.02,
    the norm ratios to the fp32 gradient within 0.05 of the Python path's, and the classifier's
    gradient (no compounding) to 2e-2. A wrong
    ReLU mask, a swapped statistics slab or a wrong block's shortcut gradient moves the affected
    layers' errors to O(1)."""
    from dcnn_amd.nn import LossFactory
    from dcnn_amd.nn.sequential import Sequential, load_tensor
    from dcnn_amd.parallel.dp import DataParallel
    res = {}
    for dev in ("GPU", "CPU"):
        args = [bins["host_api_parity"], "grads", "resnet18_tiny_imagenet", os.environ.get("DCNN_GRAD_BATCH", "16"),
                f"g_{dev}.bin"]
        if dev == "GPU":
            args += ["snap/init", "--device", "GPU"]
        (tmp_path / "snap").mkdir(exist_ok=True)
        out = _lines(_run(args, tmp_path, timeout=600))
        with open(tmp_path / f"g_{dev}.bin", "rb") as f:
            res[dev] = (float(out["loss"][0]), out["params"], [load_tensor(f).double() for _ in out["params"]])
    lg, names, gg = res["GPU"]
    lc, names_c, gc = res["CPU"]
    assert names == names_c and len(gg) == len(gc) > 40
    assert abs(lg - lc) / abs(lc) < 2e-2
    # the Python front end's GPU step on the same initial weights and batch: bf16 (the yardstick)
    # and exact fp32 (the same fused kernels and fusion plan with IEEE fp32 operands)
    from dcnn_amd.ops import hip
    with open(tmp_path / "snap" / "init.x.bin", "rb") as f:
        x = load_tensor(f).cuda()
    with open(tmp_path / "snap" / "init.y.bin", "rb") as f:
        y = load_tensor(f).reshape(-1).long().cuda()

    def py_grads(dtype):
        m = Sequential.from_file(str(tmp_path / "snap" / "init"), device="GPU:0")
        if dtype == torch.float32:
            m.set_compute_dtype(torch.float32)
        m.set_training(True)
        dp = DataParallel(m, broadcast=False)
        m.clear_gradients()
        out = dp.forward(x)
        _, grad, _ = LossFactory.create("softmax_crossentropy").loss_and_grad(out, y)
        dp.backward(grad, prescaled=True)
        torch.cuda.synchronize()
        g = [t.detach().double().cpu().reshape(c.shape) for t, c in zip(m.gradients(), gc)]
        assert len(g) == len(gc)
        return g

    gp = py_grads(torch.bfloat16)
    concat = hip.get_f32_concat()
    hip.set_f32_concat(False)
    hip.kernels().set_f32_mode(0)
    try:
        g32 = py_grads(torch.float32)
    finally:
        hip.set_f32_concat(concat)

    def err(a, b):
        return float((a - b).norm() / b.norm().clamp_min(1e-30))

    total = sum(float(b.norm()) ** 2 for b in gc) ** 0.5
    numel = sum(b.numel() for b in gc)
    rows, bad = [], []
    for k, (n, a, p, q, b) in enumerate(zip(names, gg, gp, g32, gc)):
        typical = total * (b.numel() / numel) ** 0.5
        if float(b.norm()) < 1e-4 * typical:  # conv bias before BatchNorm: exactly-zero true gradient
            if float(a.norm()) > 0.1 * typical or float(q.norm()) > 1e-2 * typical:
                bad.append((k, n, "zero-gradient parameter", float(a.norm()) / typical, float(q.norm()) / typical))
            continue
        e_cpp, e_py, e32 = err(a, b), err(p, b), err(q, b)
        ratio, ratio_py = float(a.norm() / b.norm()), float(p.norm() / b.norm())
        rows.append((k, n, round(e_cpp, 4), round(e_py, 4), round(ratio, 4), round(ratio_py, 4), round(e32, 6)))
        if e_cpp > 1.25 * e_py + 0.02 or abs(ratio - ratio_py) > 0.05 or e32 > 1e-2:
            bad.append(rows[-1])
    print("per parameter (index, name, C++ GPU bf16 error, Python GPU bf16 error, C++ GPU / CPU norm, "
          "Python GPU / CPU norm, Python GPU exact-fp32 error):", rows)
    assert rows[-1][2] < 2e-2 and rows[-2][2] < 2e-2, rows[-2:]  # classifier weights / bias
    assert not bad, bad

@pytest.mark.gpu
@pytest.mark.parametrize("switch", ["DCNN_STEM_BN_FOLD", "DCNN_BNB_MASK_X"])
def test_cpp_fusion_switch_matches_unfused(bins, tmp_path, switch):
    """Two C++ engine fusions against their switched-off form on the same weights and batch, every
    parameter gradient bit-identical:
    * DCNN_STEM_BN_FOLD: the stem BatchNorm's backward folded into the stem's weight-gradient
      kernel (gpu_ops::stem_wgrad_bn: dy' = A dy + B (x - mean) + D per channel on the staged dY
      tile, the BatchNorm's parameter gradients from the same reduced sums) vs bn_bwd_slab +
      stem_wgrad (same arithmetic and bf16 rounding of dy');
    * DCNN_BNB_MASK_X: the halo dgrad's backward-BatchNorm epilogue recomputing the ReLU mask from
      the BatchNorm input (x * gamma istd + (beta - mean gamma istd) > 0, the forward apply's own
      expressions) vs reading it from the BatchNorm output."""
    from dcnn_amd.nn.sequential import load_tensor
    res = {}
    for fold in ("1", "0"):
        env = dict(os.environ, **{switch: fold})
        r = subprocess.run([bins["host_api_parity"], "grads", "resnet18_tiny_imagenet", "64", f"g{fold}.bin",
                            "--device", "GPU"], cwd=tmp_path, env=env, stdout=subprocess.PIPE,
                           stderr=subprocess.STDOUT, text=True, timeout=600)
        assert r.returncode == 0, r.stdout[-3000:]
        out = _lines(r.stdout)
        with open(tmp_path / f"g{fold}.bin", "rb") as f:
            res[fold] = (out["params"], [load_tensor(f) for _ in out["params"]])
    names, g1 = res["1"]
    names0, g0 = res["0"]
    assert names == names0 and len(g1) > 40
    for n, a, b in zip(names, g1, g0):
        assert torch.equal(a, b), (n, float((a - b).abs().max()), float(b.abs().max()))
    # the fold touches the stem conv and its BatchNorm: their gradients are non-trivial
    assert float(g1[0].abs().max()) > 0 and float(g1[2].abs().max()) > 0


def _segments(out):
    rows = []
    for line in out.splitlines():
        if line.startswith("segment "):
            f = line.split()
            rows.append((f[3], float(f[5]), float(f[7]), float(f[9]), f[10], float(f[12]), float(f[14])))
    return rows


@pytest.mark.gpu
@pytest.mark.parametrize("model,batch", [("resnet18_tiny_imagenet", 64), ("resnet50_tiny_imagenet", 32)])
def test_cpp_gpu_layers_teacher_forced_absolute(bins, tmp_path, model, batch):
    """Every segment of the C++ GPU backend (a top-level layer — residual blocks with all their
    internal fusions — or a BatchNorm with the ReLU / max-pool fused into it) against the CPU
    backend's fp32 step, fed the CPU input and output gradient (teacher forcing: no error
    compounding through the network), with absolute bounds per segment: output, input gradient
    and every parameter gradient to bf16 accuracy. A deliberately dropped BatchNorm ReLU mask in
    the dgrad epilogue (DCNN_TEST_FAULT=1) must fail it.
    Reference parity: unit_tests/layer_device_agnosticity_test.cpp:60-103."""
    out = _run([bins["host_api_parity"], "blocks", model, str(batch), "--device", "GPU"], tmp_path, timeout=600)
    rows = _segments(out)
    assert len(rows) >= 10, out[-2000:]
    print("segments (name, fwd rel, bwd rel, param rel, worst param, bwd cosine, param cosine):")
    for row in rows:
        print(row)
    env = dict(os.environ, DCNN_TEST_FAULT="1")
    r = subprocess.run([bins["host_api_parity"], "blocks", model, str(batch), "--device", "GPU"], cwd=tmp_path,
                       env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=600)
    faulty = _segments(r.stdout)
    print("with the fault:")
    for row in faulty:
        print(row)
    # measured on MI355X (ResNet-18 b64 / ResNet-50 b32): fwd <= 0.009, bwd <= 0.104 (cosine >=
    # 0.9946), param <= 0.114 (cosine >= 0.9935); with the fault: bwd >= 0.74, param >= 0.99
    # (the input gradient is compared with the CPU gradient masked by the producing ReLU where the
    # GPU conv masks it in its dgrad epilogue: host_api_parity.cpp blocks mode)
    bad = [r for r in rows if r[1] > 2e-2 or r[2] > 0.2 or r[3] > 0.2 or r[5] < 0.99 or r[6] < 0.99]
    assert not bad, bad
    assert len(faulty) == len(rows), r.stdout[-2000:]
    blocks = [(g, f) for g, f in zip(rows, faulty) if "block" in g[0]]
    assert blocks
    for good, bad_row in blocks:
        assert bad_row[0] == good[0]
        # the fault drops the mask in every block's first dgrad: input and parameter gradients
        # fall far outside the bounds above
        assert bad_row[2] > 0.4 and bad_row[3] > 0.5 and bad_row[6] < 0.9, (good, bad_row)


def test_cpp_and_python_cpu_gradients_identical(bins, tmp_path):
    """The C++ host API and the Python front end on the CPU backend: the same initial ResNet-18
    weights and batch give bit-identical parameter gradients (both run the native fp32 kernels;
    the check covers the layer order, the gradient layouts and the snapshot / batch hand-off the
    GPU test above relies on)."""
    from dcnn_amd.nn import LossFactory
    from dcnn_amd.nn.sequential import Sequential, load_tensor
    from dcnn_amd.parallel.dp import DataParallel
    (tmp_path / "snap").mkdir()
    out = _lines(_run([bins["host_api_parity"], "grads", "resnet18_tiny_imagenet", "4", "g.bin", "snap/init"],
                      tmp_path, timeout=300))
    with open(tmp_path / "g.bin", "rb") as f:
        gc = [load_tensor(f) for _ in out["params"]]
    m = Sequential.from_file(str(tmp_path / "snap" / "init"))
    m.set_training(True)
    with open(tmp_path / "snap" / "init.x.bin", "rb") as f:
        x = load_tensor(f)
    with open(tmp_path / "snap" / "init.y.bin", "rb") as f:
        y = load_tensor(f).reshape(-1).long()
    dp = DataParallel(m, broadcast=False)
    m.clear_gradients()
    loss, grad, _ = LossFactory.create("softmax_crossentropy").loss_and_grad(dp.forward(x), y)
    assert abs(float(loss) - float(out["loss"][0])) < 1e-5
    dp.backward(grad, prescaled=True)
    gp = m.gradients()
    assert len(gp) == len(gc) > 40
    for k, (a, b) in enumerate(zip(gp, gc)):
        assert torch.equal(a.detach().reshape(b.shape), b), k


@pytest.mark.gpu
def test_cpp_train_graph_replay_matches_eager(bins, tmp_path):
    """dcnn::TrainGraph (gpu::Graph capture of the whole C++ training step on the thread's flow,
    graph-owned allocations, device-resident Adam scalars, deferred loss readback): the replayed
    steps give bit-identical losses and trained weights to the eager steps (deterministic kernels),
    and the warm-up steps of the capture do not train."""
    args = ["train", "resnet18_tiny_imagenet", "4", "8"]
    e = _lines(_run([bins["host_api_parity"], *args, "snap/e", "--device", "GPU"], tmp_path, timeout=300))
    g = _lines(_run([bins["host_api_parity"], *args, "snap/g", "--device", "GPU", "--graph"], tmp_path, timeout=300))
    assert e["losses"] == g["losses"], (e["losses"], g["losses"])
    assert (tmp_path / "snap" / "e.bin").read_bytes() == (tmp_path / "snap" / "g.bin").read_bytes()


@pytest.mark.gpu
def test_cpp_tiny_imagenet_trainer_graph_bench(bins, tmp_path):
    out = _run([bins["tiny_imagenet_resnet18"], "--device", "GPU", "--batch", "64", "--steps", "10", "--bench"],
               tmp_path, timeout=300)
    assert '"hipgraph": true' in out and re.search(r"\"value\": (\S+),", out), out
    print(out)


@pytest.mark.gpu
def test_cpp_data_parallel_world1_matches_single(bins, tmp_path):
    """C++ data parallelism (dcnn/dist.hpp: rendezvous, in-tree RCCL communicator, the gradient
    all-reduce inside the captured step) at world size 1: the RCCL mean over one rank is the
    gradient itself, so the captured step trains exactly like the single-process one."""
    import json
    import socket
    with socket.socket() as s_:
        s_.bind(("127.0.0.1", 0))
        port = s_.getsockname()[1]
    cmd = [bins["tiny_imagenet_resnet18"], "--device", "GPU", "--batch", "64", "--steps", "6", "--bench"]
    plain = json.loads([l for l in _run(cmd, tmp_path, timeout=300).splitlines() if l.startswith("{")][-1])
    env = dict(os.environ, RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    r = subprocess.run(cmd + ["--dp"], cwd=tmp_path, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                       timeout=300, env=env)
    assert r.returncode == 0, r.stdout[-3000:]
    dp = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert dp["world"] == 1 and dp["data_parallel"] == "rccl" and dp["hipgraph"] is True
    assert dp["loss"] == plain["loss"], (dp, plain)
    # the overlapped bucketed mean (buckets forked from the backward's layer hook onto the
    # communicator's flow inside the capture; 1 MB buckets: several) and the one-shot mean
    for extra, check in (({"DCNN_DP_BUCKET_MB": "1"}, lambda d: d["dp_buckets"] > 3),
                         ({"DCNN_DP_OVERLAP": "0"}, lambda d: d["dp_buckets"] == 0)):
        r = subprocess.run(cmd + ["--dp"], cwd=tmp_path, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                           timeout=300, env=dict(env, **extra))
        assert r.returncode == 0, r.stdout[-3000:]
        d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
        assert check(d) and d["loss"] == plain["loss"], (extra, d, plain)
    print(plain, dp)


@pytest.mark.gpu
def test_bench_default_engine_contract_line(bins, tmp_path):
    """`python bench.py` on one GPU runs the C++ engine (--engine auto) and prints the contract's
    single JSON line with the whole-job value, the timed step count and the engine named."""
    import json
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--batch", "64", "--steps", "4", "--warmup", "2"],
                       cwd=tmp_path, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 4 and d["warmup"] == 2 and d["dtype"] == "bf16"
    assert d["config"]["engine"] == "native (C++ host API)" and d["config"]["global_batch"] == 64
    assert abs(d["value"] - 64 * 1000.0 / d["ms_per_step"]) < 0.02 * d["value"]
