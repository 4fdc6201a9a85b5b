"""Data parallelism over torch.distributed (gloo on CPU, world_size 2): bucketed all-reduce fired
from inside backward must equal single-process micro-batched training, replicas must stay
bit-identical, and bench.py must run under torchrun."""
import json
import os
import socket
import subprocess
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_dir, bucket_mb):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from dcnn_amd.models import zoo
    from dcnn_amd.nn import SGD, LossFactory
    from dcnn_amd.parallel.dp import DataParallel
    from dcnn_amd.runtime.step import TrainStep
    model = zoo.create_model("resnet9_cifar10")
    model.set_seed(100 + rank)          # different init per rank: broadcast must unify it
    model.initialize()
    dp = DataParallel(model, bucket_mb=bucket_mb)
    opt = SGD(0.05, 0.9)
    opt.attach(model)
    step = TrainStep(dp, LossFactory.create("softmax_crossentropy"), opt)
    g = torch.Generator().manual_seed(7)
    x = torch.randn(8, 3, 32, 32, generator=g)
    y = torch.randint(0, 10, (8,), generator=g)
    step(x[rank * 4:(rank + 1) * 4], y[rank * 4:(rank + 1) * 4])
    one = [p.detach().clone() for p in model.parameters()]
    step(x[rank * 4:(rank + 1) * 4], y[rank * 4:(rank + 1) * 4])
    torch.save({"params": [p.detach().clone() for p in model.parameters()], "one": one, "nbuckets": len(dp.buckets)},
               os.path.join(out_dir, f"rank{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("bucket_mb", [0.5, 64.0])
def test_dp_matches_single_process(tmp_path, bucket_mb):
    mp.spawn(_worker, args=(2, _free_port(), str(tmp_path), bucket_mb), nprocs=2, join=True)
    r0 = torch.load(tmp_path / "rank0.pt", weights_only=True)
    r1 = torch.load(tmp_path / "rank1.pt", weights_only=True)
    if bucket_mb < 1:
        assert r0["nbuckets"] > 1
    for a, b in zip(r0["params"], r1["params"]):
        assert torch.equal(a, b)  # replicas identical
    # single-process reference: rank 0's init, two half-batches with gradient 1/2 each
    from dcnn_amd.models import zoo
    from dcnn_amd.nn import SGD, LossFactory
    ref = zoo.create_model("resnet9_cifar10")
    ref.set_seed(100)
    ref.initialize()
    opt = SGD(0.05, 0.9)
    opt.attach(ref)
    lf = LossFactory.create("softmax_crossentropy")
    g = torch.Generator().manual_seed(7)
    x = torch.randn(8, 3, 32, 32, generator=g)
    y = torch.randint(0, 10, (8,), generator=g)
    opt.clear_gradients()
    for r in range(2):
        out = ref.forward(x[r * 4:(r + 1) * 4], r)
        _, grad, _ = lf.loss_and_grad(out, y[r * 4:(r + 1) * 4])
        ref.backward(grad * 0.5, r)
    opt.update()
    # one step: equal up to summation-order rounding (later steps diverge chaotically through
    # ReLU / max-pool argmax flips, so they are only checked for replica agreement above)
    for a, b in zip(r0["one"], ref.parameters()):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-7)


def test_bench_under_torchrun_cpu():
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--batch", "4", "--device", "cpu", "--graph", "0", "--model", "mnist_cnn"]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=600,
                       env=dict(os.environ, OMP_NUM_THREADS="1"))
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    d = lines[0]
    assert d["n_gpus"] == 2 and d["config"]["global_batch"] == 8 and d["value"] > 0
    assert d["config"]["parallelism"] == "dp2"


def _bf16_worker(rank, world, port, out_dir, grad_dtype):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from dcnn_amd.models import zoo
    from dcnn_amd.nn import SGD, LossFactory
    from dcnn_amd.parallel.dp import DataParallel
    model = zoo.create_model("mnist_cnn")
    model.set_seed(5)
    model.initialize()
    dp = DataParallel(model, bucket_mb=0.05, grad_dtype=grad_dtype)
    lf = LossFactory.create("softmax_crossentropy")
    g = torch.Generator().manual_seed(3 + rank)
    x = torch.randn(8, 1, 28, 28, generator=g)
    y = torch.randint(0, 10, (8,), generator=g)
    model.clear_gradients()
    out = dp.forward(x)
    _, grad, _ = lf.loss_and_grad(out, y)
    dp.backward(grad)
    torch.save({"g": model.arena.grad.clone(), "nb": len(dp.buckets)}, os.path.join(out_dir, f"{grad_dtype}{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def test_dp_bf16_gradient_allreduce_matches_fp32(tmp_path):
    """bf16 wire format (all_to_all shards, fp32 rank-order sum, all_gather): every rank ends
    with the same gradient, equal to the fp32 all-reduce up to one bf16 rounding of the sum
    (plus the bf16 rounding of each rank's contribution)."""
    for dt in ("fp32", "bf16"):
        mp.spawn(_bf16_worker, args=(3, _free_port(), str(tmp_path), dt), nprocs=3, join=True)
    f = [torch.load(tmp_path / f"fp32{r}.pt", weights_only=True)["g"] for r in range(3)]
    b = [torch.load(tmp_path / f"bf16{r}.pt", weights_only=True) for r in range(3)]
    assert b[0]["nb"] > 1
    for r in range(1, 3):
        assert torch.equal(b[0]["g"], b[r]["g"])
    ref = f[0]
    err = (b[0]["g"] - ref).abs()
    assert float(err.max()) <= 2 * 2 ** -8 * float(ref.abs().max()) + 1e-12
    assert float((b[0]["g"] - ref).norm()) <= 2 ** -7 * float(ref.norm())
