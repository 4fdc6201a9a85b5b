"""Data parallel on the GPU with the hipGraph-segmented train step: two ranks share cuda:0 (the
one-GPU box) over gloo, so the segment-replay + bucket all-reduce path of runtime/step.py runs
with world_size 2.  Every bucket must be reduced: the replicas see different data, so a missed
bucket would make their parameters diverge."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, port, out, use_graph):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=2)
    from dcnn_amd.models import zoo
    from dcnn_amd.nn import Adam, LossFactory
    from dcnn_amd.parallel.dp import DataParallel
    from dcnn_amd.runtime.step import TrainStep
    m = zoo.create_model("resnet18_tiny_imagenet")
    m.set_seed(1 + rank)
    m.set_device("GPU:0")
    m.initialize()
    m.set_first_layer_input_grad(False)
    dp = DataParallel(m, bucket_mb=8.0)
    opt = Adam(1e-3)
    opt.attach(m)
    st = TrainStep(dp, LossFactory.create("softmax_crossentropy"), opt, use_graph=use_graph)
    g = torch.Generator().manual_seed(10 + rank)
    x = torch.randn(32, 3, 64, 64, generator=g).cuda()
    y = torch.randint(0, 200, (32,), generator=g).cuda()
    losses = [float(st(x, y)) for _ in range(6)]
    torch.cuda.synchronize()
    torch.save({"p": m.arena.data.cpu(), "losses": losses, "buckets": len(dp.buckets)}, os.path.join(out, f"{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("use_graph", [True, False])
def test_gpu_dp_two_ranks_shared_gpu(tmp_path, use_graph):
    mp.spawn(_worker, args=(_port(), str(tmp_path), use_graph), nprocs=2, join=True)
    r0 = torch.load(tmp_path / "0.pt", weights_only=True)
    r1 = torch.load(tmp_path / "1.pt", weights_only=True)
    assert r0["buckets"] > 1
    assert torch.equal(r0["p"], r1["p"]), (r0["p"] - r1["p"]).abs().max()
    assert r0["losses"][-1] < r0["losses"][0]


def _rccl_worker(rank, port, out, with_pg, use_graph):
    """World size 1 over the real RCCL backend: graph capture/replay must coexist with the
    process group's watchdog, and the bucket all-reduces run between segment replays."""
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    if with_pg:
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    from dcnn_amd.models import zoo
    from dcnn_amd.nn import Adam, LossFactory
    from dcnn_amd.parallel.dp import DataParallel
    from dcnn_amd.runtime.step import TrainStep
    m = zoo.create_model("resnet18_tiny_imagenet")
    m.set_seed(5)
    m.set_device("GPU:0")
    # fp32 compute: run-to-run noise of the statistics atomics is ~1e-3 of a first-step weight
    # gradient there (bf16 roundings amplify it to ~20% at random init)
    m.set_compute_dtype(torch.float32)
    m.initialize()
    m.set_first_layer_input_grad(False)
    dp = DataParallel(m, bucket_mb=4.0)
    opt = Adam(1e-3)
    opt.attach(m)
    st = TrainStep(dp, LossFactory.create("softmax_crossentropy"), opt, use_graph=use_graph)
    g = torch.Generator().manual_seed(11)
    x = torch.randn(32, 3, 64, 64, generator=g).cuda()
    y = torch.randint(0, 200, (32,), generator=g).cuda()
    losses = [float(st(x, y))]
    grad = m.arena.grad.cpu()  # gradients of the first step (left in the arena after the update)
    losses += [float(st(x, y)) for _ in range(3)]
    torch.cuda.synchronize()
    big = [(o, s.shape) for o, s in zip(m.arena.offsets, m.arena.specs) if torch.Size(s.shape).numel() >= 4096]
    torch.save({"g": grad, "losses": losses, "segs": len(st._segs) if use_graph else 0,
                "big": [(o, torch.Size(sh).numel()) for o, sh in big]},
               os.path.join(out, f"pg{int(with_pg)}g{int(use_graph)}.pt"))
    if with_pg:
        dist.destroy_process_group()


def test_gpu_dp_rccl_world1_graph_segments(tmp_path):
    """Segmented-graph step with an RCCL group == unsegmented graph step == eager step; the
    graph warm-up must not train (first-step losses agree with eager)."""
    for with_pg, use_graph in ((True, True), (False, True), (False, False)):
        mp.spawn(_rccl_worker, args=(_port(), str(tmp_path), with_pg, use_graph), nprocs=1, join=True)
    a = torch.load(tmp_path / "pg1g1.pt", weights_only=True)
    b = torch.load(tmp_path / "pg0g1.pt", weights_only=True)
    e = torch.load(tmp_path / "pg0g0.pt", weights_only=True)
    assert a["segs"] > 1 and b["segs"] == 1
    for r in (a, b):
        # weight gradients (biases ahead of a BatchNorm have ~zero true gradient: skipped)
        for o, n in e["big"]:
            ge, gr = e["g"][o:o + n], r["g"][o:o + n]
            assert (ge - gr).norm() <= 3e-2 * ge.norm(), (o, n, (ge - gr).norm(), ge.norm())
        assert abs(r["losses"][0] - e["losses"][0]) < 1e-5 * abs(e["losses"][0]), (r["losses"], e["losses"])
        for lr_, le in zip(r["losses"], e["losses"]):
            assert abs(lr_ - le) < 3e-2 * max(1.0, abs(le)), (r["losses"], e["losses"])


def _bnfree_model(seed):
    from dcnn_amd.nn import SequentialBuilder
    m = (SequentialBuilder("dp_exact").input([3, 16, 16])
         .conv2d(16, 3, 3, 1, 1, 1, 1).activation("relu").maxpool2d(2, 2, 2, 2)
         .conv2d(32, 3, 3, 1, 1, 1, 1).activation("relu").flatten().dense(10).build())
    m.set_seed(seed)
    m.set_device("GPU:0")
    m.set_compute_dtype(torch.float32)
    m.initialize()
    m.set_first_layer_input_grad(False)
    return m


def _exact_worker(rank, world, port, out, use_graph):
    """fp32 + SGD, BN-free: each rank trains its half of the batch; after the bucket all-reduce
    the gradient and the updated parameters must equal a single process on the whole batch."""
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    from dcnn_amd.nn import SGD, LossFactory
    from dcnn_amd.parallel.dp import DataParallel
    from dcnn_amd.runtime.step import TrainStep
    m = _bnfree_model(3)
    dp = DataParallel(m, bucket_mb=0.004)  # ~1 KB buckets: several fire points inside backward
    opt = SGD(0.1)
    opt.attach(m)
    st = TrainStep(dp, LossFactory.create("softmax_crossentropy"), opt, use_graph=use_graph)
    g = torch.Generator().manual_seed(21)
    x = torch.randn(16, 3, 16, 16, generator=g)
    y = torch.randint(0, 10, (16,), generator=g)
    per = 16 // world
    xs, ys = x[rank * per:(rank + 1) * per].cuda(), y[rank * per:(rank + 1) * per].cuda()
    p0 = m.arena.data.cpu().clone()
    st(xs, ys)
    torch.cuda.synchronize()
    torch.save({"g": m.arena.grad.cpu(), "p": m.arena.data.cpu(), "p0": p0, "buckets": len(dp.buckets)},
               os.path.join(out, f"w{world}r{rank}g{int(use_graph)}.pt"))
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


@pytest.mark.parametrize("use_graph", [False, True])
def test_gpu_dp_two_ranks_equal_single_process(tmp_path, use_graph):
    mp.spawn(_exact_worker, args=(2, _port(), str(tmp_path), use_graph), nprocs=2, join=True)
    mp.spawn(_exact_worker, args=(1, _port(), str(tmp_path), use_graph), nprocs=1, join=True)
    r0 = torch.load(tmp_path / f"w2r0g{int(use_graph)}.pt", weights_only=True)
    r1 = torch.load(tmp_path / f"w2r1g{int(use_graph)}.pt", weights_only=True)
    ref = torch.load(tmp_path / f"w1r0g{int(use_graph)}.pt", weights_only=True)
    assert r0["buckets"] > 2
    assert torch.equal(r0["p0"], ref["p0"])
    assert torch.equal(r0["g"], r1["g"]) and torch.equal(r0["p"], r1["p"])
    # averaged half-batch gradients == whole-batch gradient (fp32; summation order differs)
    torch.testing.assert_close(r0["g"], ref["g"], rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(r0["p"], ref["p"], rtol=1e-5, atol=1e-6)
