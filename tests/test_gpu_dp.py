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


def _rccl_worker(rank, port, out, with_pg, use_graph, whole=True):
    """World size 1 over the real RCCL backend: graph capture/replay must coexist with the
    process group's watchdog; the bucket all-reduces are captured inside the step graph
    (``whole``) or run between segment replays (DCNN_DP_CAPTURE=0)."""
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), DCNN_DP_CAPTURE="1" if whole else "0",
                      DCNN_DP_FORCE_COLLECTIVES="1")  # world 1 skips the identity all-reduce otherwise
    torch.cuda.set_device(0)
    if with_pg:
        os.environ.setdefault("TORCH_NCCL_CUDA_EVENT_CACHE", "0")  # (as dcnn_amd/__init__.py)
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    from dcnn_amd.models import zoo
    from dcnn_amd.nn import Adam, LossFactory
    from dcnn_amd.parallel.dp import DataParallel
    from dcnn_amd.runtime.step import TrainStep
    m = zoo.create_model("resnet18_tiny_imagenet")
    m.set_seed(5)
    m.set_device("GPU:0")
    # fp32 compute (the kernels are deterministic: eager and graph steps run the same kernels in
    # the same order, so every variant must agree bit for bit)
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
    torch.save({"g": grad, "losses": losses, "segs": len(getattr(st, "_segs", [])) if use_graph else 0,
                "whole": st._whole, "big": [(o, torch.Size(sh).numel()) for o, sh in big]},
               os.path.join(out, f"pg{int(with_pg)}g{int(use_graph)}w{int(whole)}.pt"))
    if with_pg:
        dist.destroy_process_group()


def test_gpu_dp_rccl_world1_graph_segments(tmp_path):
    """RCCL group, collectives captured in the step graph == segmented graph step == graph step
    without a group (in-tree RCCL communicator, captured) == eager step, bit for bit (deterministic kernels; an all-reduce over one rank
    is exact); the graph warm-up must not train (first-step losses equal eager)."""
    for with_pg, use_graph, whole in ((True, True, True), (True, True, False), (False, True, True),
                                      (False, False, True)):
        mp.spawn(_rccl_worker, args=(_port(), str(tmp_path), with_pg, use_graph, whole), nprocs=1, join=True)
    w = torch.load(tmp_path / "pg1g1w1.pt", weights_only=True)
    a = torch.load(tmp_path / "pg1g1w0.pt", weights_only=True)
    b = torch.load(tmp_path / "pg0g1w1.pt", weights_only=True)
    e = torch.load(tmp_path / "pg0g0w1.pt", weights_only=True)
    assert w["whole"] and not a["whole"]
    # without a process group the in-tree RCCL plane carries the bucket all-reduces: captured too
    assert a["segs"] > 1 and b["whole"]
    assert w["losses"] == a["losses"] == b["losses"], (w["losses"], a["losses"], b["losses"])
    assert torch.equal(w["g"], a["g"]) and torch.equal(w["g"], b["g"])
    for r in (w, a, b):
        assert torch.equal(r["g"], e["g"]), (r["g"] - e["g"]).abs().max()
        assert r["losses"] == e["losses"], (r["losses"], e["losses"])


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


def test_gpu_bf16_grad_wire_kernels():
    """comm.hip: pack (fp32 -> bf16), fixed-order fp32 sum of the rank chunks, unpack."""
    from dcnn_amd.ops._ext import kernels, stream_ptr
    K = kernels()
    w, n, shard = 4, 1000, 1024
    g = torch.randn(n, device="cuda")
    packed = torch.zeros(shard, dtype=torch.bfloat16, device="cuda")
    K.grad_pack_bf16(g.data_ptr(), packed.data_ptr(), n, 1.0, stream_ptr())
    assert torch.equal(packed[:n], g.to(torch.bfloat16))
    src = torch.randn(w, shard, device="cuda").to(torch.bfloat16)
    red = torch.empty(shard - 3, dtype=torch.bfloat16, device="cuda")
    K.grad_sum_chunks_bf16(src.data_ptr(), w, shard, shard - 3, red.data_ptr(), stream_ptr())
    ref = src.float()[0].clone()
    for r in range(1, w):
        ref += src.float()[r]
    assert torch.equal(red, ref[:shard - 3].to(torch.bfloat16))
    out = torch.empty(n, device="cuda")
    K.grad_unpack_bf16(packed.data_ptr(), out.data_ptr(), n, stream_ptr())
    assert torch.equal(out, packed[:n].float())


def _wire_worker(rank, port, out, backend, grad_dtype):
    """World 1, forced collectives, whole-step graph capture: the bucket pipeline of
    ``grad_dtype`` (fp32 all-reduce, or bf16 pack -> reduce-scatter -> all-gather -> unpack) runs
    on the comm stream inside the captured step."""
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), DCNN_DP_FORCE_COLLECTIVES="1",
                      RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    torch.cuda.set_device(0)
    if backend == "torch":
        os.environ.setdefault("TORCH_NCCL_CUDA_EVENT_CACHE", "0")  # (as dcnn_amd/__init__.py)
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    from dcnn_amd.models import zoo
    from dcnn_amd.nn import SGD, LossFactory
    from dcnn_amd.parallel.dp import DataParallel
    from dcnn_amd.runtime.step import TrainStep
    m = zoo.create_model("resnet18_tiny_imagenet")
    m.set_seed(5)
    m.set_device("GPU:0")
    m.initialize()
    m.set_first_layer_input_grad(False)
    dp = DataParallel(m, bucket_mb=4.0, grad_dtype=grad_dtype, comm_backend=backend)
    assert dp.active and (dp.rccl is not None) == (backend == "rccl")
    opt = SGD(0.0)  # lr 0: every step sees the same weights, so the gradients stay comparable
    opt.attach(m)
    st = TrainStep(dp, LossFactory.create("softmax_crossentropy"), opt, use_graph=True)
    g = torch.Generator().manual_seed(11)
    x = torch.randn(32, 3, 64, 64, generator=g).cuda()
    y = torch.randint(0, 200, (32,), generator=g).cuda()
    losses = [float(st(x, y)) for _ in range(3)]
    torch.cuda.synchronize()
    torch.save({"g": m.arena.grad.cpu(), "losses": losses, "whole": st._whole},
               os.path.join(out, f"{backend}_{grad_dtype}.pt"))
    if dp.rccl is not None:
        dp.rccl.close()
    if dist.is_initialized():
        dist.destroy_process_group()


@pytest.mark.parametrize("backend", ["rccl", "torch"])
def test_gpu_dp_bf16_wire_captured_world1(tmp_path, backend):
    """The bf16 gradient wire in the captured step (whole graph on the in-tree plane, segmented
    on ProcessGroupNCCL): at world 1 the reduce-scatter / all-gather are identities, so the
    step's gradient must be the fp32 step's rounded to bf16."""
    for gd in ("fp32", "bf16"):
        mp.spawn(_wire_worker, args=(_port(), str(tmp_path), backend, gd), nprocs=1, join=True)
    a = torch.load(tmp_path / f"{backend}_fp32.pt", weights_only=True)
    b = torch.load(tmp_path / f"{backend}_bf16.pt", weights_only=True)
    # (ProcessGroupNCCL's bf16 pair runs between segment replays: runtime/step.py)
    assert a["whole"] and b["whole"] == (backend == "rccl")
    assert a["losses"] == b["losses"]
    assert torch.equal(b["g"], a["g"].bfloat16().float())
