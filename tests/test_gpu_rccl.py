"""In-tree RCCL communicator (csrc/kernels/rccl.cpp, parallel/rccl.py) on the GPU. One GPU per
box, so world size 1: the collectives are identities, but they run RCCL's kernels on the
compute stream, inside captured hipGraphs, and the DP step through them must equal the
ProcessGroupNCCL step bit for bit."""
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


def test_rccl_comm_world1_collectives_in_graph():
    from dcnn_amd.parallel.rccl import RcclCommunicator
    comm = RcclCommunicator(0, 1, torch.device("cuda", 0))
    x = torch.randn(1 << 16, device="cuda")
    ref = x.clone()
    comm.all_reduce(x)
    comm.broadcast(x, 0)
    torch.cuda.synchronize()
    assert torch.equal(x, ref)
    out = torch.empty_like(x)
    comm.all_gather(out, x)
    rs = torch.empty_like(x)
    comm.reduce_scatter(rs, x)
    torch.cuda.synchronize()
    assert torch.equal(out, ref) and torch.equal(rs, ref)
    # captured: a graph of (scale, all-reduce, scale) replays correctly
    y = torch.randn(4096, device="cuda")
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            y.mul_(2.0)
            comm.all_reduce(y)
            y.add_(1.0)
    torch.cuda.current_stream().wait_stream(s)
    y0 = y.clone()
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(y, y0 * 2 + 1)
    comm.close()


def _worker(rank, port, out, backend):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), DCNN_DP_FORCE_COLLECTIVES="1")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    from dcnn_amd.models import zoo
    from dcnn_amd.nn import Adam, LossFactory
    from dcnn_amd.parallel.dp import DataParallel
    from dcnn_amd.runtime.step import TrainStep
    m = zoo.create_model("resnet18_tiny_imagenet")
    m.set_seed(5)
    m.set_device("GPU:0")
    m.initialize()
    m.set_first_layer_input_grad(False)
    dp = DataParallel(m, bucket_mb=4.0, comm_backend=backend)
    assert (dp.rccl is not None) == (backend == "rccl")
    opt = Adam(1e-3)
    opt.attach(m)
    st = TrainStep(dp, LossFactory.create("softmax_crossentropy"), opt, use_graph=True)
    g = torch.Generator().manual_seed(11)
    x = torch.randn(32, 3, 64, 64, generator=g).cuda()
    y = torch.randint(0, 200, (32,), generator=g).cuda()
    losses = [float(st(x, y)) for _ in range(4)]
    torch.cuda.synchronize()
    torch.save({"p": m.arena.data.cpu(), "g": m.arena.grad.cpu(), "losses": losses, "whole": st._whole},
               os.path.join(out, f"{backend}.pt"))
    if dp.rccl is not None:
        dp.rccl.close()
    dist.destroy_process_group()


def test_rccl_dp_step_matches_process_group_nccl(tmp_path):
    """Whole-step graph with the bucket all-reduces on the in-tree communicator == the same step
    with ProcessGroupNCCL collectives: losses, gradients and parameters bit-identical."""
    for backend in ("torch", "rccl"):
        mp.spawn(_worker, args=(_port(), str(tmp_path), backend), nprocs=1, join=True)
    a = torch.load(tmp_path / "torch.pt", weights_only=True)
    b = torch.load(tmp_path / "rccl.pt", weights_only=True)
    assert a["whole"] and b["whole"]
    assert a["losses"] == b["losses"]
    assert torch.equal(a["g"], b["g"]) and torch.equal(a["p"], b["p"])
