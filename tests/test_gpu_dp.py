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
