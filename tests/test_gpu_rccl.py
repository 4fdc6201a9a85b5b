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
    os.environ.setdefault("TORCH_NCCL_CUDA_EVENT_CACHE", "0")  # (as dcnn_amd/__init__.py)
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


def _worker_no_c10d(rank, port, out):
    """The bench configuration: no torch.distributed at all; rank / world from the environment,
    the in-tree communicator bootstraps itself (world 1 here: forced collectives on the comm
    stream, captured in the step graph)."""
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), DCNN_DP_FORCE_COLLECTIVES="1",
                      RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    torch.cuda.set_device(0)
    from dcnn_amd.models import zoo
    from dcnn_amd.nn import Adam, LossFactory
    from dcnn_amd.parallel.dp import DataParallel
    from dcnn_amd.runtime.step import TrainStep
    m = zoo.create_model("resnet18_tiny_imagenet")
    m.set_seed(5)
    m.set_device("GPU:0")
    m.initialize()
    m.set_first_layer_input_grad(False)
    dp = DataParallel(m, bucket_mb=4.0)  # default plane without c10d: in-tree RCCL
    assert not dist.is_initialized() and dp.comm_backend == "rccl" and dp.rccl is not None and dp.active
    opt = Adam(1e-3)
    opt.attach(m)
    st = TrainStep(dp, LossFactory.create("softmax_crossentropy"), opt, use_graph=True)
    g = torch.Generator().manual_seed(11)
    x = torch.randn(32, 3, 64, 64, generator=g).cuda()
    y = torch.randint(0, 200, (32,), generator=g).cuda()
    losses = [float(st(x, y)) for _ in range(4)]
    dp.barrier()
    assert dp.max_over_ranks(3.5) == 3.5
    torch.cuda.synchronize()
    torch.save({"p": m.arena.data.cpu(), "g": m.arena.grad.cpu(), "losses": losses, "whole": st._whole},
               os.path.join(out, "noc10d.pt"))
    dp.rccl.close()


def test_rccl_dp_without_c10d_matches_process_group_nccl(tmp_path):
    """Comm-stream bucket all-reduces (forked / joined inside the captured step graph) with no
    torch.distributed group == the ProcessGroupNCCL step, bit for bit."""
    mp.spawn(_worker, args=(_port(), str(tmp_path), "torch"), nprocs=1, join=True)
    mp.spawn(_worker_no_c10d, args=(_port(), str(tmp_path)), nprocs=1, join=True)
    a = torch.load(tmp_path / "torch.pt", weights_only=True)
    b = torch.load(tmp_path / "noc10d.pt", weights_only=True)
    assert a["whole"] and b["whole"]
    assert a["losses"] == b["losses"]
    assert torch.equal(a["g"], b["g"]) and torch.equal(a["p"], b["p"])


def test_rccl_p2p_directions_on_own_streams():
    """RcclP2P (pipeline plane): one communicator + stream per direction. At world 1 a grouped
    self send/recv per direction moves the data; forward and backward traffic interleaved (as in
    1F1B) on their own streams, consumed on the compute stream."""
    from dcnn_amd.ops._ext import kernels
    from dcnn_amd.parallel.rccl import RcclP2P
    p2p = RcclP2P(0, 1, torch.device("cuda", 0))
    K = kernels()
    assert set(p2p.comms) == {"fwd", "bwd", "cfwd", "cbwd"}
    assert len({id(s) for s in p2p.streams.values()}) == 4
    acts = [torch.randn(8, 64, 16, 16, device="cuda").bfloat16() for _ in range(3)]
    grads = [torch.randn(8, 64, 16, 16, device="cuda").bfloat16() for _ in range(3)]
    ra = [torch.empty_like(t) for t in acts]
    rg = [torch.empty_like(t) for t in grads]

    def exchange():
        for k in range(3):
            for key, src, dst in (("fwd", acts[k], ra[k]), ("bwd", grads[k], rg[k])):
                # self send + recv must be grouped (one rank): enqueue both on the direction stream
                s = p2p.streams[key]
                s.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(s):
                    K.rccl.group_start()
                    p2p.comms[key].send(src, 0)
                    p2p.comms[key].recv(dst, 0)
                    K.rccl.group_end()
                torch.cuda.current_stream().wait_stream(s)
            ra[k].mul_(2)
            rg[k].add_(1)

    exchange()
    torch.cuda.synchronize()
    for k in range(3):
        assert torch.equal(ra[k], acts[k] * 2) and torch.equal(rg[k], grads[k] + 1)
    p2p.barrier()
    p2p.close()
