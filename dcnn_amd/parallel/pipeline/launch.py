"""One-process-per-GPU pipeline launcher (torchrun entry point).

    python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \\
        --master-port 29500 -m dcnn_amd.parallel.pipeline.launch --model resnet50_tiny_imagenet \\
        --batch 256 --microbatches 8 --schedule semi_async --steps 20

Rank r hosts stage r on GPU r (pipeline neighbours are direct xGMI peers); rank 0 also runs
the coordinator (loss, micro-batch schedule) on its main thread while its stage runs on a
worker thread.  The control plane is the native TCP communicator on 127.0.0.1
(``--base-port`` + rank); activations and gradients move GPU-to-GPU over RCCL
(``transport="p2p"``) or inline through TCP (``--transport message``).  On GPUs the P2P plane is
torch.distributed isend/irecv on four process groups (``--p2p torch``, default) or the
framework's own (``--p2p rccl``: parallel/rccl.py ``RcclP2P``, one communicator and one HIP
stream per direction, bootstrapped over the native TCP plane — no torch.distributed; opt-in
until a multi-GPU run of it is on record). On the CPU the same code runs over gloo. Schedules: ``sync`` (GPipe), ``semi_async``, ``1f1b``.
"""
from __future__ import annotations

import argparse
import json
import os
import time

import torch
import torch.distributed as dist


def run(argv=None) -> dict:
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet50_tiny_imagenet")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--microbatches", type=int, default=8)
    ap.add_argument("--schedule", default="semi_async", choices=["semi_async", "sync", "1f1b"])
    ap.add_argument("--p2p", default=os.environ.get("DCNN_P2P_BACKEND", "torch"), choices=["rccl", "torch"],
                    help="GPU data plane: torch.distributed groups (default) or the in-tree RCCL plane (no c10d)")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--transport", default="p2p", choices=["p2p", "message"])
    ap.add_argument("--partitioner", default="flops", choices=["flops", "naive"])
    ap.add_argument("--base-port", type=int, default=int(os.environ.get("DCNN_PIPE_PORT", "29650")))
    ap.add_argument("--lr", type=float, default=1e-3)
    ap.add_argument("--cpu", action="store_true")
    ap.add_argument("--seed", type=int, default=1234)
    a = ap.parse_args(argv)

    from ...models import zoo
    from ...nn.optimizers import Adam
    from .config import Endpoint
    from .coordinator import DistributedCoordinator
    from .partitioner import create_partitioner
    from .transport import make_groups
    from .worker import NetworkStageWorker

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    use_gpu = torch.cuda.is_available() and not a.cpu
    in_tree = use_gpu and a.p2p == "rccl"
    if in_tree:
        from ..rccl import RcclP2P
        torch.cuda.set_device(local)
        groups = RcclP2P(rank, world, torch.device("cuda", local))
        barrier = groups.barrier
    else:
        if use_gpu:
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")
        groups = make_groups()
        barrier = dist.barrier
    worker = NetworkStageWorker(a.base_port + rank, host="127.0.0.1", p2p_groups=groups, verbose=True)
    barrier()  # every stage listens before the coordinator dials
    result = {}
    if rank == 0:
        worker.start_thread()
        in_shape = zoo.INPUT_SHAPES[a.model]
        model = zoo.create_model(a.model)
        devs = [f"GPU:{r}" if use_gpu else "CPU" for r in range(world)]
        coord = DistributedCoordinator(
            model, Adam(a.lr), "softmax_crossentropy",
            [Endpoint.network("127.0.0.1", a.base_port + r) for r in range(world)],
            num_microbatches=a.microbatches, host="127.0.0.1", port=a.base_port + world,
            stage_ranks=list(range(world)), coordinator_rank=0, p2p_groups=groups,
            partitioner=create_partitioner(a.partitioner, [a.batch // a.microbatches] + list(in_shape)),
            device=devs[0], stage_devices=devs, transport=a.transport, seed=a.seed)
        coord.initialize()
        coord.deploy_stages()
        coord.start()
        dev = torch.device("cuda", local) if use_gpu else torch.device("cpu")
        g = torch.Generator().manual_seed(a.seed)
        ncls = zoo.NUM_CLASSES[a.model]
        x = torch.randn([a.batch] + list(in_shape), generator=g).to(dev)
        y = torch.randint(0, ncls, (a.batch,), generator=g).to(dev)
        if use_gpu:
            x = x.bfloat16().contiguous(memory_format=torch.channels_last)
        for _ in range(a.warmup):
            coord.train_step(x, y, a.schedule)
        coord.barrier()
        t0 = time.perf_counter()
        loss = 0.0
        for _ in range(a.steps):
            loss = coord.train_step(x, y, a.schedule)
        coord.barrier()
        dt = time.perf_counter() - t0
        result = {"metric": f"pipeline images/sec {a.model}", "value": round(a.batch * a.steps / dt, 1),
                  "unit": "images/sec", "stages": world, "microbatches": a.microbatches,
                  "schedule": a.schedule, "transport": a.transport, "p2p": "rccl" if in_tree else "torch", "ms_per_step": round(dt / a.steps * 1e3, 3),
                  "partitions": [(p.start_layer, p.end_layer) for p in coord.partitions], "loss": round(loss, 4)}
        print(json.dumps(result), flush=True)
        coord.stop()
        worker.stage.thread.join(timeout=60)
        worker.comm.close()
    else:
        worker.run()
    # receive buffers ever allocated by this rank's P2P data plane (persistent per-(peer, command,
    # micro-batch) slots: a fixed number however many steps ran)
    allocs = sum(getattr(getattr(o, "transport", None), "slot_allocs", 0)
                 for o in ([coord] if rank == 0 else []) + [getattr(worker, "stage", None)])
    print(json.dumps({"rank": rank, "slot_allocs": allocs, "steps": a.warmup + a.steps}), flush=True)
    barrier()
    if in_tree:
        groups.close()
    else:
        dist.destroy_process_group()
    return result


if __name__ == "__main__":
    run()
