#!/usr/bin/env python3
"""Pipeline-parallel training throughput (images/sec) with the in-process coordinator.

The BASELINE.json pipeline configs are ResNet-50 Tiny-ImageNet with a 4-stage sync (GPipe-style)
schedule and an 8-stage semi-async schedule (reference include/pipeline/coordinator.hpp:273
``async_process_batch``, examples/sync_pipeline_coordinator.cpp:185-198 for the per-batch
timing it prints).  Stages run on their own threads (reference
include/pipeline/in_process_coordinator.hpp) and are placed round-robin on the visible GPUs:
with one GPU every stage shares cuda:0, so the number measures the schedule, the stage
runtime and the micro-batch kernels, not xGMI hops.  The one-process-per-GPU RCCL path is
``python -m dcnn_amd.parallel.pipeline.launch`` (torchrun).

    python benchmarks/pipeline_bench.py --stages 4 --schedule sync
    python benchmarks/pipeline_bench.py --stages 8 --schedule semi_async

Synthetic 64x64 RGB inputs + random labels, random init, bf16 compute, Adam; every timed step
runs forward, loss, backward and the parameter update on every stage.
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet50_tiny_imagenet")
    ap.add_argument("--stages", type=int, default=4)
    ap.add_argument("--schedule", default="sync", choices=["sync", "semi_async", "1f1b"])
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--microbatches", type=int, default=8)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--partitioner", default="flops", choices=["flops", "naive"])
    ap.add_argument("--cpu", action="store_true")
    ap.add_argument("--no-graph", action="store_true", help="eager stages (no per-micro-batch hipGraphs)")
    ap.add_argument("--profiling", action="store_true", help="per-layer HIP-event timings on eager steps")
    a = ap.parse_args(argv)

    from dcnn_amd.models import zoo
    from dcnn_amd.nn.optimizers import Adam
    from dcnn_amd.parallel.pipeline import InProcessCoordinator
    from dcnn_amd.parallel.pipeline.partitioner import create_partitioner

    use_gpu = torch.cuda.is_available() and not a.cpu
    ngpu = torch.cuda.device_count() if use_gpu else 0
    devs = [f"GPU:{i % ngpu}" if use_gpu else "CPU" for i in range(a.stages)]
    in_shape = list(zoo.INPUT_SHAPES[a.model])
    model = zoo.create_model(a.model)
    coord = InProcessCoordinator(model, Adam(1e-3), "softmax_crossentropy", num_stages=a.stages,
                                 num_microbatches=a.microbatches,
                                 partitioner=create_partitioner(a.partitioner, [a.batch // a.microbatches] + in_shape),
                                 device=devs[0], stage_devices=devs, seed=1234,
                                 use_graph=use_gpu and not a.no_graph, profiling=a.profiling)
    dev = torch.device("cuda", 0) if use_gpu else torch.device("cpu")
    try:
        coord.initialize()
        coord.deploy_stages()
        coord.start()
        g = torch.Generator().manual_seed(7)
        x = torch.randn([a.batch] + in_shape, generator=g).to(dev)
        y = torch.randint(0, zoo.NUM_CLASSES[a.model], (a.batch,), generator=g).to(dev)
        if use_gpu:
            x = x.bfloat16().contiguous(memory_format=torch.channels_last)
        first = None
        for _ in range(a.warmup):
            l = coord.train_step(x, y, a.schedule)
            first = l if first is None else first
        coord.barrier()
        if use_gpu:
            torch.cuda.synchronize()
        t0 = time.perf_counter()
        loss = float("nan")
        for _ in range(a.steps):
            loss = coord.train_step(x, y, a.schedule)
        coord.barrier()
        if use_gpu:
            torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        res = {"metric": f"pipeline images/sec {a.model}", "value": round(a.batch * a.steps / dt, 1),
               "unit": "images/sec", "stages": a.stages, "gpus": max(ngpu, 0), "stage_devices": devs,
               "schedule": a.schedule, "hipgraph": use_gpu and not a.no_graph, "microbatches": a.microbatches, "batch": a.batch,
               "ms_per_step": round(dt / a.steps * 1e3, 3), "steps": a.steps, "warmup": a.warmup,
               "dtype": "bf16" if use_gpu else "fp32", "data": "synthetic", "coordinator": "in_process",
               "partitions": [(p.start_layer, p.end_layer) for p in coord.partitions],
               "first_loss": round(float(first), 4) if first is not None else None, "loss": round(float(loss), 4)}
        print(json.dumps(res), flush=True)
        return res
    finally:
        coord.stop()


if __name__ == "__main__":
    main()
