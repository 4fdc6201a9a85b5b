#!/usr/bin/env python3
"""Headline benchmark: ResNet-18 Tiny-ImageNet training throughput (images/sec, whole node).

Model: `create_resnet18_tiny_imagenet` (reference include/nn/example_models.hpp:306), random
init, synthetic 64x64 RGB inputs + random labels of that shape, bf16 compute with fp32 master
weights, Adam, softmax cross-entropy. Data parallel over RCCL, one process per GPU:

  python bench.py --gpus 1 --steps 50 --warmup 10
  python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
      --master-port 29500 bench.py --gpus 8 --steps 50 --warmup 10

Weak scaling: every rank trains --batch images per step (global batch = batch x gpus). The
gradient all-reduce is bucketed, overlaps the backward and is captured in the step graph. On the
C++ engine (the default) it runs on the in-tree RCCL communicator; on the Python engine on
torch.distributed's ProcessGroupNCCL (RCCL) by default, or on the framework's own RCCL
communicator (parallel/rccl.py, no c10d) with --dp-backend rccl.
Exactly K steps are timed between a barrier + device synchronisation on both sides; the
slowest rank's time is reported. Every timed step runs the full forward, loss, backward,
gradient all-reduce and optimizer update.

Engines: the same step on the C++ host API (bin/tiny_imagenet_resnet18: the framework's own
Tensor, flows and gpu::Graph capture; no torch in the timed process; one child process per rank
under the same launcher variables; at N > 1 rank 0's weights are broadcast and the bucketed,
overlapped gradient mean runs over the in-tree RCCL communicator (dcnn/dist.hpp) inside the captured
step) or on the Python front end (torch tensors, torch.cuda graphs). --engine auto (the default)
picks the C++ engine for ResNet-18/34 at batch <= 256 at EVERY N, so the 1- and N-GPU points of the
scaling curve come from the same code (same-box A/B at N = 1: profiles/engine_ab_r5.md), and the
Python one for ResNet-50 and larger batches (1-2% faster there). A C++ run that fails on any rank
(the ranks agree over a CPU-only gloo group of this launcher process; no GPU work in it) falls back
to the Python engine on every rank.
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
# ProcessGroupNCCL's event cache vs collectives recorded under hipGraph capture (dcnn_amd/__init__.py)
os.environ.setdefault("TORCH_NCCL_CUDA_EVENT_CACHE", "0")

METRIC = "images/sec (whole node) ResNet-18 Tiny-ImageNet training at 1/2/4/8 MI355X"
ROOT = os.path.dirname(os.path.abspath(__file__))


class NativeFailed(Exception):
    pass


def _agree_group(timeout_s):
    """A CPU-only gloo group of the launcher processes (no GPU): the ranks' agreement on whether
    every C++ child succeeded."""
    import datetime
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=timeout_s))


def native_main(a):
    """The timed steps run in the C++ trainer (one child process per rank, the launcher's RANK /
    WORLD_SIZE / LOCAL_RANK / MASTER_* passed through; the child's own rendezvous at MASTER_PORT +
    17); its JSON line becomes this contract's line on rank 0. Raises NativeFailed (on every rank)
    when any rank's child failed."""
    import subprocess
    world, rank = int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0"))
    if a.gpus != world and world > 1:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={world}")
    if (a.device, a.dtype) not in (("cuda", "bf16"), ("cpu", "fp32")):
        raise SystemExit("--engine native: bf16 on GPUs (or the fp32 CPU backend)")
    model = a.model
    if os.environ.get("DCNN_BENCH_FAULT_RANK") == str(rank):  # (tests: this rank's child fails)
        model = "no_such_model"
    cmd = [os.path.join(ROOT, "dcnn_amd", "bin", "tiny_imagenet_resnet18"), "--device",
           "GPU" if a.device == "cuda" else "CPU", "--model", model,
           "--batch", str(a.batch), "--steps", str(a.steps), "--warmup", str(a.warmup), "--loss", "softmax_ce",
           "--bench"] + (["--dp"] if world > 1 else [])
    env = dict(os.environ)
    env.setdefault("MASTER_ADDR", "127.0.0.1")
    env.setdefault("MASTER_PORT", "29533")
    env.setdefault("DCNN_DP_BUCKET_MB", str(a.bucket_mb))
    env.setdefault("DCNN_DIST_TIMEOUT", "180")
    if world > 1:
        _agree_group(a.native_timeout + 300)
    ok, out, err = False, "", ""
    try:
        r = subprocess.run(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                           timeout=a.native_timeout)
        ok, out, err = r.returncode == 0, r.stdout, r.stderr
        if not ok:
            err += f"\n[bench] rank {rank}: C++ engine exited {r.returncode}"
    except subprocess.TimeoutExpired as e:
        out = e.stdout.decode() if isinstance(e.stdout, bytes) else (e.stdout or "")
        err = (e.stderr.decode() if isinstance(e.stderr, bytes) else (e.stderr or "")) + \
            f"\n[bench] rank {rank}: C++ engine timed out after {a.native_timeout} s"
    lines = [l for l in out.splitlines() if l.startswith("{")]
    ok = ok and (rank != 0 or bool(lines))
    if world > 1:
        flag = torch.tensor([1 if ok else 0], dtype=torch.int32)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        all_ok = bool(flag.item())
        dist.destroy_process_group()
    else:
        all_ok = ok
    if not all_ok:
        print(out[-2000:] + err[-4000:], file=sys.stderr, flush=True)
        raise NativeFailed(f"rank {rank}: {'ok' if ok else 'failed'}; another rank failed" if ok else f"rank {rank} failed")
    if rank != 0:
        return
    d = json.loads(lines[-1])
    from dcnn_amd.models import INPUT_SHAPES
    C, H, W = INPUT_SHAPES[a.model]
    print(json.dumps({
        "metric": METRIC if a.model == "resnet18_tiny_imagenet" else f"images/sec (whole node) {a.model} training",
        "value": round(d["value"], 2), "unit": "images/sec", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
        "ms_per_step": round(d["ms_per_step"], 4), "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": a.dtype, "data": d.get("data", f"synthetic {H}x{W}x{C}"),
        "config": {"model": a.model, "global_batch": a.batch * world, "per_gpu_batch": a.batch, "seq_len": None,
                   "image_size": [C, H, W], "parallelism": f"dp{world}", "optimizer": "adam",
                   "grad_allreduce": "fp32" if world > 1 else None, "data_plane": d.get("data_parallel"),
                   "dp_buckets": d.get("dp_buckets") if world > 1 else None,
                   "hipgraph": d.get("hipgraph"), "final_loss": round(d.get("loss", float("nan")), 4),
                   "f32_mode": None, "engine": "native (C++ host API)"},
    }), flush=True)


def auto_native(a):
    """--engine auto: the C++ engine covers this run (bf16 on GPUs, the default step options, a
    model of the C++ factory at batch <= 256, the trainer binary built), at any N."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    default_step = (a.graph == 1 and not a.pg and not a.profile and a.grad_dtype == "fp32")
    return (a.gpus == world and a.device == "cuda" and a.dtype == "bf16" and default_step
            and a.model in ("resnet18_tiny_imagenet", "resnet34_tiny_imagenet") and a.batch <= 256
            and os.access(os.path.join(ROOT, "dcnn_amd", "bin", "tiny_imagenet_resnet18"), os.X_OK)
            and torch.cuda.device_count() >= world)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=8)
    ap.add_argument("--batch", type=int, default=int(os.environ.get("DCNN_BENCH_BATCH", "256")))
    ap.add_argument("--model", default="resnet18_tiny_imagenet")
    ap.add_argument("--graph", type=int, default=int(os.environ.get("DCNN_BENCH_GRAPH", "1")),
                    help="capture the per-step compute in a hipGraph (1) or run eagerly (0)")
    ap.add_argument("--bucket-mb", type=float, default=4.0)
    ap.add_argument("--grad-dtype", default="fp32", choices=["fp32", "bf16"],
                    help="gradient all-reduce wire format (bf16: packed shards reduce-scattered + all-gathered)")
    ap.add_argument("--pg", action="store_true",
                    help="create the RCCL process group even at world size 1 (torch data plane)")
    ap.add_argument("--dp-backend", default=os.environ.get("DCNN_DP_BACKEND", "torch"), choices=["rccl", "torch"],
                    help="gradient data plane on GPUs: torch.distributed's ProcessGroupNCCL (RCCL; default) or "
                         "the framework's own RCCL communicator (rank/world from the launcher env, unique id "
                         "over the native TCP plane, no torch.distributed; opt-in, exits non-zero if it cannot "
                         "be built)")
    ap.add_argument("--engine", default=os.environ.get("DCNN_BENCH_ENGINE", "auto"), choices=["auto", "python", "native"],
                    help="native: the C++ host API trainer; python: the Python front end's captured step; auto "
                         "(default): native for ResNet-18/34 at any N (python if it fails on any rank), python "
                         "otherwise")
    ap.add_argument("--native-timeout", type=int, default=int(os.environ.get("DCNN_BENCH_NATIVE_TIMEOUT", "420")),
                    help="seconds the C++ engine's run may take before it counts as failed")
    ap.add_argument("--profile", action="store_true", help="print per-layer device times")
    ap.add_argument("--device", default="cuda")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"],
                    help="compute dtype (fp32: the MFMA f32 path, e.g. the ResNet-9 CIFAR-10 fp32 config)")
    ap.add_argument("--f32-mode", default=os.environ.get("DCNN_BENCH_F32_MODE", "concat"),
                    choices=["concat", "split", "exact"],
                    help="fp32 convolution arithmetic: exact = IEEE fp32 inputs on the f32 MFMA "
                         "(v_mfma_f32_16x16x4_f32) everywhere; concat = 3xbf16 split precision on the "
                         "halo convs ([hi|lo|hi] channels, ~2^-16 relative per product) + exact elsewhere; "
                         "split = 3xbf16 on the gathered GEMMs too")
    a = ap.parse_args()
    if a.engine == "native":
        try:
            return native_main(a)
        except NativeFailed as e:
            raise SystemExit(f"[bench] C++ engine failed: {e}")
    if a.engine == "auto" and auto_native(a):
        try:
            return native_main(a)
        except NativeFailed as e:  # (every rank raises: the agreement above)
            print(f"[bench] C++ engine failed ({e}); running the Python engine", file=sys.stderr, flush=True)

    from dcnn_amd.parallel.dp import DataParallel, init_distributed
    from dcnn_amd.parallel.rccl import env_rank_world
    from dcnn_amd.models import INPUT_SHAPES, NUM_CLASSES, create_model
    from dcnn_amd.nn import Adam, LossFactory
    from dcnn_amd.runtime.step import TrainStep

    in_tree = a.device == "cuda" and a.dp_backend == "rccl" and not a.pg
    if in_tree:
        rank, world, local = env_rank_world()  # no torch.distributed: the in-tree plane bootstraps itself
    else:
        rank, world, local = init_distributed("nccl" if a.device == "cuda" else "gloo")
    if a.pg and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        if a.device == "cuda":
            torch.cuda.set_device(0)
            dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
        else:
            dist.init_process_group("gloo", rank=0, world_size=1)
    if a.gpus != world and world > 1:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={world}")
    dev = torch.device("cuda", local) if a.device == "cuda" else torch.device("cpu")
    if dev.type == "cuda":
        torch.cuda.set_device(dev)

    if a.dtype == "fp32" and dev.type == "cuda":
        from dcnn_amd.ops import hip as _hip
        _hip.set_f32_concat(a.f32_mode == "concat")
        _hip.kernels().set_f32_mode(1 if a.f32_mode == "split" else 0)

    model = create_model(a.model)
    model.set_seed(1234)
    model.set_device(f"GPU:{local}" if dev.type == "cuda" else "CPU")
    if a.dtype == "fp32" and dev.type == "cuda":
        model.set_compute_dtype(torch.float32)
    model.initialize()
    model.set_first_layer_input_grad(False)
    plane = "torch"
    if in_tree:
        try:
            dp = DataParallel(model, bucket_mb=a.bucket_mb, grad_dtype=a.grad_dtype, comm_backend="rccl")
            plane = "rccl" if dp.rccl is not None else "none"
        except Exception as e:
            # no silent switch of planes: a rank failing alone (e.g. a bootstrap timeout) while the
            # others are inside ncclCommInitRank would otherwise split the job across two planes
            print(f"[bench] rank {rank}: in-tree RCCL plane failed ({e}); rerun with --dp-backend torch",
                  file=sys.stderr, flush=True)
            os._exit(3)
    else:
        dp = DataParallel(model, bucket_mb=a.bucket_mb, grad_dtype=a.grad_dtype, comm_backend="torch")
    if plane == "torch" and not dist.is_initialized():
        plane = "none"
    opt = Adam(1e-3)
    opt.attach(model)
    loss_fn = LossFactory.create("softmax_crossentropy")

    C, H, W = INPUT_SHAPES[a.model]
    ncls = NUM_CLASSES[a.model]
    g = torch.Generator(device="cpu").manual_seed(100 + rank)
    nbuf = 4
    xs = [torch.randn(a.batch, C, H, W, generator=g).to(dev) for _ in range(nbuf)]
    ys = [torch.randint(0, ncls, (a.batch,), generator=g).to(dev) for _ in range(nbuf)]

    step = TrainStep(dp, loss_fn, opt, use_graph=bool(a.graph) and dev.type == "cuda")

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        if world > 1:
            dp.barrier()

    for i in range(a.warmup):
        step(xs[i % nbuf], ys[i % nbuf])
    sync()
    t0 = time.perf_counter()
    for i in range(a.steps):
        step(xs[i % nbuf], ys[i % nbuf])
    sync()
    t1 = time.perf_counter()
    el = dp.max_over_ranks(t1 - t0)  # the slowest rank's time
    loss_val = float(step.last_loss.item()) if step.last_loss is not None else float("nan")
    ms = el / a.steps * 1e3
    imgs = a.batch * world * a.steps / el
    timed_with_graph = bool(step.use_graph)  # what the timed loop ran (--profile switches it off below)
    if rank == 0:
        print(json.dumps({
            "metric": METRIC if a.model == "resnet18_tiny_imagenet" else f"images/sec (whole node) {a.model} training",
            "value": round(imgs, 2), "unit": "images/sec", "n_gpus": world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": round(ms, 4), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": a.dtype if dev.type == "cuda" else "fp32", "data": f"synthetic (random {H}x{W}x{C} inputs + random labels, random init)",
            "config": {"model": a.model, "global_batch": a.batch * world, "per_gpu_batch": a.batch, "seq_len": None,
                       "image_size": [C, H, W], "parallelism": f"dp{world}", "optimizer": "adam",
                       "grad_allreduce": a.grad_dtype if world > 1 else None,
                       "data_plane": plane if world > 1 else None,
                       "hipgraph": timed_with_graph, "final_loss": round(loss_val, 4),
                       "f32_mode": (a.f32_mode if a.dtype == "fp32" and dev.type == "cuda" else None)},
        }), flush=True)
    if a.profile and rank == 0:
        # per-layer HIP-event profile, after the JSON line (eager steps: one event pair per layer)
        model.enable_profiling(True)
        step.use_graph = False
        for i in range(3):
            step(xs[0], ys[0])
        print(model.print_profiling_summary(), file=sys.stderr)
    if world > 1:
        dp.barrier()
    if dp.rccl is not None:
        dp.rccl.close()
    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
