#!/usr/bin/env python3
"""Semi-asynchronous pipeline (reference examples/semi_async_pipeline_coordinator.cpp and
coordinator_tiny_imagenet.cpp): forwards of every micro-batch issued at once, each output's
loss/backward launched on arrival, stages prioritising forward jobs.

    python examples/semi_async_pipeline_coordinator.py --local --model resnet9_cifar10
    python examples/semi_async_pipeline_coordinator.py --model resnet18_tiny_imagenet --dataset tiny
"""
from common import loaders, parse

from dcnn_amd.models import create_model
from dcnn_amd.nn import Adam
from dcnn_amd.parallel.pipeline import (DistributedCoordinator, Endpoint, FlopPartitioner, InProcessCoordinator,
                                        train_model)
from dcnn_amd.models import INPUT_SHAPES
from dcnn_amd.utils import get_env


def extra(ap):
    ap.add_argument("--local", action="store_true")
    ap.add_argument("--model", default="resnet9_cifar10")
    ap.add_argument("--dataset", default="cifar10", choices=["mnist", "cifar10", "cifar100", "tiny"])
    ap.add_argument("--stages", type=int, default=2)


a, cfg = parse(__doc__, extra)
tr, te = loaders(a.dataset, a, cfg)
model = create_model(a.model)
m = cfg.num_microbatches
part = FlopPartitioner([max(cfg.batch_size // m, 1)] + list(INPUT_SHAPES[a.model]))
devs = [a.device] * a.stages if not a.device.startswith("GPU") else \
    [f"GPU:{i % max(__import__('torch').cuda.device_count(), 1)}" for i in range(a.stages)]
kw = dict(num_microbatches=m, partitioner=part, stage_devices=devs, device=devs[0])
if a.local:
    coord = InProcessCoordinator(model, Adam(1e-3), "logsoftmax_crossentropy", num_stages=a.stages, **kw)
else:
    eps = [Endpoint.network(get_env(f"WORKER{i + 1}_HOST", "127.0.0.1"), get_env(f"WORKER{i + 1}_PORT", 8001 + i))
           for i in range(a.stages)]
    coord = DistributedCoordinator(model, Adam(1e-3), "logsoftmax_crossentropy", eps, **kw)
coord.initialize()
print("partitions:", coord.partitions)
coord.deploy_stages()
from dcnn_amd.utils.metrics import maybe_start_cpu_logger  # noqa: E402
cpu_log = maybe_start_cpu_logger("coordinator")  # CPU_LOG_DIR=./logs -> tools/plot_cpu_range.py
coord.start()
tr.prepare_batches(cfg.batch_size)
te.prepare_batches(cfg.batch_size)
train_model(coord, tr, te, epochs=cfg.epochs, schedule="semi_async", print_interval=cfg.progress_print_interval,
            max_batches=a.max_batches or None)
for line in coord.print_profiling_on_all_stages():
    pass
coord.stop()
if cpu_log is not None:
    print(f"CPU log: {cpu_log.stop()}")
