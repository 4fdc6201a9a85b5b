#!/usr/bin/env python3
"""Synchronous (GPipe) pipeline over network workers (reference
examples/sync_pipeline_coordinator.cpp): MNIST CNN split across WORKER1/WORKER2, per-phase
timings printed per batch.  Start the workers first:

    python -m dcnn_amd.parallel.pipeline.worker 8001 &  python -m dcnn_amd.parallel.pipeline.worker 8002 &
    python examples/sync_pipeline_coordinator.py

``--local`` runs both stages in-process instead (no workers needed).
"""
import time

from common import loaders, parse

from dcnn_amd.models import create_model
from dcnn_amd.nn import Adam
from dcnn_amd.parallel.pipeline import DistributedCoordinator, Endpoint, InProcessCoordinator
from dcnn_amd.parallel.pipeline.messages import CommandType as C
from dcnn_amd.utils import get_env


def extra(ap):
    ap.add_argument("--local", action="store_true")
    ap.add_argument("--model", default="mnist_cnn")


a, cfg = parse(__doc__, extra)
tr, te = loaders("mnist", a, cfg)
model = create_model(a.model)
m = cfg.num_microbatches
kw = dict(num_microbatches=m, stage_devices=[a.device, a.device], device=a.device if a.device != "GPU" else "GPU:0")
if a.local:
    coord = InProcessCoordinator(model, Adam(1e-3), "logsoftmax_crossentropy", num_stages=2, **kw)
else:
    eps = [Endpoint.network(get_env("WORKER1_HOST", "127.0.0.1"), get_env("WORKER1_PORT", 8001)),
           Endpoint.network(get_env("WORKER2_HOST", "127.0.0.1"), get_env("WORKER2_PORT", 8002))]
    coord = DistributedCoordinator(model, Adam(1e-3), "logsoftmax_crossentropy", eps,
                                   host=get_env("COORDINATOR_HOST", "127.0.0.1"),
                                   port=get_env("COORDINATOR_PORT", 0), **kw)
coord.initialize()
coord.deploy_stages()
from dcnn_amd.utils.metrics import maybe_start_cpu_logger  # noqa: E402
cpu_log = maybe_start_cpu_logger("coordinator")  # CPU_LOG_DIR=./logs -> tools/plot_cpu_range.py
coord.start()
tr.prepare_batches(cfg.batch_size)
for ep in range(cfg.epochs):
    tr.reset()
    nb = 0
    while True:
        b = tr.get_next_batch()
        if b is None:
            break
        x, y = b
        xs, ys = coord.split(x, y)
        t0 = time.perf_counter()
        for i, xi in enumerate(xs):
            coord.forward(xi, i)
        outs = {int(msg.mb_id): coord._output(msg) for msg in coord.join(C.FORWARD_JOB, m)}
        t1 = time.perf_counter()
        loss = 0.0
        grads = []
        for i in range(m):
            l, g, _ = coord._loss_grad(outs[i], ys[i], i)
            loss += float(l) / m
            grads.append(g)
        t2 = time.perf_counter()
        for i, g in enumerate(grads):
            coord.backward(g, i)
        coord.join(C.BACKWARD_JOB, m)
        t3 = time.perf_counter()
        coord.update_parameters()
        t4 = time.perf_counter()
        nb += 1
        if cfg.progress_print_interval and nb % cfg.progress_print_interval == 0:
            print(f"batch {nb}: loss {loss:.4f} | forward {1e6 * (t1 - t0):.0f} us, loss {1e6 * (t2 - t1):.0f} us, "
                  f"backward {1e6 * (t3 - t2):.0f} us, update {1e6 * (t4 - t3):.0f} us", flush=True)
        if a.max_batches and nb >= a.max_batches:
            break
    te.prepare_batches(cfg.batch_size)
    from dcnn_amd.parallel.pipeline import validate_semi_async_epoch
    v = validate_semi_async_epoch(coord, te, a.max_batches)
    print(f"epoch {ep + 1}: val loss {v['loss']:.4f} acc {v['accuracy'] * 100:.2f}%", flush=True)
coord.print_profiling_on_all_stages()
coord.stop()
if cpu_log is not None:
    print(f"CPU log: {cpu_log.stop()}")
