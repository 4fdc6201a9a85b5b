"""Pipeline training loops (reference include/pipeline/train.hpp:14-136).

``train_semi_async_epoch`` splits each batch into micro-batches, runs the coordinator's
schedule (semi-async by default) and the parameter update; ``validate_semi_async_epoch``
runs forward-only in eval mode; ``train_model`` drives epochs with an optional scheduler.
Per-batch wall time is recorded (the reference prints "Async process" µs per batch).
"""
from __future__ import annotations

import time
from typing import Optional

from . import messages as M


def train_semi_async_epoch(coord, loader, schedule: str = "semi_async", print_interval: int = 0,
                           max_batches: Optional[int] = None, metrics=None) -> dict:
    coord.broadcast(M.CommandType.TRAIN_MODE)
    loader.reset()
    tot_loss, tot_correct, n_samples, n_batches = 0.0, 0, 0, 0
    t_epoch = time.perf_counter()
    batch_us = []
    while True:
        b = loader.get_next_batch()
        if b is None:
            break
        x, y = b
        t0 = time.perf_counter()
        loss = coord.train_step(x, y, schedule)
        batch_us.append((time.perf_counter() - t0) * 1e6)
        tot_loss += loss
        tot_correct += coord.last_correct
        n_samples += x.shape[0]
        n_batches += 1
        if print_interval and n_batches % print_interval == 0:
            print(f"  batch {n_batches}: loss {loss:.4f} acc {coord.last_correct / x.shape[0]:.4f} "
                  f"({batch_us[-1]:.0f} us)", flush=True)
            if metrics is not None:
                metrics.log("pipeline_batch", batch=n_batches, loss=loss, acc=coord.last_correct / x.shape[0],
                            batch_us=batch_us[-1], schedule=schedule)
        if max_batches and n_batches >= max_batches:
            break
    secs = time.perf_counter() - t_epoch
    return {"loss": tot_loss / max(n_batches, 1), "accuracy": tot_correct / max(n_samples, 1),
            "batches": n_batches, "samples": n_samples, "epoch_ms": secs * 1e3,
            "images_per_sec": n_samples / secs if secs > 0 else 0.0,
            "avg_batch_us": sum(batch_us) / max(len(batch_us), 1)}


def validate_semi_async_epoch(coord, loader, max_batches: Optional[int] = None) -> dict:
    coord.broadcast(M.CommandType.EVAL_MODE)
    loader.reset()
    tot_loss, tot_correct, n, nb = 0.0, 0, 0, 0
    while True:
        b = loader.get_next_batch()
        if b is None:
            break
        x, y = b
        loss, correct = coord.evaluate_batch(x, y)
        tot_loss += loss
        tot_correct += correct
        n += x.shape[0]
        nb += 1
        if max_batches and nb >= max_batches:
            break
    coord.broadcast(M.CommandType.TRAIN_MODE)
    return {"loss": tot_loss / max(nb, 1), "accuracy": tot_correct / max(n, 1), "batches": nb}


def train_model(coord, train_loader, test_loader=None, epochs: int = 1, schedule: str = "semi_async",
                scheduler=None, print_interval: int = 0, max_batches: Optional[int] = None, metrics=None) -> list:
    """Epoch loop; ``metrics`` (default: a MetricsSink on ``METRICS_FILE`` when set) gets per-interval
    and per-epoch JSON records."""
    from ...utils.metrics import MetricsSink
    if metrics is None:
        metrics = MetricsSink(tag="pipeline")
    history = []
    for ep in range(epochs):
        tr = train_semi_async_epoch(coord, train_loader, schedule, print_interval, max_batches, metrics)
        rec = {"epoch": ep + 1, "train": tr}
        if test_loader is not None:
            rec["val"] = validate_semi_async_epoch(coord, test_loader, max_batches)
        print(f"epoch {ep + 1}: loss {tr['loss']:.4f} acc {tr['accuracy']:.4f} "
              f"{tr['epoch_ms']:.0f} ms ({tr['images_per_sec']:.0f} img/s)"
              + (f" | val loss {rec['val']['loss']:.4f} acc {rec['val']['accuracy']:.4f}" if "val" in rec else ""),
              flush=True)
        if scheduler is not None:  # schedulers drive the coordinator (get/set_learning_rate)
            if getattr(scheduler, "type_name", "") == "reduce_lr_on_plateau":
                scheduler.step(rec.get("val", tr)["loss"])
            else:
                scheduler.step()
        history.append(rec)
        metrics.log("pipeline_epoch", epoch=ep + 1, schedule=schedule,
                    **{f"train_{k}": v for k, v in tr.items()},
                    **({f"val_{k}": v for k, v in rec["val"].items()} if "val" in rec else {}))
    return history
