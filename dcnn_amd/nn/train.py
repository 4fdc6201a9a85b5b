"""Single-process / data-parallel trainers (reference include/nn/train.hpp:46-481).

``TrainingConfig`` keeps the reference fields and ``load_from_env`` keys (EPOCHS, BATCH_SIZE,
LR_DECAY_FACTOR, LR_DECAY_INTERVAL, PROGRESS_PRINT_INTERVAL, NUM_THREADS, PROFILER_TYPE,
PRINT_LAYER_PROFILING, NUM_MICROBATCHES, DEVICE_TYPE) plus MI355X options (hipGraph
capture, bucket size).  ``train_classification_model`` runs epochs of
``train_class_epoch`` + ``validate_class_model``, snapshots the best validation model to
``model_snapshots/<name>`` (weights .bin/.json + .state sidecar with BN statistics,
optimizer moments, epoch and LR — a true resume point the reference lacks) and
decays the LR every ``lr_decay_interval`` epochs (or steps a scheduler).

Loss and correct-count accumulate on the device; the host synchronises only at print
intervals and epoch ends.  Under ``torch.distributed`` each rank trains on its shard of the
epoch and gradients are all-reduced by ``DataParallel`` (overlapped with backward).
"""
from __future__ import annotations

import math
import os
import time
from dataclasses import dataclass
from typing import Optional

import torch
import torch.distributed as dist

from ..utils.env import get_env
from ..utils.memory import get_memory_usage_kb
from ..utils.profiling import ProfilerType

DEFAULT_EPOCH = 10
DEFAULT_BATCH_SIZE = 32
DEFAULT_LR_DECAY_FACTOR = 0.9
DEFAULT_LR_DECAY_INTERVAL = 5
DEFAULT_PRINT_INTERVAL = 100
DEFAULT_NUM_THREADS = 8


@dataclass
class TrainingConfig:
    epochs: int = DEFAULT_EPOCH
    batch_size: int = DEFAULT_BATCH_SIZE
    lr_decay_factor: float = DEFAULT_LR_DECAY_FACTOR
    lr_decay_interval: int = DEFAULT_LR_DECAY_INTERVAL
    progress_print_interval: int = DEFAULT_PRINT_INTERVAL
    num_threads: int = DEFAULT_NUM_THREADS
    profiler_type: ProfilerType = ProfilerType.NONE
    print_layer_profiling: bool = False
    device_type: str = "CPU"
    num_microbatches: int = 2
    use_graph: bool = True          # hipGraph-captured step on the GPU
    bucket_mb: float = 4.0          # DP all-reduce bucket size (small trailing bucket = little exposed comm)
    snapshot_dir: str = "model_snapshots"
    max_batches_per_epoch: int = 0  # 0 = full epoch

    def load_from_env(self) -> "TrainingConfig":
        self.epochs = get_env("EPOCHS", DEFAULT_EPOCH)
        self.batch_size = get_env("BATCH_SIZE", DEFAULT_BATCH_SIZE)
        self.lr_decay_factor = get_env("LR_DECAY_FACTOR", DEFAULT_LR_DECAY_FACTOR)
        self.lr_decay_interval = get_env("LR_DECAY_INTERVAL", DEFAULT_LR_DECAY_INTERVAL)
        self.progress_print_interval = get_env("PROGRESS_PRINT_INTERVAL", DEFAULT_PRINT_INTERVAL)
        self.profiler_type = ProfilerType.parse(get_env("PROFILER_TYPE", "NONE"))
        self.num_threads = get_env("NUM_THREADS", DEFAULT_NUM_THREADS)
        self.print_layer_profiling = get_env("PRINT_LAYER_PROFILING", False)
        self.num_microbatches = get_env("NUM_MICROBATCHES", 2)
        self.device_type = get_env("DEVICE_TYPE", "CPU").upper()
        self.use_graph = get_env("USE_HIPGRAPH", True)
        return self

    def print_config(self) -> None:
        print("Training Configuration:")
        for k, v in self.__dict__.items():
            print(f"  {k}: {v.name if isinstance(v, ProfilerType) else v}")


class _Acc:
    """Device-side running sums of loss / corrects (no per-batch host sync)."""

    def __init__(self, device):
        self.loss = torch.zeros((), dtype=torch.float64, device=device)
        self.correct = torch.zeros((), dtype=torch.int64, device=device)
        self.samples = 0
        self.batches = 0

    def add(self, loss, correct, n):
        self.loss += loss.reshape(()).to(torch.float64)
        if correct is not None:
            self.correct += correct.reshape(()).to(torch.int64)
        self.samples += n
        self.batches += 1

    def result(self):
        tot = torch.stack([self.loss, self.correct.to(torch.float64)]).cpu()
        return float(tot[0]) / max(self.batches, 1), float(tot[1]) / max(self.samples, 1)


def _shard(loader):
    """Restrict this epoch's sample order to the local rank's shard."""
    if dist.is_initialized() and dist.get_world_size() > 1 and loader.order is not None:
        r, w = dist.get_rank(), dist.get_world_size()
        n = (len(loader.order) // w) * w
        loader.order = loader.order[:n][r::w].copy()


def train_class_epoch(model, train_loader, optimizer, loss_function, config: Optional[TrainingConfig] = None,
                      step=None, metrics=None) -> tuple:
    """One epoch; returns (avg loss, accuracy). ``step`` is a prebuilt ``TrainStep``; ``metrics``
    a :class:`~dcnn_amd.utils.metrics.MetricsSink` that gets a record per print interval."""
    from ..runtime.step import TrainStep
    config = config or TrainingConfig()
    model.set_training(True)
    train_loader.reset()
    _shard(train_loader)
    dev = model.device.torch_device
    if step is None:
        step = TrainStep(model, loss_function, optimizer, use_graph=config.use_graph and model.device.is_gpu())
    acc = _Acc(dev)
    graph_bs = None
    while True:
        b = train_loader.get_next_batch()
        if b is None:
            break
        x, y = b
        x, y = x.to(dev, non_blocking=True), y.to(dev, non_blocking=True)
        n = x.shape[0]
        if step.use_graph and graph_bs is None:
            graph_bs = n
        if step.use_graph and n != graph_bs:
            loss = step.eager(x, y)  # ragged last batch: same kernels, not captured
        else:
            loss = step(x, y)
        acc.add(loss, step.last_correct, n)
        if config.progress_print_interval and acc.batches % config.progress_print_interval == 0:
            if model.enable_profiling_ and config.profiler_type != ProfilerType.NONE:
                model.print_profiling_summary()
            l, a = acc.result()
            print(f"Batch ID: {acc.batches}, Batch's Loss: {float(loss):.4f}, Cumulative Accuracy: {a * 100:.2f}%",
                  flush=True)
            if metrics is not None:
                metrics.log("batch", batch=acc.batches, loss=float(loss), cumulative_acc=a,
                            lr=optimizer.get_learning_rate())
        if model.enable_profiling_ and config.profiler_type == ProfilerType.NORMAL:
            model.clear_profiling_data()
        if config.max_batches_per_epoch and acc.batches >= config.max_batches_per_epoch:
            break
    return acc.result()


def validate_class_model(model, test_loader, loss_function, max_batches: int = 0) -> tuple:
    model.set_training(False)
    test_loader.reset()
    dev = model.device.torch_device
    acc = _Acc(dev)
    with torch.no_grad():
        while True:
            b = test_loader.get_next_batch()
            if b is None:
                break
            x, y = b
            out = model.forward(x.to(dev), 0, return_on_input_device=False)
            model.clear_cache(0)
            loss, _, correct = loss_function.loss_and_grad(out, y.to(dev), want_grad=False)
            acc.add(loss, correct, x.shape[0])
            if max_batches and acc.batches >= max_batches:
                break
    model.set_training(True)
    return acc.result()


def save_checkpoint(model, optimizer, path: str, epoch: int = 0, extra: Optional[dict] = None) -> None:
    """Reference-format weights (.json/.bin) + .state sidecar (BN stats, optimizer, epoch, LR)."""
    state = {"epoch": int(epoch), "learning_rate": float(optimizer.get_learning_rate()) if optimizer else 0.0}
    if optimizer is not None:
        for k, v in optimizer.state_dict().items():
            state[f"optimizer:{k}"] = v
    if extra:
        state.update(extra)
    model.save_to_file(path, save_state=False)
    model.save_state(path + ".state", extra=state)


def load_checkpoint(model, optimizer, path: str) -> int:
    """Restore weights, BN statistics and optimizer state; returns the saved epoch."""
    model.load_weights_file(path + ".bin")
    st = model.load_state(path + ".state") if os.path.exists(path + ".state") else {}
    if optimizer is not None and st:
        if not optimizer.params:
            optimizer.attach(model)
        optimizer.load_state_dict({k.split(":", 1)[1]: v for k, v in st.items() if k.startswith("optimizer:")})
        if "learning_rate" in st:
            optimizer.set_learning_rate(float(st["learning_rate"]))
    return int(st.get("epoch", 0))


def train_classification_model(model, train_loader, test_loader, optimizer, loss_function,
                               config: Optional[TrainingConfig] = None, scheduler=None, data_parallel=None,
                               start_epoch: int = 0, metrics=None) -> list:
    """Epoch loop (reference include/nn/train.hpp:191-268). ``metrics``: a MetricsSink (default:
    one on ``METRICS_FILE`` when set) receiving per-interval and per-epoch JSON records."""
    from ..parallel.dp import DataParallel
    from ..runtime.step import TrainStep
    from ..utils.metrics import MetricsSink
    config = config or TrainingConfig()
    if not model.initialized:
        model.initialize()
    rank = dist.get_rank() if dist.is_initialized() else 0
    dp = data_parallel or DataParallel(model, bucket_mb=config.bucket_mb)
    optimizer.attach(model)
    train_loader.prepare_batches(config.batch_size)
    test_loader.prepare_batches(config.batch_size)
    model.enable_profiling(config.profiler_type != ProfilerType.NONE)
    if rank == 0:
        print(f"Training batches: {train_loader.num_batches()}\nValidation batches: {test_loader.num_batches()}")
        model.print_summary([config.batch_size] + train_loader.get_data_shape())
    step = TrainStep(dp, loss_function, optimizer, use_graph=config.use_graph and model.device.is_gpu())
    if metrics is None and rank == 0:
        metrics = MetricsSink(tag=model.name())
    best = -math.inf
    history = []
    for epoch in range(start_epoch, config.epochs):
        if rank == 0:
            print(f"Epoch {epoch + 1}/{config.epochs}", flush=True)
        t0 = time.perf_counter()
        tr_loss, tr_acc = train_class_epoch(model, train_loader, optimizer, loss_function, config, step,
                                            metrics if rank == 0 else None)
        if model.device.is_gpu():
            torch.cuda.synchronize()
        train_ms = (time.perf_counter() - t0) * 1e3
        dp.sync_batchnorm_buffers()
        va_loss, va_acc = validate_class_model(model, test_loader, loss_function, config.max_batches_per_epoch)
        n_img = train_loader.size() if not config.max_batches_per_epoch else \
            min(train_loader.size(), config.max_batches_per_epoch * config.batch_size)
        rec = {"epoch": epoch + 1, "train_loss": tr_loss, "train_acc": tr_acc, "val_loss": va_loss, "val_acc": va_acc,
               "train_ms": train_ms, "images_per_sec": n_img / (train_ms / 1e3) if train_ms else 0.0}
        history.append(rec)
        if rank == 0 and metrics is not None:
            metrics.log("epoch", lr=optimizer.get_learning_rate(), host_mem_mb=get_memory_usage_kb() // 1024, **rec)
        if rank == 0:
            if va_acc > best:
                best = va_acc
                print(f"New best validation accuracy: {best * 100:.2f}%")
                path = os.path.join(config.snapshot_dir, model.name())
                try:
                    save_checkpoint(model, optimizer, path, epoch + 1)
                    print(f"Model saved to {path}")
                except OSError as e:
                    print(f"Error saving model: {e}")
            print("-" * 60)
            print(f"Epoch {epoch + 1}/{config.epochs} completed in {train_ms:.0f}ms "
                  f"({rec['images_per_sec']:.0f} images/sec)")
            print(f"Training   - Loss: {tr_loss:.4f}, Accuracy: {tr_acc * 100:.2f}%")
            print(f"Validation - Loss: {va_loss:.4f}, Accuracy: {va_acc * 100:.2f}%")
            print("=" * 60, flush=True)
        if model.enable_profiling_:
            model.clear_profiling_data()
        if scheduler is not None:
            if getattr(scheduler, "type_name", "") == "reduce_lr_on_plateau":
                scheduler.step(va_loss)
            else:
                scheduler.step()
        elif config.lr_decay_interval and (epoch + 1) % config.lr_decay_interval == 0:
            cur = optimizer.get_learning_rate()
            optimizer.set_learning_rate(cur * config.lr_decay_factor)
            if rank == 0:
                print(f"Learning rate decayed: {cur:.6f} -> {cur * config.lr_decay_factor:.6f}")
        if rank == 0:
            print(f"{get_memory_usage_kb() // 1024} MB of memory used.")
    return history


# ---------------------------------------------------------------- regression (reference train_reg_epoch)
def train_reg_epoch(model, loader, optimizer, loss_function, config: Optional[TrainingConfig] = None):
    from ..runtime.step import TrainStep
    config = config or TrainingConfig()
    model.set_training(True)
    loader.reset()
    dev = model.device.torch_device
    step = TrainStep(model, loss_function, optimizer, use_graph=False)
    acc = _Acc(dev)
    while True:
        b = loader.get_next_batch()
        if b is None:
            break
        x, y = b
        loss = step(x.to(dev), y.to(dev))
        acc.add(loss, None, x.shape[0])
    return acc.result()[0]


def validate_reg_model(model, loader, loss_function) -> tuple:
    """(avg loss, mean Euclidean error of the prediction) on the loader's (normalised) targets."""
    model.set_training(False)
    loader.reset()
    dev = model.device.torch_device
    tot, err, n, nb = 0.0, 0.0, 0, 0
    while True:
        b = loader.get_next_batch()
        if b is None:
            break
        x, y = b
        out = model.forward(x.to(dev), 0, return_on_input_device=False).float().reshape(x.shape[0], -1)
        model.clear_cache(0)
        y = y.to(dev).float().reshape(out.shape)
        tot += float(loss_function.loss_and_grad(out, y, want_grad=False)[0])
        err += float(torch.linalg.vector_norm(out - y, dim=1).sum())
        n += x.shape[0]
        nb += 1
    model.set_training(True)
    return tot / max(nb, 1), err / max(n, 1)


def train_regression_model(model, train_loader, test_loader, optimizer, loss_function,
                           config: Optional[TrainingConfig] = None) -> list:
    config = config or TrainingConfig()
    if not model.initialized:
        model.initialize()
    optimizer.attach(model)
    train_loader.prepare_batches(config.batch_size)
    test_loader.prepare_batches(config.batch_size)
    best, _ = validate_reg_model(model, test_loader, loss_function)
    hist = []
    for epoch in range(config.epochs):
        t0 = time.perf_counter()
        tr = train_reg_epoch(model, train_loader, optimizer, loss_function, config)
        va, verr = validate_reg_model(model, test_loader, loss_function)
        hist.append({"epoch": epoch + 1, "train_loss": tr, "val_loss": va, "val_error": verr,
                     "ms": (time.perf_counter() - t0) * 1e3})
        print(f"Epoch {epoch + 1}/{config.epochs}: train loss {tr:.4f} | val loss {va:.4f} error {verr:.4f}",
              flush=True)
        if va < best:
            best = va
            save_checkpoint(model, optimizer, os.path.join(config.snapshot_dir, model.name()), epoch + 1)
        if config.lr_decay_interval and (epoch + 1) % config.lr_decay_interval == 0:
            optimizer.set_learning_rate(optimizer.get_learning_rate() * config.lr_decay_factor)
    return hist
