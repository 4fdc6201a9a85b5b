"""Trainer loop, env config, checkpoint/resume (reference include/nn/train.hpp)."""
import os

import numpy as np
import pytest
import torch

from dcnn_amd.data import ArrayDataLoader, SyntheticDataLoader
from dcnn_amd.models import zoo
from dcnn_amd.nn import (Adam, LossFactory, SequentialBuilder, TrainingConfig, load_checkpoint, save_checkpoint,
                         train_classification_model, train_regression_model)
from dcnn_amd.nn.schedulers import SchedulerFactory
from dcnn_amd.utils import ProfilerType


def test_config_from_env(monkeypatch):
    for k, v in dict(EPOCHS="3", BATCH_SIZE="64", LR_DECAY_FACTOR="0.5", LR_DECAY_INTERVAL="2",
                     PROGRESS_PRINT_INTERVAL="7", PROFILER_TYPE="CUMULATIVE", PRINT_LAYER_PROFILING="true",
                     NUM_MICROBATCHES="4", DEVICE_TYPE="gpu").items():
        monkeypatch.setenv(k, v)
    c = TrainingConfig().load_from_env()
    assert (c.epochs, c.batch_size, c.lr_decay_factor, c.lr_decay_interval, c.progress_print_interval) == \
        (3, 64, 0.5, 2, 7)
    assert c.profiler_type == ProfilerType.CUMULATIVE and c.print_layer_profiling and c.num_microbatches == 4
    assert c.device_type == "GPU"


def _separable(n, seed):
    g = np.random.default_rng(seed)
    y = g.integers(0, 4, n)
    x = g.normal(0, 0.3, (n, 1, 8, 8)).astype(np.float32)
    for i in range(n):
        r, c = divmod(int(y[i]), 2)
        x[i, 0, r * 4:(r + 1) * 4, c * 4:(c + 1) * 4] += 1.5
    return x, y


def _tiny_cnn():
    return (SequentialBuilder("tiny_cnn").input([1, 8, 8]).conv2d(8, 3, 3, 1, 1, 1, 1).batchnorm().activation("relu")
            .maxpool2d(2, 2, 2, 2).flatten().dense(4).build())


def test_train_classification_learns_and_snapshots(tmp_path):
    xtr, ytr = _separable(256, 0)
    xte, yte = _separable(64, 1)
    tr = ArrayDataLoader(xtr, ytr, 4, shuffle=True, seed=0)
    te = ArrayDataLoader(xte, yte, 4)
    model = _tiny_cnn()
    model.set_seed(0)
    opt = Adam(0.01)
    cfg = TrainingConfig(epochs=3, batch_size=32, progress_print_interval=0, lr_decay_interval=2,
                         lr_decay_factor=0.5, snapshot_dir=str(tmp_path))
    hist = train_classification_model(model, tr, te, opt, LossFactory.create("softmax_crossentropy"), cfg)
    assert hist[-1]["val_acc"] > 0.9
    assert opt.get_learning_rate() == pytest.approx(0.005)
    snap = os.path.join(str(tmp_path), "tiny_cnn")
    assert os.path.exists(snap + ".bin") and os.path.exists(snap + ".state")


def test_scheduler_drives_trainer(tmp_path):
    x, y = _separable(64, 2)
    ld = ArrayDataLoader(x, y, 4)
    model = _tiny_cnn()
    opt = Adam(0.01)
    sch = SchedulerFactory.create_from_config({"type": "step_lr", "parameters": {"step_size": 1, "gamma": 0.1}}, opt) \
        if hasattr(SchedulerFactory, "create_from_config") else None
    if sch is None:
        pytest.skip("scheduler factory API")
    train_classification_model(model, ld, ld, opt, LossFactory.create("softmax_crossentropy"),
                               TrainingConfig(epochs=2, batch_size=32, progress_print_interval=0,
                                              snapshot_dir=str(tmp_path)), scheduler=sch)
    assert opt.get_learning_rate() == pytest.approx(1e-4)


def test_checkpoint_resume_is_exact(tmp_path):
    x, y = _separable(64, 3)
    lf = LossFactory.create("softmax_crossentropy")
    from dcnn_amd.runtime.step import TrainStep

    def run(model, opt, steps):
        st = TrainStep(model, lf, opt)
        for i in range(steps):
            st(torch.from_numpy(x[i * 16:(i + 1) * 16]), torch.from_numpy(y[i * 16:(i + 1) * 16]))

    a = _tiny_cnn()
    a.set_seed(1)
    a.initialize()
    oa = Adam(0.01)
    oa.attach(a)
    run(a, oa, 2)
    path = str(tmp_path / "ck")
    save_checkpoint(a, oa, path, epoch=5)
    b = _tiny_cnn()
    b.set_seed(99)
    b.initialize()
    ob = Adam(0.5)
    assert load_checkpoint(b, ob, path) == 5
    assert ob.get_learning_rate() == pytest.approx(0.01)
    run(a, oa, 2)
    run(b, ob, 2)
    for p, q in zip(a.parameters(), b.parameters()):
        torch.testing.assert_close(p, q)


def test_regression_trainer(tmp_path):
    g = np.random.default_rng(0)
    x = g.normal(0, 1, (256, 6)).astype(np.float32)
    w = g.normal(0, 1, (6, 2)).astype(np.float32)
    y = (x @ w).astype(np.float32)
    ld = ArrayDataLoader(x.reshape(256, 6, 1, 1), y, 0, shuffle=True)
    model = SequentialBuilder("reg").input([6, 1, 1]).flatten().dense(16).activation("relu").dense(2).build()
    hist = train_regression_model(model, ld, ld, Adam(0.01), LossFactory.create("mse"),
                                  TrainingConfig(epochs=8, batch_size=32, snapshot_dir=str(tmp_path)))
    assert hist[-1]["val_loss"] < 0.3 * hist[0]["val_loss"] + 1e-3
