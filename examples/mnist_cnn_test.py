#!/usr/bin/env python3
"""Evaluate a saved MNIST snapshot (reference examples/mnist_cnn_test.cpp).

    python examples/mnist_cnn_test.py --snapshot model_snapshots/mnist_cnn
"""
from common import loaders, parse

from dcnn_amd.nn import LossFactory, Sequential, validate_class_model

a, cfg = parse(__doc__, lambda ap: ap.add_argument("--snapshot", default="model_snapshots/mnist_cnn"))
model = Sequential.from_file(a.snapshot, device=a.device)
_, te = loaders("mnist", a, cfg)
te.prepare_batches(cfg.batch_size)
loss, acc = validate_class_model(model, te, LossFactory.create("logsoftmax_crossentropy"))
print(f"Test loss {loss:.4f}, accuracy {acc * 100:.2f}%")
