#!/usr/bin/env python3
"""MNIST CNN trainer (reference examples/mnist_cnn_trainer.cpp): create_mnist_trainer, Adam,
log-softmax cross-entropy, contrast + gaussian-noise augmentation.

    DEVICE_TYPE=GPU EPOCHS=5 python examples/mnist_cnn_trainer.py
"""
from common import loaders, parse, place

from dcnn_amd.data import AugmentationBuilder
from dcnn_amd.models import create_model
from dcnn_amd.nn import Adam, LossFactory, train_classification_model
from dcnn_amd.utils import get_env

a, cfg = parse(__doc__)
cfg.print_config()
tr, te = loaders("mnist", a, cfg)
tr.set_augmentation(AugmentationBuilder().contrast(0.3, 0.15).gaussian_noise(0.3, 0.05).build())
model = place(create_model("mnist_cnn"), a)
opt = Adam(get_env("LR_INITIAL", 0.01), 0.9, 0.999, 1e-8)
train_classification_model(model, tr, te, opt, LossFactory.create("logsoftmax_crossentropy"), cfg)
