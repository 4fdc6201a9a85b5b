#!/usr/bin/env python3
"""CIFAR-100 CNN trainer (reference examples/cifar100_cnn_trainer.cpp): Adam, cross-entropy on
probabilities (softmax head)."""
from common import loaders, parse, place

from dcnn_amd.nn import Adam, LossFactory, SequentialBuilder, train_classification_model
from dcnn_amd.utils import get_env

a, cfg = parse(__doc__)
tr, te = loaders("cifar100", a, cfg)
model = (SequentialBuilder("cifar100_cnn").input([3, 32, 32])
         .conv2d(64, 3, 3, 1, 1, 1, 1).batchnorm().activation("relu").maxpool2d(2, 2, 2, 2)
         .conv2d(128, 3, 3, 1, 1, 1, 1).batchnorm().activation("relu").maxpool2d(2, 2, 2, 2)
         .conv2d(256, 3, 3, 1, 1, 1, 1).batchnorm().activation("relu").maxpool2d(2, 2, 2, 2)
         .flatten().dense(512).activation("relu").dropout(0.3).dense(100).activation("softmax").build())
model = place(model, a)
opt = Adam(get_env("LR_INITIAL", 0.001), 0.9, 0.999, 1e-8)
train_classification_model(model, tr, te, opt, LossFactory.create("crossentropy"), cfg)
