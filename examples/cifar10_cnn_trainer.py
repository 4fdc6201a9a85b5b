#!/usr/bin/env python3
"""CIFAR-10 CNN trainer (reference examples/cifar10_cnn_trainer.cpp): flip/contrast/noise/crop
augmentation, Adam, softmax cross-entropy."""
from common import loaders, parse, place

from dcnn_amd.data import AugmentationBuilder
from dcnn_amd.models import create_model
from dcnn_amd.nn import Adam, LossFactory, train_classification_model
from dcnn_amd.utils import get_env

a, cfg = parse(__doc__, lambda ap: ap.add_argument("--model", default="cifar10_cnn_v2"))
tr, te = loaders("cifar10", a, cfg)
tr.set_augmentation(AugmentationBuilder().horizontal_flip(0.25).contrast(0.3, 0.15).gaussian_noise(0.3, 0.05)
                    .random_crop(0.4, 4).build())
model = place(create_model(a.model), a)
opt = Adam(get_env("LR_INITIAL", 0.001), 0.9, 0.999, 1e-8)
train_classification_model(model, tr, te, opt, LossFactory.create("softmax_crossentropy"), cfg)
