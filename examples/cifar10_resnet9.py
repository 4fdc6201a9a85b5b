#!/usr/bin/env python3
"""CIFAR-10 ResNet-9 (reference examples/cifar10_resnet9.cpp): crop + flip + cutout + normalize,
Adam with L2 weight decay 5e-4, log-softmax cross-entropy.  ``--fp32`` runs the fp32 MFMA path
(BASELINE config "CIFAR-10 ResNet-9 fp32 on one MI355X")."""
from common import loaders, parse, place

from dcnn_amd.data import AugmentationBuilder
from dcnn_amd.models import create_model
from dcnn_amd.nn import Adam, LossFactory, train_classification_model
from dcnn_amd.utils import get_env

MEAN, STD = (0.49139968, 0.48215827, 0.44653124), (0.24703233, 0.24348505, 0.26158768)
a, cfg = parse(__doc__)
tr, te = loaders("cifar10", a, cfg)
tr.set_augmentation(AugmentationBuilder().random_crop(0.5, 4).horizontal_flip(0.5).cutout(0.5, 8)
                    .normalize(MEAN, STD).build())
te.set_augmentation(AugmentationBuilder().normalize(MEAN, STD).build())
model = place(create_model("resnet9_cifar10"), a)
opt = Adam(get_env("LR_INITIAL", 0.001), 0.9, 0.999, 1e-8, 5e-4)
train_classification_model(model, tr, te, opt, LossFactory.create("logsoftmax_crossentropy"), cfg)
