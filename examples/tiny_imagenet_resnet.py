#!/usr/bin/env python3
"""Tiny-ImageNet ResNet-18/34/50 trainers (reference examples/tiny_imagenet_resnet{18,34,50}.cpp):
flip + crop + normalize, Adam (eps 1e-7), log-softmax cross-entropy, per-layer profiling.

    DEVICE_TYPE=GPU python examples/tiny_imagenet_resnet.py --depth 18 --batch-size 256
"""
from common import loaders, parse, place

from dcnn_amd.data import AugmentationBuilder
from dcnn_amd.models import create_model
from dcnn_amd.nn import Adam, LossFactory, train_classification_model
from dcnn_amd.utils import get_env

MEAN, STD = (0.485, 0.456, 0.406), (0.229, 0.224, 0.225)
a, cfg = parse(__doc__, lambda ap: ap.add_argument("--depth", type=int, default=18, choices=[18, 34, 50]))
tr, te = loaders("tiny", a, cfg)
tr.set_augmentation(AugmentationBuilder().horizontal_flip(0.2).random_crop(0.25, 4).normalize(MEAN, STD).build())
te.set_augmentation(AugmentationBuilder().normalize(MEAN, STD).build())
model = place(create_model(f"resnet{a.depth}_tiny_imagenet"), a)
opt = Adam(get_env("LR_INITIAL", 0.001), 0.9, 0.999, 1e-7)
train_classification_model(model, tr, te, opt, LossFactory.create("logsoftmax_crossentropy"), cfg)
