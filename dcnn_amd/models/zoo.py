"""Model zoo: the 13 builders of the reference (`include/nn/example_models.hpp:13-437`),
same layer sequence, names and hyper-parameters, so checkpoints are interchangeable.
"""
from __future__ import annotations

from ..nn.sequential import Sequential, SequentialBuilder


def create_mnist_trainer() -> Sequential:
    return (SequentialBuilder("mnist_cnn_model").input([1, 28, 28])
            .conv2d(8, 5, 5, 1, 1, 0, 0, True, "conv1").batchnorm(1e-5, 0.1, True, "bn1")
            .activation("relu", "relu1").maxpool2d(3, 3, 3, 3, 0, 0, "pool1")
            .conv2d(16, 1, 1, 1, 1, 0, 0, True, "conv2_1x1").batchnorm(1e-5, 0.1, True, "bn2")
            .activation("relu", "relu2")
            .conv2d(48, 5, 5, 1, 1, 0, 0, True, "conv3").batchnorm(1e-5, 0.1, True, "bn3")
            .activation("relu", "relu3").maxpool2d(2, 2, 2, 2, 0, 0, "pool2")
            .flatten("flatten").dense(10, True, "output").build())


def create_cifar10_trainer_v1() -> Sequential:
    return (SequentialBuilder("cifar10_cnn_classifier_v1").input([3, 32, 32])
            .conv2d(16, 3, 3, 1, 1, 0, 0, True, "conv1").batchnorm(1e-5, 0.1, True, "bn1")
            .activation("relu", "relu1").maxpool2d(3, 3, 3, 3, 0, 0, "maxpool1")
            .conv2d(64, 3, 3, 1, 1, 0, 0, True, "conv2").activation("relu", "relu2")
            .maxpool2d(4, 4, 4, 4, 0, 0, "maxpool2").flatten("flatten").dense(10, True, "fc1").build())


def _vgg_body(b: SequentialBuilder) -> SequentialBuilder:
    return (b.conv2d(64, 3, 3, 1, 1, 1, 1, False, "conv0").batchnorm(1e-5, 0.1, True, "bn0").activation("relu", "relu0")
            .conv2d(64, 3, 3, 1, 1, 1, 1, False, "conv1").batchnorm(1e-5, 0.1, True, "bn1").activation("relu", "relu1")
            .maxpool2d(2, 2, 2, 2, 0, 0, "pool0")
            .conv2d(128, 3, 3, 1, 1, 1, 1, False, "conv2").batchnorm(1e-5, 0.1, True, "bn2").activation("relu", "relu2")
            .conv2d(128, 3, 3, 1, 1, 1, 1, False, "conv3").batchnorm(1e-5, 0.1, True, "bn3").activation("relu", "relu3")
            .maxpool2d(2, 2, 2, 2, 0, 0, "pool1")
            .conv2d(256, 3, 3, 1, 1, 1, 1, False, "conv4").batchnorm(1e-5, 0.1, True, "bn5").activation("relu", "relu5")
            .conv2d(256, 3, 3, 1, 1, 1, 1, False, "conv5").activation("relu", "relu6")
            .conv2d(256, 3, 3, 1, 1, 1, 1, False, "conv6").batchnorm(1e-5, 0.1, True, "bn6").activation("relu", "relu6")
            .maxpool2d(2, 2, 2, 2, 0, 0, "pool2")
            .conv2d(512, 3, 3, 1, 1, 1, 1, False, "conv7").batchnorm(1e-5, 0.1, True, "bn8").activation("relu", "relu7")
            .conv2d(512, 3, 3, 1, 1, 1, 1, False, "conv8").batchnorm(1e-5, 0.1, True, "bn9").activation("relu", "relu8")
            .conv2d(512, 3, 3, 1, 1, 1, 1, False, "conv9").batchnorm(1e-5, 0.1, True, "bn10").activation("relu", "relu9")
            .maxpool2d(2, 2, 2, 2, 0, 0, "pool3").flatten("flatten"))


def create_cifar10_trainer_v2() -> Sequential:
    b = _vgg_body(SequentialBuilder("cifar10_cnn_classifier").input([3, 32, 32]))
    return b.dense(512, True, "fc0").activation("relu", "relu10").dense(10, True, "fc1").build()


def create_resnet9_cifar10() -> Sequential:
    return (SequentialBuilder("ResNet-9-CIFAR10").input([3, 32, 32])
            .conv2d(64, 3, 3, 1, 1, 1, 1, True, "conv1").batchnorm(1e-5, 0.1, True, "bn1").activation("relu", "relu1")
            .conv2d(128, 3, 3, 1, 1, 1, 1, True, "conv2").batchnorm(1e-5, 0.1, True, "bn2").activation("relu", "relu2")
            .maxpool2d(2, 2, 2, 2, 0, 0, "pool1")
            .basic_residual_block(128, 128, 1, "res_block1").basic_residual_block(128, 128, 1, "res_block2")
            .conv2d(256, 3, 3, 1, 1, 1, 1, True, "conv3").batchnorm(1e-5, 0.1, True, "bn3").activation("relu", "relu3")
            .maxpool2d(2, 2, 2, 2, 0, 0, "pool2")
            .basic_residual_block(256, 256, 1, "res_block3").basic_residual_block(256, 256, 1, "res_block4")
            .conv2d(512, 3, 3, 1, 1, 1, 1, True, "conv4").batchnorm(1e-5, 0.1, True, "bn4").activation("relu", "relu4")
            .maxpool2d(2, 2, 2, 2, 0, 0, "pool3")
            .basic_residual_block(512, 512, 1, "res_block5")
            .avgpool2d(4, 4, 1, 1, 0, 0, "avgpool").flatten("flatten").dense(10, True, "output").build())


def create_resnet18_cifar10() -> Sequential:
    b = (SequentialBuilder("ResNet-18-CIFAR10").input([3, 32, 32])
         .conv2d(64, 3, 3, 1, 1, 1, 1, True, "conv1").batchnorm(1e-5, 0.1, True, "bn1").activation("relu", "relu1")
         .basic_residual_block(64, 64, 1, "layer1_block1").basic_residual_block(64, 64, 1, "layer1_block2")
         .basic_residual_block(64, 128, 2, "layer2_block1").basic_residual_block(128, 128, 1, "layer2_block2")
         .basic_residual_block(128, 128, 1, "layer2_block3")
         .basic_residual_block(128, 256, 2, "layer3_block1").basic_residual_block(256, 256, 1, "layer3_block2")
         .basic_residual_block(256, 256, 1, "layer3_block3")
         .basic_residual_block(256, 512, 2, "layer4_block1").basic_residual_block(512, 512, 1, "layer4_block2"))
    return b.avgpool2d(4, 4, 4, 4, 0, 0, "avgpool").flatten("flatten").dense(10, True, "output").build()


def create_resnet20_cifar10() -> Sequential:
    b = (SequentialBuilder("ResNet-20-CIFAR10").input([3, 32, 32])
         .conv2d(64, 3, 3, 1, 1, 1, 1, True, "conv1").batchnorm(1e-5, 0.1, True, "bn1").activation("relu", "relu1"))
    for i in range(1, 4):
        b.basic_residual_block(64, 64, 1, f"layer1_block{i}")
    b.basic_residual_block(64, 128, 2, "layer2_block1")
    for i in range(2, 4):
        b.basic_residual_block(128, 128, 1, f"layer2_block{i}")
    b.basic_residual_block(128, 256, 2, "layer3_block1")
    for i in range(2, 4):
        b.basic_residual_block(256, 256, 1, f"layer3_block{i}")
    return b.avgpool2d(8, 8, 1, 1, 0, 0, "avgpool").flatten("flatten").dense(10, True, "output").build()


def _resnet50_body(b: SequentialBuilder) -> SequentialBuilder:
    b.bottleneck_residual_block(64, 64, 256, 1, "layer1_block1")
    b.bottleneck_residual_block(256, 64, 256, 1, "layer1_block2")
    b.bottleneck_residual_block(256, 64, 256, 1, "layer1_block3")
    b.bottleneck_residual_block(256, 128, 512, 2, "layer2_block1")
    for i in range(2, 5):
        b.bottleneck_residual_block(512, 128, 512, 1, f"layer2_block{i}")
    b.bottleneck_residual_block(512, 256, 1024, 2, "layer3_block1")
    for i in range(2, 7):
        b.bottleneck_residual_block(1024, 256, 1024, 1, f"layer3_block{i}")
    b.bottleneck_residual_block(1024, 512, 2048, 2, "layer4_block1")
    for i in range(2, 4):
        b.bottleneck_residual_block(2048, 512, 2048, 1, f"layer4_block{i}")
    return b


def create_resnet50_cifar10() -> Sequential:
    b = (SequentialBuilder("ResNet-50-CIFAR10").input([3, 32, 32])
         .conv2d(64, 3, 3, 1, 1, 1, 1, True, "conv1").batchnorm(1e-5, 0.1, True, "bn1").activation("relu", "relu1"))
    return _resnet50_body(b).flatten("flatten").dense(10, True, "fc").build()


def create_resnet9_tiny_imagenet() -> Sequential:
    return (SequentialBuilder("ResNet-9-Tiny-ImageNet").input([3, 64, 64])
            .conv2d(64, 3, 3, 1, 1, 1, 1, False, "conv1").batchnorm(1e-5, 0.1, True, "bn1").activation("relu", "relu1")
            .conv2d(128, 3, 3, 1, 1, 1, 1, False, "conv2").batchnorm(1e-5, 0.1, True, "bn2").activation("relu", "relu2")
            .maxpool2d(2, 2, 2, 2, 0, 0, "pool1").basic_residual_block(128, 128, 1, "res1")
            .conv2d(256, 3, 3, 1, 1, 1, 1, False, "conv3").batchnorm(1e-5, 0.1, True, "bn3").activation("relu", "relu3")
            .maxpool2d(2, 2, 2, 2, 0, 0, "pool2").basic_residual_block(256, 256, 1, "res2")
            .conv2d(512, 3, 3, 1, 1, 1, 1, False, "conv4").batchnorm(1e-5, 0.1, True, "bn4").activation("relu", "relu4")
            .maxpool2d(2, 2, 2, 2, 0, 0, "pool3").basic_residual_block(512, 512, 1, "res3")
            .avgpool2d(4, 4, 1, 1, 0, 0, "avgpool").flatten("flatten").dense(200, True, "fc").build())


def create_cnn_tiny_imagenet() -> Sequential:
    b = _vgg_body(SequentialBuilder("sequential").input([3, 64, 64]))
    return b.dense(1024, True, "fc0").activation("relu", "relu10").dense(200, True, "fc1").build()


def create_resnet18_tiny_imagenet() -> Sequential:
    """Headline model (example_models.hpp:306-331): ~11.3 M params, ~1.08 GFLOP/sample fwd."""
    return (SequentialBuilder("ResNet-18-Tiny-ImageNet").input([3, 64, 64])
            .conv2d(32, 3, 3, 1, 1, 1, 1, False, "conv1").batchnorm(1e-3, 0.1, True, "bn1")
            .activation("relu", "relu1").maxpool2d(2, 2, 2, 2, 0, 0, "maxpool")
            .basic_residual_block(32, 64, 1, "layer1_block1").basic_residual_block(64, 64, 1, "layer1_block2")
            .basic_residual_block(64, 128, 2, "layer2_block1").basic_residual_block(128, 128, 1, "layer2_block2")
            .basic_residual_block(128, 256, 2, "layer3_block1").basic_residual_block(256, 256, 1, "layer3_block2")
            .basic_residual_block(256, 512, 2, "layer4_block1").basic_residual_block(512, 512, 1, "layer4_block2")
            .avgpool2d(4, 4, 1, 1, 0, 0, "avgpool").flatten("flatten").dense(200, True, "fc").build())


def create_resnet34_tiny_imagenet() -> Sequential:
    b = (SequentialBuilder("ResNet-34-Tiny-ImageNet").input([3, 64, 64])
         .conv2d(32, 3, 3, 1, 1, 1, 1, False, "conv1").batchnorm(1e-3, 0.1, True, "bn1")
         .activation("relu", "relu1").maxpool2d(2, 2, 2, 2, 0, 0, "maxpool"))
    b.basic_residual_block(32, 64, 1, "layer1_block1")
    for i in range(2, 4):
        b.basic_residual_block(64, 64, 1, f"layer1_block{i}")
    b.basic_residual_block(64, 128, 2, "layer2_block1")
    for i in range(2, 5):
        b.basic_residual_block(128, 128, 1, f"layer2_block{i}")
    b.basic_residual_block(128, 256, 2, "layer3_block1")
    for i in range(2, 7):
        b.basic_residual_block(256, 256, 1, f"layer3_block{i}")
    b.basic_residual_block(256, 512, 2, "layer4_block1")
    for i in range(2, 4):
        b.basic_residual_block(512, 512, 1, f"layer4_block{i}")
    return b.avgpool2d(4, 4, 1, 1, 0, 0, "avgpool").flatten("flatten").dense(200, True, "fc").build()


def create_resnet50_tiny_imagenet() -> Sequential:
    b = (SequentialBuilder("ResNet-50-Tiny-ImageNet").input([3, 64, 64])
         .conv2d(64, 3, 3, 1, 1, 1, 1, True, "conv1").batchnorm(1e-5, 0.1, True, "bn1")
         .activation("relu", "relu1").maxpool2d(3, 3, 2, 2, 1, 1, "maxpool"))
    return _resnet50_body(b).avgpool2d(4, 4, 1, 1, 0, 0, "avgpool").flatten("flatten").dense(200, True, "fc").build()


def create_resnet50_imagenet() -> Sequential:
    b = (SequentialBuilder("ResNet-50-ImageNet").input([3, 224, 224])
         .conv2d(64, 7, 7, 2, 2, 3, 3, True, "conv1").batchnorm(1e-5, 0.1, True, "bn1")
         .activation("relu", "relu1").maxpool2d(3, 3, 2, 2, 1, 1, "maxpool"))
    return _resnet50_body(b).avgpool2d(7, 7, 1, 1, 0, 0, "avgpool").flatten("flatten").dense(1000, True, "fc").build()


MODELS = {
    "mnist_cnn": create_mnist_trainer,
    "cifar10_cnn_v1": create_cifar10_trainer_v1,
    "cifar10_cnn_v2": create_cifar10_trainer_v2,
    "resnet9_cifar10": create_resnet9_cifar10,
    "resnet18_cifar10": create_resnet18_cifar10,
    "resnet20_cifar10": create_resnet20_cifar10,
    "resnet50_cifar10": create_resnet50_cifar10,
    "resnet9_tiny_imagenet": create_resnet9_tiny_imagenet,
    "cnn_tiny_imagenet": create_cnn_tiny_imagenet,
    "resnet18_tiny_imagenet": create_resnet18_tiny_imagenet,
    "resnet34_tiny_imagenet": create_resnet34_tiny_imagenet,
    "resnet50_tiny_imagenet": create_resnet50_tiny_imagenet,
    "resnet50_imagenet": create_resnet50_imagenet,
}

INPUT_SHAPES = {
    "mnist_cnn": (1, 28, 28), "cifar10_cnn_v1": (3, 32, 32), "cifar10_cnn_v2": (3, 32, 32),
    "resnet9_cifar10": (3, 32, 32), "resnet18_cifar10": (3, 32, 32), "resnet20_cifar10": (3, 32, 32),
    "resnet50_cifar10": (3, 32, 32), "resnet9_tiny_imagenet": (3, 64, 64), "cnn_tiny_imagenet": (3, 64, 64),
    "resnet18_tiny_imagenet": (3, 64, 64), "resnet34_tiny_imagenet": (3, 64, 64),
    "resnet50_tiny_imagenet": (3, 64, 64), "resnet50_imagenet": (3, 224, 224),
}

NUM_CLASSES = {k: (10 if ("cifar" in k or "mnist" in k) else (1000 if k == "resnet50_imagenet" else 200))
               for k in MODELS}


def create_model(name: str) -> Sequential:
    if name not in MODELS:
        raise KeyError(f"unknown model {name!r}; available: {sorted(MODELS)}")
    return MODELS[name]()
