"""Layer registry: LayerFactory (type string -> layer) and LayerBuilder (shape-inferring list
builder). Reference: `include/nn/layers.hpp:50-483`.
"""
from __future__ import annotations

from typing import Callable, Dict, List, Optional

from .base import Layer, LayerConfig, ParameterizedLayer, StatelessLayer
from .conv import Conv2D, Dense
from .misc import Activation, AvgPool2D, Dropout, Flatten, MaxPool2D
from .norm import BatchNorm, GroupNorm
from .residual import ResidualBlock, plan_fusion


class LayerFactory:
    _creators: Dict[str, Callable[[LayerConfig], Layer]] = {}

    @classmethod
    def register_layer(cls, type_name: str, creator: Callable[[LayerConfig], Layer]) -> None:
        cls._creators[type_name] = creator

    @classmethod
    def register_defaults(cls) -> None:
        for L in (Dense, Conv2D, Activation, MaxPool2D, AvgPool2D, Dropout, BatchNorm, GroupNorm, Flatten,
                  ResidualBlock):
            cls.register_layer(L.type_name, L.from_config)

    @classmethod
    def create(cls, type_name: str, config) -> Layer:
        if not cls._creators:
            cls.register_defaults()
        if type_name not in cls._creators:
            raise ValueError(f"Unknown layer type: {type_name}")
        if not isinstance(config, LayerConfig):
            config = LayerConfig(config.get("name", ""), config.get("parameters", {}), type_name)
        return cls._creators[type_name](config)

    @classmethod
    def available_types(cls) -> List[str]:
        if not cls._creators:
            cls.register_defaults()
        return list(cls._creators)


LayerFactory.register_defaults()


def create_layer(type_name: str, config) -> Layer:
    return LayerFactory.create(type_name, config)


class LayerBuilder:
    """Builds a list of layers, inferring input channels / features from the running shape."""

    def __init__(self, name: str = "Block"):
        self.name = name
        self.layers: List[Layer] = []
        self.input_shape: Optional[List[int]] = None  # (C, H, W) without batch

    def input(self, shape) -> "LayerBuilder":
        self.input_shape = list(shape)
        return self

    def is_input_shape_set(self) -> bool:
        return self.input_shape is not None

    def get_current_shape(self) -> List[int]:
        if self.input_shape is None:
            raise RuntimeError("Input shape must be set before adding layers (use .input())")
        s = [1] + list(self.input_shape)
        for l in self.layers:
            s = l.compute_output_shape(s)
        return s

    def _auto(self, name, prefix):
        return name if name else f"{prefix}_{len(self.layers)}"

    def add_layer(self, layer: Layer) -> "LayerBuilder":
        self.layers.append(layer)
        return self

    def dense(self, output_features, use_bias=True, name=""):
        s = self.get_current_shape()
        feat = 1
        for d in s[1:]:
            feat *= d
        return self.add_layer(Dense(feat, output_features, use_bias, self._auto(name, "dense")))

    def conv2d(self, out_channels, kernel_h, kernel_w, stride_h=1, stride_w=1, pad_h=0, pad_w=0, use_bias=True,
               name=""):
        s = self.get_current_shape()
        return self.add_layer(Conv2D(s[1], out_channels, kernel_h, kernel_w, stride_h, stride_w, pad_h, pad_w,
                                     use_bias, self._auto(name, "conv2d")))

    def batchnorm(self, epsilon=1e-5, momentum=0.1, affine=True, name=""):
        s = self.get_current_shape()
        return self.add_layer(BatchNorm(s[1], epsilon, momentum, affine, self._auto(name, "batchnorm")))

    def groupnorm(self, num_groups, epsilon=1e-5, affine=True, name=""):
        s = self.get_current_shape()
        return self.add_layer(GroupNorm(int(num_groups), s[1], epsilon, affine, self._auto(name, "groupnorm")))

    def activation(self, activation_name, name=""):
        return self.add_layer(Activation(activation_name, self._auto(name, "activation")))

    def maxpool2d(self, pool_h, pool_w, stride_h=0, stride_w=0, pad_h=0, pad_w=0, name=""):
        return self.add_layer(MaxPool2D(pool_h, pool_w, stride_h, stride_w, pad_h, pad_w,
                                        self._auto(name, "maxpool2d")))

    def avgpool2d(self, pool_h, pool_w, stride_h=1, stride_w=1, pad_h=0, pad_w=0, name=""):
        return self.add_layer(AvgPool2D(pool_h, pool_w, stride_h, stride_w, pad_h, pad_w,
                                        self._auto(name, "avgpool2d")))

    def dropout(self, dropout_rate, name=""):
        return self.add_layer(Dropout(dropout_rate, self._auto(name, "dropout")))

    def flatten(self, name=""):
        return self.add_layer(Flatten(self._auto(name, "flatten")))

    def build(self) -> List[Layer]:
        out, self.layers = self.layers, []
        return out


def residual_block(main_path, shortcut_path, activation="relu", name="residual_block") -> ResidualBlock:
    return ResidualBlock(main_path, shortcut_path, activation, name)


__all__ = ["Layer", "LayerConfig", "ParameterizedLayer", "StatelessLayer", "Conv2D", "Dense", "BatchNorm",
           "GroupNorm", "MaxPool2D", "AvgPool2D", "Dropout", "Flatten", "Activation", "ResidualBlock",
           "LayerFactory", "LayerBuilder", "create_layer", "residual_block", "plan_fusion"]
