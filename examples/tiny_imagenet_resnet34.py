#!/usr/bin/env python3
"""Alias of tiny_imagenet_resnet.py --depth 34 (reference examples/tiny_imagenet_resnet34.cpp)."""
import os
import runpy
import sys

sys.argv += ["--depth", "34"]
runpy.run_path(os.path.join(os.path.dirname(os.path.abspath(__file__)), "tiny_imagenet_resnet.py"), run_name="__main__")
