#!/usr/bin/env python3
"""Pipeline stage worker CLI (reference examples/network_worker.cpp):

    python examples/network_worker.py 8001 [--gpu] [--num-threads N] [--ecore] [--show-cores]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dcnn_amd.parallel.pipeline.worker import main  # noqa: E402

sys.exit(main())
