"""The C++ engine's GPU data path (dcnn/train.hpp DeviceImageDataset, csrc/host/data_gpu.hip): a
synthetic Tiny-ImageNet JPEG directory is decoded by the native decoder into HBM (uint8) and the C++
trainer assembles every batch with one augment_batch launch (crop, flip, normalisation) — in the
timed step with --bench, and through train_model otherwise (the loss must fall).
Reference: include/data_loading/tiny_imagenet_data_loader.hpp:481, include/nn/train.hpp:108-147."""
import json
import os
import re
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "dcnn_amd", "bin", "tiny_imagenet_resnet18")


@pytest.fixture(scope="module")
def tiny_dir(tmp_path_factory):
    sys.path.insert(0, os.path.join(ROOT, "benchmarks"))
    from loader_bench import make_dataset
    d = str(tmp_path_factory.mktemp("tin"))
    make_dataset(d, classes=8, per_class=80, val_per_class=8)
    return d


def _run(args, timeout=300):
    r = subprocess.run([EXE, *args], stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=timeout)
    assert r.returncode == 0, r.stdout[-3000:]
    return r.stdout


def test_cpp_device_data_bench(tiny_dir):
    out = _run(["--device", "GPU", "--data", tiny_dir, "--device-data", "--bench", "--batch", "64", "--steps", "20",
                "--warmup", "3"])
    assert re.search(r"device dataset: 640 images, 7\.9 MB of HBM \(uint8\)", out), out
    d = json.loads([l for l in out.splitlines() if l.startswith("{")][-1])
    assert d["value"] > 0 and d["hipgraph"] and "augment_batch" in d["data"], d


def test_cpp_device_data_trains(tiny_dir):
    out = _run(["--device", "GPU", "--data", tiny_dir, "--device-data", "--epochs", "3", "--batch", "32",
                "--lr", "1e-3"])
    losses = [float(v) for v in re.findall(r"train loss ([0-9.]+)", out)]
    assert len(losses) >= 2 and losses[-1] < losses[0], out[-2000:]
