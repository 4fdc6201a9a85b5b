"""Pipeline stages on the GPU (bf16 HIP kernels): in-process coordinator with stages sharing
cuda:0 (the one-GPU box); the multi-GPU RCCL path is covered on CPU by test_pipeline.py."""
import pytest
import torch

from dcnn_amd.models import zoo
from dcnn_amd.nn.optimizers import Adam
from dcnn_amd.parallel.pipeline import FlopPartitioner, InProcessCoordinator

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("schedule", ["sync", "semi_async"])
def test_gpu_pipeline_trains(schedule):
    model = zoo.create_model("resnet18_tiny_imagenet")
    coord = InProcessCoordinator(model, Adam(1e-3), "softmax_crossentropy", num_stages=2, num_microbatches=4,
                                 partitioner=FlopPartitioner([8, 3, 64, 64]), device="GPU:0",
                                 stage_devices=["GPU:0", "GPU:0"], seed=11)
    try:
        coord.initialize()
        coord.deploy_stages()
        coord.start()
        g = torch.Generator().manual_seed(0)
        x = torch.randn(32, 3, 64, 64, generator=g).cuda()
        y = torch.randint(0, 200, (32,), generator=g).cuda()
        losses = [coord.train_step(x, y, schedule) for _ in range(8)]
        assert all(l == l for l in losses)
        assert losses[-1] < losses[0]
        st = coord.status()
        assert all(s["device"].startswith("cuda") for s in st)
    finally:
        coord.stop()


def _pipeline_run(use_graph, schedule, steps=4, stages=2, mbs=4):
    model = zoo.create_model("resnet18_tiny_imagenet")
    coord = InProcessCoordinator(model, Adam(1e-3), "softmax_crossentropy", num_stages=stages, num_microbatches=mbs,
                                 partitioner=FlopPartitioner([8, 3, 64, 64]), device="GPU:0",
                                 stage_devices=["GPU:0"] * stages, seed=11, use_graph=use_graph)
    try:
        coord.initialize()
        coord.deploy_stages()
        coord.start()
        g = torch.Generator().manual_seed(0)
        x = torch.randn(32, 3, 64, 64, generator=g).cuda()
        y = torch.randint(0, 200, (32,), generator=g).cuda()
        losses = [coord.train_step(x, y, schedule) for _ in range(steps)]
        params = coord.collect_parameters()
        st = coord.status()
        return losses, params, st
    finally:
        coord.stop()


@pytest.mark.parametrize("schedule", ["sync", "semi_async", "1f1b"])
def test_gpu_pipeline_graph_matches_eager(schedule):
    """Stages replaying per-micro-batch hipGraphs (from step 2 on) train exactly like eager stages:
    sync (fixed accumulation order) bit-for-bit, semi-async up to the gradient-accumulation order."""
    le, pe, _ = _pipeline_run(False, schedule)
    lg, pg, st = _pipeline_run(True, schedule)
    assert all(s["graphs"]["replays"] > 0 for s in st), st
    if schedule in ("sync", "1f1b"):
        assert le == lg
        for a, b in zip(pe, pg):
            assert torch.equal(a, b)
    else:
        for a, b in zip(le, lg):
            assert abs(a - b) <= 1e-3 * abs(a) + 1e-4
        for a, b in zip(pe, pg):
            assert torch.allclose(a, b, rtol=1e-3, atol=1e-4)
