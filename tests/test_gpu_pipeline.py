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
