"""Native per-step activation arena (runtime/arena.py, csrc/kernels/runtime.cpp ActArena).

A ResNet-18 training step on the GPU keeps every activation, statistics slab and workspace in
the native arena: PyTorch's caching allocator stays flat, the native allocator accounts for the
activation bytes, nothing grows after step 2, and the arena path is bit-identical to the
PyTorch-allocator path (eager and captured)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _setup(arena_on, batch=32, seed=5):
    from dcnn_amd.models import zoo
    from dcnn_amd.nn import Adam, LossFactory
    from dcnn_amd.runtime import arena
    from dcnn_amd.runtime.step import TrainStep

    def make_step(*a, **k):
        arena.set_enabled(arena_on)
        try:
            return TrainStep(*a, **k)
        finally:
            arena.set_enabled(True)

    m = zoo.create_model("resnet18_tiny_imagenet")
    m.set_seed(seed)
    m.set_device("GPU:0")
    m.initialize()
    m.set_first_layer_input_grad(False)
    opt = Adam(1e-3)
    opt.attach(m)
    return m, opt, LossFactory.create("softmax_crossentropy"), make_step


def _data(batch, seed=11):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(batch, 3, 64, 64, generator=g).cuda(), torch.randint(0, 200, (batch,), generator=g).cuda()


def test_arena_step_keeps_torch_allocator_flat():
    from dcnn_amd.device import get_gpu
    m, opt, loss_fn, TrainStep = _setup(True)
    st = TrainStep(m, loss_fn, opt, use_graph=False)
    assert st.arena is not None
    x, y = _data(32)
    torch.cuda.synchronize()
    base = torch.cuda.memory_allocated()
    losses, grows, resv = [], [], []
    for k in range(5):
        losses.append(st(x, y))
        torch.cuda.synchronize()
        # only the returned loss / correct scalars (512-byte blocks) may live on PyTorch's allocator
        assert torch.cuda.memory_allocated() - base <= 64 * 1024, (k, torch.cuda.memory_allocated() - base)
        s = st.arena.stats()
        grows.append(s["grows"])
        resv.append(get_gpu(0).allocator_stats()["reservation_grows"])
    s = st.arena.stats()
    assert s["fallbacks"] == 0 and s["chunks"] == 1
    assert grows[1:] == [grows[1]] * 4, grows          # no growth after step 2
    assert resv[2:] == [resv[2]] * 3, resv
    # the arena holds the step's activations: at least the saved conv outputs of a ResNet-18 step
    # (32 images x 64 ch x 32 x 32 x bf16 per stage-1 activation, ~10 of them)
    assert s["high_water_bytes"] > 10 * 32 * 64 * 32 * 32 * 2
    ast = get_gpu(0).allocator_stats()
    assert ast["arena_capacity_bytes"] >= s["high_water_bytes"]
    assert ast["in_use_bytes"] >= ast["arena_capacity_bytes"]
    assert all(torch.isfinite(l).all() for l in losses)


@pytest.mark.parametrize("graph", [False, True])
def test_arena_bit_identical_to_torch_allocator(graph):
    x, y = _data(32)
    res = []
    for on in (True, False):
        m, opt, loss_fn, TrainStep = _setup(on)
        st = TrainStep(m, loss_fn, opt, use_graph=graph)
        assert (st.arena is not None) == on
        losses = [float(st(x, y)) for _ in range(4)]
        torch.cuda.synchronize()
        res.append((losses, m.arena.data.clone(), m.arena.grad.clone()))
        if on and graph:
            s = st.arena.stats()
            assert s["fallbacks"] == 0 and st._pins
    (la, pa, ga), (lb, pb, gb) = res
    assert la == lb
    assert torch.equal(pa, pb) and torch.equal(ga, gb)
