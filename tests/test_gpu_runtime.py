"""Native HIP device runtime (csrc/kernels/runtime.cpp via dcnn_amd.device): flows, tasks,
pool allocator reuse, DLPack buffers, async copies, and the training step's allocation steady state."""
import pytest
import torch

from dcnn_amd.device import create_task, get_gpu

pytestmark = pytest.mark.gpu


def test_device_properties_and_memory():
    g = get_gpu(0)
    p = g.properties()
    assert p["arch"].startswith("gfx950") and p["multiprocessors"] > 0 and p["warp_size"] == 64
    assert g.get_total_memory() > g.get_available_memory() > 0
    assert g.name()


def test_flow_task_ordering_and_timing():
    g = get_gpu(0)
    flow = g.get_flow("worker", )
    x = torch.randn(1 << 22, device="cuda")
    flow.wait(create_task(g, "default"))    # the worker flow reads x: order it after x's producer
    t0 = create_task(g, "worker", timing=True)
    with torch.cuda.stream(flow.stream):
        y = x * 2 + 1
    t1 = create_task(g, "worker", timing=True)
    g.get_flow("default").wait(t1)          # the compute stream waits for the worker flow only
    z = y.sum()
    t1.sync()
    assert t1.is_ready() and t0.elapsed_ms(t1) >= 0.0
    torch.testing.assert_close(z, (x * 2 + 1).sum())


def test_allocator_reuse_and_dlpack_buffers():
    g = get_gpu(0)
    a = g.allocate((1024, 256), torch.float32, zero=True)
    assert a.is_cuda and a.shape == (1024, 256) and float(a.abs().sum()) == 0.0
    a += 3
    assert float(a.mean()) == 3.0
    b = g.allocate(4096, torch.bfloat16)
    assert b.dtype == torch.bfloat16
    del a, b
    torch.cuda.synchronize()
    s0 = g.allocator_stats()
    for _ in range(20):  # same sizes, stream-ordered frees: served from the pool's cache
        t = g.allocate((1024, 256), torch.float32)
        t.fill_(1.0)
        del t
    torch.cuda.synchronize()
    s1 = g.allocator_stats()
    assert s1["allocations"] - s0["allocations"] == 20
    assert s1["reservation_grows"] - s0["reservation_grows"] <= 1, (s0, s1)


def test_async_copies():
    g = get_gpu(0)
    src = torch.arange(1 << 16, dtype=torch.float32).pin_memory()
    dst = g.allocate(1 << 16, torch.float32)
    g.copy_to_device(dst, src)                       # H2D on the default flow
    back = torch.empty(1 << 16).pin_memory()
    g.copy_to_device(back, dst)                      # D2H
    g.get_flow("default").synchronize()
    assert torch.equal(back, src)


def test_training_step_allocation_steady_state():
    """A hipGraph training step: the arenas/optimizer moments come from the native pool once at
    setup; over steady-state steps neither the native pool nor PyTorch's caching allocator
    reserves new memory (no per-step hipMalloc)."""
    from dcnn_amd.models import zoo
    from dcnn_amd.nn import Adam, LossFactory
    from dcnn_amd.runtime.step import TrainStep
    g = get_gpu(0)
    m = zoo.create_model("resnet9_cifar10")
    m.set_seed(1)
    m.set_device("GPU:0")
    m.initialize()
    m.set_first_layer_input_grad(False)
    opt = Adam(1e-3)
    opt.attach(m)
    step = TrainStep(m, LossFactory.create("softmax_crossentropy"), opt, use_graph=True)
    x = torch.randn(64, 3, 32, 32, device="cuda")
    y = torch.randint(0, 10, (64,), device="cuda")
    for _ in range(3):
        step(x, y)
    torch.cuda.synchronize()
    s0, t0 = g.allocator_stats(), torch.cuda.memory_stats()
    for _ in range(10):
        step(x, y)
    torch.cuda.synchronize()
    s1, t1 = g.allocator_stats(), torch.cuda.memory_stats()
    assert s1["reservation_grows"] == s0["reservation_grows"] and s1["allocations"] == s0["allocations"]
    assert t1["segment.all.allocated"] == t0["segment.all.allocated"]
    assert t1["reserved_bytes.all.current"] == t0["reserved_bytes.all.current"]
    assert s1["in_use_bytes"] >= 3 * m.arena.numel * 4  # data + grad + Adam moments live in the pool


def test_zero_fill_replays_in_graph():
    """hip.zero_ inside a captured graph zeroes on EVERY replay (a captured hipMemsetAsync node
    did not on ROCm 7.2: garbage from the second replay on)."""
    from dcnn_amd.ops import hip
    for n in (1000, 11_300_000):
        t = get_gpu(0).allocate(n, torch.float32)
        s = torch.cuda.Stream()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            hip.zero_(t)
        for _ in range(3):
            t.fill_(1.0)
            g.replay()
            torch.cuda.synchronize()
            assert float(t.abs().sum()) == 0.0
