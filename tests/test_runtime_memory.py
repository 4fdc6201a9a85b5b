import torch

from dcnn_amd.runtime.memory import GrowBuffer, MemPool


def test_mempool_reuse_and_borrow():
    p = MemPool("cpu", max_cached=4)
    a = p.get(100)
    p.put(a)
    b = p.get(80)
    assert b.data_ptr() == a.data_ptr() and b.numel() == 80 and p.hits == 1
    p.put(b)
    with p.borrow(50) as t:
        assert t.numel() == 50
    assert p.cached_bytes() == 100 * 4


def test_grow_buffer():
    g = GrowBuffer("cpu")
    x = g.ensure(10)
    y = g.ensure(5)
    assert y.data_ptr() == x.data_ptr() and g.capacity == 10
    g.ensure(20)
    assert g.capacity == 20
