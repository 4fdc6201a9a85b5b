"""HBM-resident data plane (data/device_loader.py, csrc/kernels/augment.hip).

CPU: the op-list translation and the host reference of the counter-based augmentation chain.
GPU: the kernel reproduces the host reference draw for draw on every op (flips, rotation,
brightness, contrast, gaussian noise, random crop, cutout, normalisation), gathers the right
samples and labels, stores decoded-image datasets as uint8, and an epoch visits every sample
once. Reference: include/data_augmentation/augmentation.hpp:114 (the op chain),
include/data_loading/tiny_imagenet_data_loader.hpp:481 (batches of the epoch order)."""
import numpy as np
import pytest
import torch

from dcnn_amd.data import AugmentationBuilder
from dcnn_amd.data.device_loader import aug_uniform, device_ops, reference_augment

ALL_OPS = (AugmentationBuilder().horizontal_flip(0.5).vertical_flip(0.5).rotation(0.5, 15.0).brightness(0.7, 0.2)
           .contrast(0.7, 0.2).gaussian_noise(0.5, 0.05).random_crop(0.8, 4).cutout(0.6, 8))


def test_device_ops_translation():
    st = AugmentationBuilder().horizontal_flip(0.5).random_crop(0.5, 4).normalize().build()
    ops = device_ops(st, 3)
    assert [o[0] for o in ops] == [0, 6, 8]
    assert ops[2][2] == pytest.approx([0.485, 0.456, 0.406, 0.229, 0.224, 0.225])
    one = device_ops(AugmentationBuilder().normalize((0.5,), (0.25,)).build(), 1)
    assert one[0][2] == [0.5, 0.5, 0.5, 0.25, 0.25, 0.25]
    b = AugmentationBuilder()
    for _ in range(13):
        b.horizontal_flip()
    with pytest.raises(ValueError):
        device_ops(b.build(), 3)


def test_reference_chain_semantics():
    g = np.random.default_rng(0)
    img = g.random((3, 8, 8), dtype=np.float32)
    assert np.array_equal(reference_augment(img, 5, [(0, 1.0, [])], 1), img[:, :, ::-1])
    assert np.array_equal(reference_augment(img, 5, [(1, 1.0, [])], 1), img[:, ::-1, :])
    assert np.array_equal(reference_augment(img, 5, [(6, 1.0, [0.0])], 1), img)       # crop, pad 0
    assert np.array_equal(reference_augment(img, 5, [(0, 0.0, [])], 1), img)          # p = 0: skipped
    out = reference_augment(img, 5, [(7, 1.0, [3.0])], 1)                             # cutout 3x3
    assert (out == 0).sum() >= 9 * 3 and np.array_equal(out[out != 0], img[out != 0])
    n = reference_augment(img, 5, [(8, 1.0, [0.5] * 3 + [0.25] * 3)], 1)
    np.testing.assert_allclose(n, (img - 0.5) / 0.25, rtol=1e-6)
    # draws depend on (seed, sample, op, draw) only
    assert aug_uniform(3, 7, 1, 0) == aug_uniform(3, 7, 1, 0) != aug_uniform(3, 8, 1, 0)
    u = np.array([aug_uniform(9, s, 0, 0) for s in range(4000)])
    assert 0 <= u.min() and u.max() < 1 and abs(u.mean() - 0.5) < 0.02


@pytest.mark.gpu
def test_device_augment_matches_host_reference():
    from dcnn_amd.data import DeviceDataLoader
    g = np.random.default_rng(1)
    N, C, H, W = 40, 3, 16, 24
    data = (g.integers(0, 256, (N, C, H, W)) / 255.0).astype(np.float32)
    labels = g.integers(0, 10, N)
    ld = DeviceDataLoader(data=data, labels=labels, num_classes=10, batch_size=16, shuffle=True, seed=4)
    assert ld.storage == "u8"
    st = ALL_OPS.normalize().build()
    ld.set_augmentation(st)
    ops = device_ops(st, C)
    ld.reset()
    order = ld.order.copy()
    seen, k = [], 0
    while True:
        b = ld.get_next_batch()
        if b is None:
            break
        x, y = b
        torch.cuda.synchronize()
        xs, ys = x.cpu().numpy(), y.cpu().numpy()
        for b in range(len(xs)):
            s = int(order[k])
            ref = reference_augment(data[s], s, ops, ld.seed_for_epoch())
            diff = np.abs(xs[b] - ref)
            # (rotation: a floor() at an exact pixel boundary may land on the other side in fp32)
            assert (diff > 1e-4).mean() < 2e-3 and diff.max() < 50, (s, float(diff.max()))
            assert ys[b] == labels[s]
            seen.append(s)
            k += 1
    assert sorted(seen) == list(range(N))


@pytest.mark.gpu
def test_device_loader_plain_gather_and_f32_storage():
    from dcnn_amd.data import DeviceDataLoader
    g = np.random.default_rng(2)
    data = g.standard_normal((33, 1, 28, 28)).astype(np.float32)  # not k / 255: stays fp32
    labels = g.integers(0, 10, 33)
    ld = DeviceDataLoader(data=data, labels=labels, num_classes=10, batch_size=8, drop_last=True, one_hot=True)
    assert ld.storage == "f32" and ld.num_batches() == 4
    batches = list(ld)
    assert len(batches) == 4
    x, y = batches[1]
    assert torch.equal(x.cpu(), torch.from_numpy(data[8:16]))
    assert y.shape == (8, 10, 1, 1) and torch.equal(y.view(8, 10).argmax(1).cpu(), torch.from_numpy(labels[8:16]))


@pytest.mark.gpu
def test_device_loader_reshuffles_every_epoch():
    """The epoch order is reshuffled in place on the host; the device copy must follow it."""
    from dcnn_amd.data import DeviceDataLoader
    n = 24
    data = np.arange(n, dtype=np.float32).reshape(n, 1, 1, 1) * np.ones((1, 1, 2, 2), np.float32) + 0.5
    labels = np.arange(n) % 10
    ld = DeviceDataLoader(data=data, labels=labels, num_classes=10, batch_size=8, shuffle=True, seed=7)
    seen = []
    for _ in range(3):
        xs = [x[:, 0, 0, 0].cpu().numpy() for x, _ in ld]
        got = np.concatenate(xs) - 0.5
        assert sorted(got.tolist()) == list(range(n))  # every sample once
        assert np.array_equal(got, ld.order.astype(np.float32))  # in this epoch's host order
        seen.append(got)
    assert not np.array_equal(seen[0], seen[1]) and not np.array_equal(seen[1], seen[2])
