"""Native dataset parsers, JPEG decoder, augmentation and loader iteration.

The reference's only data test reads the real Tiny-ImageNet from disk; here every
format is exercised on small synthetic fixture files written by the test itself (PIL is used
only to *encode* the JPEG fixtures and as the decode oracle)."""
import io
import os

import numpy as np
import pytest
import torch

from dcnn_amd.data import (AugmentationBuilder, CIFAR10DataLoader, CIFAR100DataLoader, MNISTDataLoader,
                           SyntheticDataLoader, TinyImageNetDataLoader, WiFiDataLoader)
from dcnn_amd.ops._ext import native

nd = native().data


def test_mnist_csv(tmp_path):
    rng = np.random.default_rng(0)
    px = rng.integers(0, 256, (5, 784))
    lab = rng.integers(0, 10, 5)
    p = tmp_path / "train.csv"
    with open(p, "w") as f:
        f.write("label," + ",".join(f"p{i}" for i in range(784)) + "\n")
        for l, row in zip(lab, px):
            f.write(f"{l}," + ",".join(map(str, row)) + "\n")
    ld = MNISTDataLoader(batch_size=2)
    assert ld.load_data(str(p))
    np.testing.assert_array_equal(ld.labels, lab)
    np.testing.assert_allclose(ld.data.reshape(5, -1), px / 255.0, rtol=1e-6)
    assert ld.get_data_shape() == [1, 28, 28]


def test_cifar10_and_100(tmp_path):
    rng = np.random.default_rng(1)
    img = rng.integers(0, 256, (4, 3072), dtype=np.uint8)
    lab = rng.integers(0, 10, 4, dtype=np.uint8)
    p = tmp_path / "b.bin"
    p.write_bytes(b"".join(bytes([l]) + r.tobytes() for l, r in zip(lab, img)))
    ld = CIFAR10DataLoader()
    ld.load_multiple_files([str(p), str(p)])
    assert ld.size() == 8
    np.testing.assert_array_equal(ld.labels[:4], lab)
    np.testing.assert_allclose(ld.data[:4].reshape(4, -1), img / 255.0, rtol=1e-6)
    coarse = rng.integers(0, 20, 4, dtype=np.uint8)
    fine = rng.integers(0, 100, 4, dtype=np.uint8)
    p100 = tmp_path / "c.bin"
    p100.write_bytes(b"".join(bytes([c, f]) + r.tobytes() for c, f, r in zip(coarse, fine, img)))
    f_ld, c_ld = CIFAR100DataLoader(False), CIFAR100DataLoader(True)
    f_ld.load_data(str(p100))
    c_ld.load_data(str(p100))
    np.testing.assert_array_equal(f_ld.labels, fine)
    np.testing.assert_array_equal(c_ld.labels, coarse)
    assert (f_ld.num_classes, c_ld.num_classes) == (100, 20)


def _jpeg(arr, **kw):
    from PIL import Image
    b = io.BytesIO()
    Image.fromarray(arr).save(b, "JPEG", quality=95, **kw)
    return b.getvalue()


@pytest.mark.parametrize("kw", [dict(subsampling=0), dict(subsampling=2), dict(subsampling=1), {"gray": True}])
def test_jpeg_decoder_matches_pil(kw):
    pytest.importorskip("PIL")
    from PIL import Image
    yy, xx = np.mgrid[0:48, 0:40]
    img = np.stack([128 + 90 * np.sin(xx / 6.0), 128 + 90 * np.cos(yy / 7.0), 128 + 50 * np.sin((xx + yy) / 9.0)], -1)
    img = img.astype(np.uint8)
    if kw.get("gray"):
        data = _jpeg(img[..., 0])
    else:
        data = _jpeg(img, **kw)
    ref = np.asarray(Image.open(io.BytesIO(data)).convert("RGB")).astype(int)
    mine = nd.decode_jpeg(data).astype(int)
    assert mine.shape == ref.shape
    assert np.abs(mine - ref).mean() < 1.0 and np.abs(mine - ref).max() <= 4


def test_jpeg_rejects_garbage():
    with pytest.raises(Exception):
        nd.decode_jpeg(b"\xff\xd8\xff\xc2garbage")


def test_tiny_imagenet_directory(tmp_path):
    pytest.importorskip("PIL")
    rng = np.random.default_rng(2)
    root = tmp_path / "tiny"
    wn = ["n001", "n002"]
    (root).mkdir()
    (root / "wnids.txt").write_text("\n".join(wn) + "\n")
    (root / "words.txt").write_text("n001\tcat\nn002\tdog\n")
    imgs = {}
    for w in wn:
        d = root / "train" / w / "images"
        d.mkdir(parents=True)
        for k in range(3):
            a = rng.integers(0, 256, (64, 64, 3), dtype=np.uint8)
            a = (a // 64 * 64 + 32).astype(np.uint8)
            (d / f"{w}_{k}.JPEG").write_bytes(_jpeg(a, subsampling=0))
            imgs[(w, k)] = a
    (root / "val" / "images").mkdir(parents=True)
    (root / "val" / "images" / "val_0.JPEG").write_bytes(_jpeg(imgs[("n002", 0)], subsampling=0))
    (root / "val" / "val_annotations.txt").write_text("val_0.JPEG\tn002\t0\t0\t63\t63\n")
    tr = TinyImageNetDataLoader()
    tr.load_data(str(root), train=True)
    assert tr.size() == 6 and tr.decode_failures == 0
    assert list(tr.labels) == [0, 0, 0, 1, 1, 1]
    assert tr.class_names == {"n001": "cat", "n002": "dog"}
    from PIL import Image
    ref = np.asarray(Image.open(root / "train" / "n002" / "images" / "n002_1.JPEG").convert("RGB"))
    np.testing.assert_allclose(tr.data[4].transpose(1, 2, 0) * 255, ref, atol=3.5)
    va = TinyImageNetDataLoader()
    va.load_data(str(root), train=False, cache=True)
    assert va.size() == 1 and va.labels[0] == 1
    va2 = TinyImageNetDataLoader()
    va2.load_data(str(root), train=False, cache=True)  # from the .npz cache
    np.testing.assert_array_equal(va2.data, va.data)


def test_wifi_csv(tmp_path):
    p = tmp_path / "uji.csv"
    rows = ["a,b,c,x,y", "-50,100,0,1.0,2.0", "-60,-70,-80,3.0,4.0", "bad,-40,-30,5.0,6.0"]
    p.write_text("\n".join(rows) + "\n")
    ld = WiFiDataLoader(True)
    ld.load_data(str(p), 0, 3, 3, 5)
    np.testing.assert_allclose(ld.data, [[-50, -100, -100], [-60, -70, -80], [-100, -40, -30]])
    np.testing.assert_allclose(ld.labels, [[1, 2], [3, 4], [5, 6]])
    ld.normalize_data()
    np.testing.assert_allclose(ld.data.mean(0), 0, atol=1e-5)
    np.testing.assert_allclose(ld.denormalize_targets(ld.labels), [[1, 2], [3, 4], [5, 6]], rtol=1e-5)


def _batch(n=6, c=3, h=8, w=8, seed=0):
    return np.random.default_rng(seed).random((n, c, h, w), dtype=np.float32)


def test_augment_flip_normalize_exact():
    b = _batch()
    s = AugmentationBuilder().horizontal_flip(1.0).vertical_flip(1.0).normalize((0.5, 0.4, 0.3), (0.2, 0.3, 0.4)).build(7)
    out = s.apply(b.copy())
    ref = (b[:, :, ::-1, ::-1] - np.array([0.5, 0.4, 0.3])[None, :, None, None]) / \
        np.array([0.2, 0.3, 0.4])[None, :, None, None]
    np.testing.assert_allclose(out, ref, rtol=1e-5, atol=1e-6)


def test_augment_crop_cutout_semantics():
    b = _batch(4, 1, 10, 10)
    out = AugmentationBuilder().random_crop(1.0, 2).build(3).apply(b.copy())
    for i in range(4):
        # some integer shift in [-2, 2]^2 with zero fill reproduces the output
        ok = False
        for dy in range(-2, 3):
            for dx in range(-2, 3):
                ref = np.zeros_like(b[i, 0])
                for y in range(10):
                    for x in range(10):
                        if 0 <= y + dy < 10 and 0 <= x + dx < 10:
                            ref[y, x] = b[i, 0, y + dy, x + dx]
                ok |= np.array_equal(ref, out[i, 0])
        assert ok
    out = AugmentationBuilder().cutout(1.0, 3).build(1).apply(np.ones((5, 2, 8, 8), np.float32))
    assert all((out[i] == 0).sum() == 2 * 9 for i in range(5))


def test_augment_photometric_ranges_and_determinism():
    b = _batch(16)
    s = AugmentationBuilder().brightness(1.0, 0.2).contrast(1.0, 0.3).gaussian_noise(1.0, 0.05).rotation(1.0, 20).build(5)
    o1 = s.clone().apply(b.copy())
    o2 = s.clone().apply(b.copy())
    np.testing.assert_array_equal(o1, o2)          # same seed -> same result (thread-count independent)
    assert o1.min() >= 0 and o1.max() <= 1
    assert not np.array_equal(o1, b)
    still = AugmentationBuilder().rotation(1.0, 0.0).build(0).apply(b.copy())
    np.testing.assert_allclose(still, b, atol=1e-6)


def test_loader_iteration_shuffle_onehot():
    ld = SyntheticDataLoader(10, (3, 4, 4), 5, seed=1, batch_size=4, shuffle=True, one_hot=True)
    seen = []
    for x, y in ld:
        assert x.shape[1:] == (3, 4, 4) and y.shape[1:] == (5, 1, 1)
        assert torch.all(y.sum(1) == 1)
        seen.append(x.shape[0])
    assert seen == [4, 4, 2]
    ld2 = SyntheticDataLoader(10, (3, 4, 4), 5, seed=1, batch_size=4, drop_last=True)
    assert ld2.num_batches() == 2 and len(list(ld2)) == 2
    # every sample exactly once per epoch
    ld3 = SyntheticDataLoader(9, (1, 2, 2), 3, seed=2, batch_size=4, shuffle=True)
    xs = torch.cat([x for x, _ in ld3]).reshape(9, -1)
    ref = torch.from_numpy(ld3.data.reshape(9, -1))
    assert sorted(map(tuple, xs.tolist())) == sorted(map(tuple, ref.tolist()))
