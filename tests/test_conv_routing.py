"""Conv algorithm routing rules of ops/hip.py (`_hconv_ok`), checked on the CPU with the kernel
library's shape query stubbed: which convs go to the halo kernel (hconv / hconv3) instead of the
gathered GEMM or the streaming 1x1 kernel."""
import pytest

from dcnn_amd.ops import fusion, hip


class _Stub:
    def hconv_supported(self, *args):
        return True


@pytest.fixture
def stub(monkeypatch):
    monkeypatch.setattr(hip, "kernels", lambda: _Stub())
    monkeypatch.setattr(fusion, "HCONV_1X1", True)


TAP1 = [(0, 0, 0, 0)]
TAPS9 = [(dy, dx, 0, 0) for dy in (-1, 0, 1) for dx in (-1, 0, 1)]


def test_3x3_same_stride1(stub):
    assert hip._hconv_ok(256, 32, 32, 32, 32, 1, 1, 64, 64, TAPS9, None)
    assert not hip._hconv_ok(256, 16, 16, 32, 32, 2, 2, 64, 128, TAPS9, None)  # strided
    # a tap two pixels away (5x5 reach) or more than 9 taps: not a halo-1 conv
    assert not hip._hconv_ok(256, 32, 32, 32, 32, 1, 1, 64, 64, [(2, 0, 0, 0), (0, 0, 0, 0)], None)
    assert not hip._hconv_ok(256, 32, 32, 32, 32, 1, 1, 64, 64, TAPS9 + [(0, 0, 0, 0)], None)


def test_1x1_only_k1024_small_grid(stub):
    # ResNet-50 batch 32: layer-3 reduce (1024 -> 256 at 8x8: 128 GEMM tiles) -> halo kernel
    assert hip._hconv_ok(32, 8, 8, 8, 8, 1, 1, 1024, 256, TAP1, None)
    assert hip._hconv_ok(32, 4, 4, 4, 4, 1, 1, 2048, 512, TAP1, None)
    # batch 256: 1024 tiles, the GEMM grid fills the chip
    assert not hip._hconv_ok(256, 8, 8, 8, 8, 1, 1, 1024, 256, TAP1, None)
    # K <= 512 1x1 convs belong to the streaming kernel / plain GEMM
    assert not hip._hconv_ok(32, 8, 8, 8, 8, 1, 1, 512, 256, TAP1, None)


def test_1x1_switch_off(stub, monkeypatch):
    monkeypatch.setattr(fusion, "HCONV_1X1", False)
    assert not hip._hconv_ok(32, 8, 8, 8, 8, 1, 1, 1024, 256, TAP1, None)


def test_1x1_split3_concat_stays_exact(stub):
    # fp32 concat callers pass Cs = 3 x Ci: a 384-channel fp32 1x1 conv (Cs = 1152) must not
    # leave the exact fp32 GEMM for the 3 x bf16 halo kernel (the K >= 1024 rule is bf16-only)
    assert not hip._hconv_ok(32, 8, 8, 8, 8, 1, 1, 3 * 384, 256, TAP1, None, True)
    assert not hip._hconv_ok(32, 4, 4, 4, 4, 1, 1, 3 * 2048, 512, TAP1, None, True)
    # 3x3 convs still take the split-precision halo path
    assert hip._hconv_ok(256, 32, 32, 32, 32, 1, 1, 3 * 64, 64, TAPS9, None, True)


def test_shared_route_table():
    """The kernel library's routing table (csrc/kernels/conv_route.cpp), which both the Python
    front end and the C++ host API's GPU backend ask: ResNet layer shapes land on the intended
    kernel families (host-side query, no GPU needed)."""
    from dcnn_amd.ops._ext import kernels
    K = kernels()

    def fwd(N, C, H, W, Co, k, s, p, mode=0):
        OH, OW = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
        return K.conv_fwd_route(N, C, H, W, Co, k, k, s, s, p, p, OH, OW, mode)

    assert fwd(256, 64, 32, 32, 64, 3, 1, 1) == K.ROUTE_HALO          # layer-1 3x3
    assert fwd(256, 256, 8, 8, 256, 3, 1, 1) == K.ROUTE_HALO          # 8x8 maps (gutter layout)
    assert fwd(256, 128, 16, 16, 256, 3, 2, 1) == K.ROUTE_GEMM_G2     # strided 3x3
    assert fwd(256, 64, 32, 32, 128, 1, 2, 0) == K.ROUTE_G1S          # strided 1x1 projection
    # K >= 1024 1x1, small grid: gemm_g2 split-K (default), the halo kernel's split-K without it
    prev = K.gemm_g2_splitk_enabled()
    try:
        K.gemm_g2_set_splitk(1)
        assert fwd(32, 1024, 8, 8, 256, 1, 1, 0) == K.ROUTE_GEMM_G2
        assert K.conv_dgrad_route(32, 256, 8, 8, 1024, 1, 1, 1, 1, 0, 0, 8, 8, 0) == K.ROUTE_GEMM_G2
        K.gemm_g2_set_splitk(0)
        assert fwd(32, 1024, 8, 8, 256, 1, 1, 0) == K.ROUTE_HALO
    finally:
        K.gemm_g2_set_splitk(prev)
    assert fwd(256, 1024, 8, 8, 256, 1, 1, 0) == K.ROUTE_GEMM_G2      # ... large grid
    assert fwd(8, 3, 32, 32, 16, 3, 1, 1) == K.ROUTE_GENERIC          # odd channel count
    assert fwd(256, 64, 32, 32, 256, 1, 1, 0, -1) != K.ROUTE_G1S      # epilogue not on g1s
    assert K.conv_dgrad_route(256, 64, 32, 32, 64, 3, 3, 1, 1, 1, 1, 32, 32, 2) == K.ROUTE_HALO
    assert K.conv_dgrad_route(256, 64, 32, 32, 256, 1, 1, 1, 1, 0, 0, 32, 32, 0) == K.ROUTE_G1S
    assert K.conv_wgrad_route(256, 64, 32, 32, 64, 3, 3, 1, 1, 1, 1, 32, 32, -1) == K.ROUTE_HALO
    assert K.conv_wgrad_route(256, 64, 32, 32, 128, 3, 3, 2, 2, 1, 1, 16, 16, -1) == K.ROUTE_HALO_S2  # stride-2 halo
    assert K.conv_wgrad_route(256, 64, 32, 32, 128, 1, 1, 2, 2, 0, 0, 16, 16, -1) == K.ROUTE_GEMM_G2  # strided 1x1
