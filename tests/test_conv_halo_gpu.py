"""Halo-tiled direct 3x3 convolution (csrc/kernels/conv_halo.hip) vs the fp32 reference.

Every configuration of the family on geometries that exercise its tile shapes: row bands of one
image (th < P), whole-image tiles with several images (ni > 1) and a partial last tile, one and
several 64-channel input chunks (single vs double-buffered halo), the residual + BN-statistics
epilogue and the fused BN-backward epilogue of a data gradient. Inputs are rounded to bf16 once;
the reference runs in fp32."""
import ctypes

import pytest
import torch

from distributed_resnet_tensorflow_amd.ops.backend import ConvGeom

pytestmark = pytest.mark.gpu

HALO_CASES = [
    # N, H, C, K
    (2, 12, 64, 64),      # 1 chunk, row bands (12x12 = 144 px: whole image fits 224/256, ni = 1..)
    (3, 14, 128, 128),    # 2 chunks, whole images, partial last tile for ni > 1
    (2, 28, 64, 128),     # row bands of 28-px rows (th = 7 / 8 / 4 ...)
    (5, 7, 256, 256),     # 4 chunks, 7x7 images, ni = 4 with 5 images: partial last tile
    (1, 20, 192, 64),     # 3 chunks (odd), th = 10 / 5 ..
]


BC = {0: 128, 1: 64, 2: 64, 3: 256, 4: 128, 5: 64}  # output channels per tile of each configuration


def _rel(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return (a - b).norm().item() / max(b.norm().item(), 1e-12)


@pytest.mark.parametrize("case", HALO_CASES)
@pytest.mark.parametrize("cfg", range(6))
def test_conv_halo_fwd(hip, ref, case, cfg):
    N, H, C, K = case
    torch.manual_seed(100 + cfg)
    x = torch.randn(N, H, H, C).bfloat16()
    w = (torch.randn(K, 3, 3, C) * (2.0 / (9 * C)) ** 0.5).bfloat16()
    res = torch.randn(N, H, H, K).bfloat16()
    g = ConvGeom(stride=1, pad_h=1, pad_w=1)
    y_ref = torch.zeros(N, H, H, K)
    st_ref = torch.zeros(2 * K)
    ref.conv_fwd(x.float(), w.float(), y_ref, g, residual=res.float(), stats=st_ref)
    y = torch.zeros(N, H, H, K, dtype=torch.bfloat16, device="cuda")
    st = torch.zeros(3, 2, K, device="cuda")
    a = hip.conv_args(x.cuda(), w.cuda(), y, g, residual=res.cuda(), stats=st)
    assert hip.L.drn_conv_halo_ok(ctypes.byref(a)) == 1
    a.cfg = hip.L.drn_conv_halo_cfg0() + cfg
    rc = hip.L.drn_conv_fwd2(ctypes.byref(a), hip.zero_page.data_ptr(), hip.stream())
    if rc != 0:  # the configuration's channel tile does not divide K (or its 256-wide tile exceeds the LDS)
        assert K % BC[cfg] != 0 or cfg == 3, (cfg, rc)
        return
    torch.cuda.synchronize()
    assert _rel(y, y_ref) < 1e-2, cfg
    s = st.sum(0).view(-1).cpu()
    assert _rel(s[:K], st_ref[:K]) < 2e-2 and _rel(s[K:], st_ref[K:]) < 2e-2


@pytest.mark.parametrize("cfg", range(6))
def test_conv_halo_dgrad_fused_bn_backward(hip, ref, cfg):
    """Data-gradient mode: the epilogue masks by the forward ReLU of bn(bn_x) and accumulates
    sum g and sum g * xhat (the fused BN-backward reduction)."""
    N, H, C, K = 2, 14, 128, 128
    torch.manual_seed(7 + cfg)
    dy = torch.randn(N, H, H, C).bfloat16()
    w = (torch.randn(K, 3, 3, C) * (2.0 / (9 * C)) ** 0.5).bfloat16()
    bx = torch.randn(N, H, H, K).bfloat16()
    sc, sh = torch.rand(K) + 0.5, torch.randn(K) * 0.3
    mu, isd = torch.randn(K) * 0.1, torch.rand(K) + 0.5
    g = ConvGeom(stride=1, pad_h=1, pad_w=1)
    y_ref = torch.zeros(N, H, H, K)
    st_ref = torch.zeros(2 * K)
    ref.conv_fwd(dy.float(), w.float(), y_ref, g, stats=st_ref, bn_bwd=(bx.float(), sc, sh, mu, isd))
    y = torch.zeros(N, H, H, K, dtype=torch.bfloat16, device="cuda")
    st = torch.zeros(2, 2, K, device="cuda")
    a = hip.conv_args(dy.cuda(), w.cuda(), y, g, stats=st,
                      bn_bwd=(bx.cuda(), sc.cuda(), sh.cuda(), mu.cuda(), isd.cuda()))
    a.cfg = hip.L.drn_conv_halo_cfg0() + cfg
    rc = hip.L.drn_conv_fwd2(ctypes.byref(a), hip.zero_page.data_ptr(), hip.stream())
    if rc != 0:
        assert cfg == 3, rc  # 256-channel tile: K = 128 does not divide
        return
    torch.cuda.synchronize()
    assert _rel(y, y_ref) < 1e-2
    s = st.sum(0).view(-1).cpu()
    assert _rel(s[:K], st_ref[:K]) < 2e-2 and _rel(s[K:], st_ref[K:]) < 3e-2


def test_conv_halo_rejects_unsupported(hip):
    """Stride 2, a fused BN prologue and C % 64 != 0 stay on the implicit-GEMM kernels."""
    for (C, s, pro) in ((64, 2, False), (64, 1, True), (96, 1, False)):
        H = 9
        P = H if s == 1 else (H - 1) // 2 + 1
        x = torch.zeros(2, H, H, C, dtype=torch.bfloat16, device="cuda")
        w = torch.zeros(64, 3, 3, C, dtype=torch.bfloat16, device="cuda")
        y = torch.zeros(2, P, P, 64, dtype=torch.bfloat16, device="cuda")
        in_bn = (torch.ones(C, device="cuda"), torch.zeros(C, device="cuda")) if pro else None
        a = hip.conv_args(x, w, y, ConvGeom(stride=s, pad_h=1, pad_w=1), in_bn=in_bn)
        assert hip.L.drn_conv_halo_ok(ctypes.byref(a)) == 0
        a.cfg = hip.L.drn_conv_halo_cfg0()
        assert hip.L.drn_conv_fwd2(ctypes.byref(a), hip.zero_page.data_ptr(), hip.stream()) != 0
