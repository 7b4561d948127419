"""Halo-tiled direct 3x3 convolution (csrc/kernels/conv_halo.hip) vs the fp32 reference.

Every configuration of the family on geometries that exercise its tile shapes: row bands of one
image (th < P) and whole images, rows cut into several 16-pixel fragments with garbage columns
past the row end (Q = 20, 28, 7), one and several 64-channel input chunks (single vs
double-buffered halo), the residual + BN-statistics epilogue and the fused BN-backward epilogue
of a data gradient. Inputs are rounded to bf16 once;
the reference runs in fp32."""
import ctypes

import pytest
import torch

from distributed_resnet_tensorflow_amd.ops.backend import ConvGeom

pytestmark = pytest.mark.gpu

HALO_CASES = [
    # N, H, C, K
    (2, 12, 64, 64),      # 1 chunk, 12-px rows: one fragment per row, 4 garbage columns
    (3, 14, 128, 128),    # 2 chunks, whole 14x14 images (th = 14) or 7-row bands
    (2, 28, 64, 128),     # two fragments per 28-px row
    (5, 7, 256, 256),     # 4 chunks, 7x7 images: 9 garbage columns per row
    (1, 20, 192, 64),     # 3 chunks (odd), 20-px rows, th = 5 / 10
]


BC = {0: 128, 1: 64, 2: 64, 3: 128, 4: 128, 5: 64}  # output channels per tile of each configuration


def _rel(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return (a - b).norm().item() / max(b.norm().item(), 1e-12)


@pytest.mark.parametrize("case", HALO_CASES)
@pytest.mark.parametrize("cfg", range(6))
@pytest.mark.parametrize("pro", [False, True])
def test_conv_halo_fwd(hip, ref, case, cfg, pro):
    """pro: the input is the raw pre-BN tensor and the kernel applies relu(x * scale + shift) to
    the staged halo (zero padding must stay zero, not relu(shift))."""
    N, H, C, K = case
    torch.manual_seed(100 + cfg)
    x = torch.randn(N, H, H, C).bfloat16()
    w = (torch.randn(K, 3, 3, C) * (2.0 / (9 * C)) ** 0.5).bfloat16()
    res = torch.randn(N, H, H, K).bfloat16()
    g = ConvGeom(stride=1, pad_h=1, pad_w=1)
    in_bn = (torch.rand(C) + 0.5, torch.randn(C) * 0.5 + 0.3) if pro else None
    y_ref = torch.zeros(N, H, H, K)
    st_ref = torch.zeros(2 * K)
    ref.conv_fwd(x.float(), w.float(), y_ref, g, in_bn=in_bn, residual=res.float(), stats=st_ref)
    y = torch.zeros(N, H, H, K, dtype=torch.bfloat16, device="cuda")
    st = torch.zeros(3, 2, K, device="cuda")
    a = hip.conv_args(x.cuda(), w.cuda(), y, g, residual=res.cuda(), stats=st,
                      in_bn=None if in_bn is None else (in_bn[0].cuda(), in_bn[1].cuda()))
    assert hip.L.drn_conv_halo_ok(ctypes.byref(a)) == 1
    a.cfg = hip.L.drn_conv_halo_cfg0() + cfg
    rc = hip.L.drn_conv_fwd2(ctypes.byref(a), hip.zero_page.data_ptr(), hip.stream())
    if rc != 0:  # the configuration's channel tile does not divide K, or its tile's halo needs > 8
        assert K % BC[cfg] != 0 or (cfg == 2 and H > 20), (cfg, rc)  # pieces per wave (448 px at W >= 28)
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
    assert rc == 0, (cfg, rc)
    torch.cuda.synchronize()
    assert _rel(y, y_ref) < 1e-2
    s = st.sum(0).view(-1).cpu()
    assert _rel(s[:K], st_ref[:K]) < 2e-2 and _rel(s[K:], st_ref[K:]) < 3e-2


@pytest.mark.parametrize("publish", [False, True])
def test_conv_halo_prologue_finalize(hip, publish):
    """Consumer-side BN finalize in the halo kernel's prologue: equal to the same conv reading
    separately finalized scale / shift; only a publishing launch writes them out."""
    from distributed_resnet_tensorflow_amd.ops.backend import BnCfin
    torch.manual_seed(3)
    N, H, C, K = 2, 14, 128, 128
    x = (torch.randn(N, H, H, C) + 0.2).bfloat16().cuda()
    w = (torch.randn(K, 3, 3, C) * 0.05).bfloat16().cuda()
    gamma, beta = (torch.rand(C) + 0.5).cuda(), (torch.randn(C) * 0.2).cuda()
    xf = x.float().reshape(-1, C)
    st = (torch.stack([xf.sum(0), (xf * xf).sum(0)]).unsqueeze(0) / 4).repeat(4, 1, 1).contiguous()
    sc0, sh0, mu0, is0 = (torch.zeros(C, device="cuda") for _ in range(4))
    hip.bn_finalize(st, 4, xf.shape[0], gamma, beta, None, None, sc0, sh0, mu0, is0, 0.997, 1e-5, update_running=False)
    g = ConvGeom(1, 1, 1)
    want = torch.empty(N, H, H, K, dtype=torch.bfloat16, device="cuda")
    a = hip.conv_args(x, w, want, g, in_bn=(sc0, sh0))
    a.cfg = hip.L.drn_conv_halo_cfg0()
    assert hip.L.drn_conv_fwd2(ctypes.byref(a), hip.zero_page.data_ptr(), hip.stream()) == 0
    sc, sh, mu, isd = (torch.full((C,), 7.0, device="cuda") for _ in range(4))
    fin = BnCfin(st, float(xf.shape[0]), gamma, beta=beta, scale=sc, shift=sh, mean=mu, invstd=isd, publish=publish)
    got = torch.empty_like(want)
    a = hip.conv_args(x, w, got, g, in_bn=(sc, sh), in_fin=fin)
    a.cfg = hip.L.drn_conv_halo_cfg0()
    assert hip.L.drn_conv_fwd2(ctypes.byref(a), hip.zero_page.data_ptr(), hip.stream()) == 0
    torch.cuda.synchronize()
    assert _rel(got, want) < 1e-2
    if publish:
        assert _rel(sc, sc0) < 1e-5 and _rel(sh, sh0) < 1e-4 and _rel(isd, is0) < 1e-5
    else:
        assert bool((sc == 7.0).all())


def test_conv_halo_rejects_unsupported(hip):
    """Stride 2, C % 64 != 0 and a BN prologue without ReLU stay on the implicit-GEMM kernels."""
    for (C, s, pro) in ((64, 2, False), (96, 1, False), (64, 1, True)):
        H = 9
        P = H if s == 1 else (H - 1) // 2 + 1
        x = torch.zeros(2, H, H, C, dtype=torch.bfloat16, device="cuda")
        w = torch.zeros(64, 3, 3, C, dtype=torch.bfloat16, device="cuda")
        y = torch.zeros(2, P, P, 64, dtype=torch.bfloat16, device="cuda")
        in_bn = (torch.ones(C, device="cuda"), torch.zeros(C, device="cuda")) if pro else None
        a = hip.conv_args(x, w, y, ConvGeom(stride=s, pad_h=1, pad_w=1), in_bn=in_bn, relu_in=not pro)
        assert hip.L.drn_conv_halo_ok(ctypes.byref(a)) == 0
        a.cfg = hip.L.drn_conv_halo_cfg0()
        assert hip.L.drn_conv_fwd2(ctypes.byref(a), hip.zero_page.data_ptr(), hip.stream()) != 0
