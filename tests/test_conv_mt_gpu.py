"""Multi-tile LDS-DMA conv family (csrc/kernels/conv_mt.hip, config ids 38..) vs the fp32
reference: every configuration x epilogue variant (residual, forward BN statistics, fused
BN-backward reduction, strided output map) x fused input-BN prologue, on geometries with
several tiles per workgroup, partial pixel / channel tiles and padding."""
import ctypes

import pytest
import torch

from distributed_resnet_tensorflow_amd.ops.backend import ConvGeom, OutMap

pytestmark = pytest.mark.gpu

MT0 = 38  # first multi-tile config id (after the 38 one-tile LDS-DMA configurations)


def rel(a, b):
    a = a.float().cpu()
    b = b.float().cpu()
    return (a - b).norm().item() / max(b.norm().item(), 1e-12)


def bf(t):
    return t.to(torch.bfloat16)


def n_mt(hip):
    return hip.L.drn_conv_glds_num_cfgs() - MT0


MT_CASES = [
    # N, H, C, K, R, stride, pad
    (4, 12, 64, 256, 1, 1, 0),    # T = 1 stage per tile, many tiles per block
    (3, 9, 128, 72, 3, 1, 1),     # K % BC != 0, 3x3 with padding, partial pixel tile
    (2, 13, 64, 128, 3, 2, 1),    # stride 2, odd size
    (2, 10, 256, 64, 1, 1, 0),    # 4 stages per tile
    (1, 7, 512, 128, 3, 1, 1),    # 72 stages per tile, M < one tile
]


def _run(hip, a, cfg):
    a.cfg = MT0 + cfg
    rc = hip.L.drn_conv_fwd2(ctypes.byref(a), hip.zero_page.data_ptr(), hip.stream())
    return rc


@pytest.mark.parametrize("case", MT_CASES)
@pytest.mark.parametrize("variant", ["plain", "pro_stats", "pro_res_stats", "stats", "res", "pro"])
def test_conv_mt_fwd(hip, ref, case, variant):
    N, H, C, K, R, s, p = case
    torch.manual_seed(3)
    P = (H + 2 * p - R) // s + 1
    x = bf(torch.randn(N, H, H, C))
    w = bf(torch.randn(K, R, R, C) * (2.0 / (R * R * C)) ** 0.5)
    g = ConvGeom(stride=s, pad_h=p, pad_w=p)
    pro = "pro" in variant
    use_res = "res" in variant
    use_st = "stats" in variant
    in_bn = (torch.rand(C) + 0.5, torch.randn(C) * 0.5) if pro else None
    res = bf(torch.randn(N, P, P, K)) if use_res else None
    y_ref = torch.zeros(N, P, P, K)
    st_ref = torch.zeros(2 * K)
    ref.conv_fwd(x.float(), w.float(), y_ref, g, in_bn=in_bn, residual=None if res is None else res.float(),
                 stats=st_ref)
    ran = 0
    for cfg in range(n_mt(hip)):
        y = torch.full((N, P, P, K), 3.0, dtype=torch.bfloat16, device="cuda")
        st = torch.zeros(3, 2, K, device="cuda") if use_st else None
        a = hip.conv_args(x.cuda(), w.cuda(), y, g, residual=None if res is None else res.cuda(), stats=st,
                          in_bn=None if in_bn is None else (in_bn[0].cuda(), in_bn[1].cuda()))
        if _run(hip, a, cfg) != 0:
            continue  # configuration's pipeline deeper than the stages of one tile
        ran += 1
        torch.cuda.synchronize()
        assert rel(y, y_ref) < 1e-2, cfg
        if use_st:
            s_hip = st.sum(0).view(-1).cpu()
            assert rel(s_hip[:K], st_ref[:K]) < 2e-2, cfg
            assert rel(s_hip[K:], st_ref[K:]) < 2e-2, cfg
    assert ran >= 3


@pytest.mark.parametrize("accumulate", [False, True])
@pytest.mark.parametrize("R", [1, 3])
def test_conv_mt_bn_bwd(hip, ref, accumulate, R):
    """Data-gradient conv with the fused BN-backward epilogue (ReLU mask, sum g, sum g*xhat),
    optionally accumulating into the existing gradient (projection blocks)."""
    torch.manual_seed(11)
    N, H, C, K = 3, 10, 128, 64   # output channels C of the data gradient
    dy = bf(torch.randn(N, H, H, K))
    wt = bf(torch.randn(C, R, R, K) * 0.05)
    xb = bf(torch.randn(N, H, H, C))
    sc, sh = torch.rand(C) + 0.5, torch.randn(C) * 0.3
    mu, istd = torch.randn(C) * 0.1, torch.rand(C) + 0.5
    res = bf(torch.randn(N, H, H, C)) if accumulate else None
    g = ConvGeom(1, (R - 1) // 2, (R - 1) // 2)
    y_ref = torch.zeros(N, H, H, C)
    st_ref = torch.zeros(2 * C)
    ref.conv_fwd(dy.float(), wt.float(), y_ref, g, residual=None if res is None else res.float(), stats=st_ref,
                 bn_bwd=(xb.float(), sc, sh, mu, istd))
    ran = 0
    for cfg in range(n_mt(hip)):
        y = res.clone().cuda() if accumulate else torch.zeros(N, H, H, C, dtype=torch.bfloat16, device="cuda")
        st = torch.zeros(2, 2, C, device="cuda")
        a = hip.conv_args(dy.cuda(), wt.cuda(), y, g, residual=y if accumulate else None, stats=st,
                          bn_bwd=(xb.cuda(), sc.cuda(), sh.cuda(), mu.cuda(), istd.cuda()))
        if _run(hip, a, cfg) != 0:
            continue
        ran += 1
        torch.cuda.synchronize()
        assert rel(y, y_ref) < 1e-2, cfg
        s_hip = st.sum(0).view(-1).cpu()
        assert rel(s_hip[:C], st_ref[:C]) < 2e-2, cfg
        assert rel(s_hip[C:], st_ref[C:]) < 2e-2, cfg
    assert ran >= 3


def test_conv_mt_out_map(hip, ref):
    """Strided output mapping (phase of a stride-2 data gradient), several tiles per block."""
    torch.manual_seed(5)
    N, P, C, K = 4, 9, 64, 64
    x = bf(torch.randn(N, P, P, C))
    w = bf(torch.randn(K, 1, 1, C) * 0.1)
    om = OutMap(P=P, Q=P, stride=2, oh=1, ow=0)
    y_ref = torch.zeros(N, 2 * P, 2 * P, K)
    ref.conv_fwd(x.float(), w.float(), y_ref, ConvGeom(1, 0, 0), out_map=om)
    for cfg in range(n_mt(hip)):
        y = torch.zeros(N, 2 * P, 2 * P, K, dtype=torch.bfloat16, device="cuda")
        a = hip.conv_args(x.cuda(), w.cuda(), y, ConvGeom(1, 0, 0), out_map=om)
        if _run(hip, a, cfg) != 0:
            continue
        torch.cuda.synchronize()
        assert rel(y, y_ref) < 1e-2, cfg


def test_conv_mt_rejects_unsupported(hip):
    """The multi-tile family refuses what its epilogue does not implement (the autotuner then
    skips it): in-kernel BN finalize, sibling-phase zero fill, C % 64 != 0."""
    x = torch.zeros(1, 4, 4, 32, dtype=torch.bfloat16, device="cuda")
    w = torch.zeros(64, 1, 1, 32, dtype=torch.bfloat16, device="cuda")
    y = torch.zeros(1, 4, 4, 64, dtype=torch.bfloat16, device="cuda")
    a = hip.conv_args(x, w, y, ConvGeom(1, 0, 0))
    assert _run(hip, a, 0) != 0
