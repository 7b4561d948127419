"""Numerics of every hand-written gfx950 kernel vs the fp32 PyTorch reference of the same op.

Inputs are rounded to bf16 once and fed to both sides; the reference then runs in fp32, so
the difference is accumulation order + the bf16 rounding of the kernel output.
"""
import ctypes

import pytest
import torch
import torch.nn.functional as F

from distributed_resnet_tensorflow_amd.ops.backend import OutMap, ConvGeom, dgrad_geom, tflip_desc, tflip_table

pytestmark = pytest.mark.gpu


def rel(a, b):
    a = a.float().cpu()
    b = b.float().cpu()
    return (a - b).norm().item() / max(b.norm().item(), 1e-12)


def bf(t):
    return t.to(torch.bfloat16)


CONV_CASES = [
    # N, H, W, C, K, R, stride, pad
    (2, 8, 8, 16, 16, 3, 1, 1),
    (2, 8, 8, 16, 32, 3, 1, 1),
    (3, 9, 9, 32, 64, 3, 2, 1),
    (2, 7, 7, 64, 256, 1, 1, 0),
    (2, 14, 14, 128, 128, 3, 2, 1),
    (2, 16, 16, 8, 64, 7, 2, 3),
    (2, 6, 6, 64, 64, 1, 2, 0),
    (1, 5, 5, 256, 512, 3, 1, 1),
]


def out_size(H, R, stride, pad):
    if stride == 1:
        return H
    return (H + (R - 1) - R) // stride + 1


@pytest.mark.parametrize("case", CONV_CASES)
@pytest.mark.parametrize("fused", [False, True])
def test_conv_fwd(hip, ref, case, fused):
    N, H, W, C, K, R, s, p = case
    torch.manual_seed(0)
    P = out_size(H, R, s, p)
    x = bf(torch.randn(N, H, W, C))
    w = bf(torch.randn(K, R, R, C) * (2.0 / (R * R * C)) ** 0.5)
    g = ConvGeom(stride=s, pad_h=p, pad_w=p)
    in_bn = None
    res = None
    if fused:
        in_bn = (torch.rand(C) + 0.5, torch.randn(C) * 0.1)
        res = bf(torch.randn(N, P, P, K))
    y_ref = torch.zeros(N, P, P, K)
    st_ref = torch.zeros(2 * K)
    ref.conv_fwd(x.float(), w.float(), y_ref, g, in_bn=in_bn, residual=None if res is None else res.float(),
                 stats=st_ref)
    y = torch.zeros(N, P, P, K, dtype=torch.bfloat16, device="cuda")
    st = torch.zeros(2, K, device="cuda")
    hip.conv_fwd(x.cuda(), w.cuda(), y, g,
                 in_bn=None if in_bn is None else (in_bn[0].cuda(), in_bn[1].cuda()),
                 residual=None if res is None else res.cuda(), stats=st)
    torch.cuda.synchronize()
    assert rel(y, y_ref) < 1e-2
    s_hip = st.view(-1).cpu()
    assert rel(s_hip[:K], st_ref[:K]) < 2e-2
    assert rel(s_hip[K:], st_ref[K:]) < 2e-2


GLDS_CASES = [
    # N, H, W, C, K, R, stride, pad   (C % 64 == 0: LDS-DMA kernel family)
    (2, 9, 9, 64, 64, 3, 1, 1),        # M=162: partial pixel tiles for every BP
    (3, 7, 7, 128, 256, 1, 1, 0),
    (2, 13, 13, 64, 128, 3, 2, 1),     # stride 2, odd size, padding
    (1, 6, 6, 192, 72, 3, 1, 1),       # K % BC != 0 (zero-page weight rows)
    (2, 8, 8, 256, 64, 1, 2, 0),
    (2, 9, 9, 96, 64, 3, 1, 1),        # C % 64 != 0: only the 32-deep-stage configs apply
    (2, 16, 16, 8, 64, 7, 2, 3),       # C == 8 (stem): row-staged, 64-deep-stage configs only
    (2, 9, 9, 8, 16, 3, 1, 1),         # C == 8, 3x3 (taps 3..7 of each stage are zero pieces)
    (2, 10, 10, 16, 16, 3, 1, 1),      # C == 16 (CIFAR stage 1): 2 chunks per tap, chunks 6, 7 zero
    (2, 9, 9, 16, 32, 3, 2, 1),        # C == 16, stride 2
    (2, 8, 8, 16, 64, 1, 1, 0),        # C == 16, 1x1 (chunks 2..7 zero)
]


N_GLDS = 38                              # one-tile LDS-DMA configurations (DRN_GLDS_NCFG)
BK32 = set(range(17, 23)) | {25, 27, 28, 29, 30, 33, 36, 37}  # 32-deep stages: C % 32 == 0 suffices
BIG = set(range(25, 31)) | {33, 34}      # 8-wave big tiles: no row-staged narrow inputs
IL = set(range(31, 38))                  # interleaved-DMA twins: no row-staged narrow inputs
KS = [0, 13, 25, 31, 32, 33]             # split-K capable


@pytest.mark.parametrize("case", GLDS_CASES)
@pytest.mark.parametrize("cfg", list(range(N_GLDS)))
@pytest.mark.parametrize("pro", [False, True])
def test_conv_fwd_glds_configs(hip, ref, case, cfg, pro):
    """Every tile/pipeline configuration of the LDS-DMA conv kernel vs the fp32 reference,
    with residual add + BN statistics epilogue; pro: the input is the raw pre-BN tensor and the
    kernel applies relu(x * scale + shift) to each landed stage in LDS (padding stays zero)."""
    N, H, W, C, K, R, s, p = case
    torch.manual_seed(10 + cfg)
    P = out_size(H, R, s, p)
    x = bf(torch.randn(N, H, W, C))
    w = bf(torch.randn(K, R, R, C) * (2.0 / (R * R * C)) ** 0.5)
    res = bf(torch.randn(N, P, P, K))
    g = ConvGeom(stride=s, pad_h=p, pad_w=p)
    in_bn = (torch.rand(C) + 0.5, torch.randn(C) * 0.5) if pro else None
    y_ref = torch.zeros(N, P, P, K)
    st_ref = torch.zeros(2 * K)
    ref.conv_fwd(x.float(), w.float(), y_ref, g, in_bn=in_bn, residual=res.float(), stats=st_ref)
    y = torch.zeros(N, P, P, K, dtype=torch.bfloat16, device="cuda")
    st = torch.zeros(3, 2, K, device="cuda")  # 3 atomic-spreading replicas
    a = hip.conv_args(x.cuda(), w.cuda(), y, g, residual=res.cuda(), stats=st,
                      in_bn=None if in_bn is None else (in_bn[0].cuda(), in_bn[1].cuda()))
    assert hip.L.drn_conv_glds_ok(a) == 1 and a.stats_rep == 3
    a.cfg = cfg
    narrow = C in (8, 16)                # row-staged: the 64-deep-stage configurations only
    if (C % 64 and not narrow and cfg not in BK32) or (narrow and (cfg in BK32 or cfg in BIG or cfg in IL)):
        assert hip.L.drn_conv_fwd2(ctypes.byref(a), hip.zero_page.data_ptr(), hip.stream()) != 0
        return
    hip.launch_conv(a)
    torch.cuda.synchronize()
    assert rel(y, y_ref) < 1e-2
    s_hip = st.sum(0).view(-1).cpu()
    assert rel(s_hip[:K], st_ref[:K]) < 2e-2
    assert rel(s_hip[K:], st_ref[K:]) < 2e-2


SPLITK_CASES = [
    # N, H, W, C, K, R, stride, pad
    (2, 9, 9, 64, 128, 3, 1, 1),       # partial pixel tiles, 9 taps
    (1, 7, 7, 256, 72, 3, 1, 1),       # K % BC != 0, uneven stage split
    (3, 8, 8, 128, 256, 1, 1, 0),      # 1x1: 2 / 4 stages split
]


@pytest.mark.parametrize("case", SPLITK_CASES)
@pytest.mark.parametrize("cfg", KS)
@pytest.mark.parametrize("ks", [2, 3])
def test_conv_fwd_splitk(hip, ref, case, cfg, ks):
    """Split-K launches (partial tiles + last-arriver epilogue) vs the fp32 reference, with the
    fused BN prologue, residual add and BN statistics, and bitwise equal across two launches
    (the partials are summed in split order, whatever the arrival order)."""
    N, H, W, C, K, R, s, p = case
    torch.manual_seed(30 + ks)
    P = out_size(H, R, s, p)
    x = bf(torch.randn(N, H, W, C))
    w = bf(torch.randn(K, R, R, C) * (2.0 / (R * R * C)) ** 0.5)
    res = bf(torch.randn(N, P, P, K))
    g = ConvGeom(stride=s, pad_h=p, pad_w=p)
    in_bn = (torch.rand(C) + 0.5, torch.randn(C) * 0.5)
    y_ref = torch.zeros(N, P, P, K)
    st_ref = torch.zeros(2 * K)
    ref.conv_fwd(x.float(), w.float(), y_ref, g, in_bn=in_bn, residual=res.float(), stats=st_ref)
    outs = []
    for _ in range(2):
        y = torch.zeros(N, P, P, K, dtype=torch.bfloat16, device="cuda")
        st = torch.zeros(3, 2, K, device="cuda")
        a = hip.conv_args(x.cuda(), w.cuda(), y, g, residual=res.cuda(), stats=st,
                          in_bn=(in_bn[0].cuda(), in_bn[1].cuda()))
        a.cfg = cfg
        hip._set_ksplit(a, ks)
        rc = hip.L.drn_conv_fwd2(ctypes.byref(a), hip.zero_page.data_ptr(), hip.stream())
        if rc != 0:
            assert R * R * C // (32 if cfg in BK32 else 64) < ks, (cfg, ks)  # fewer stages than splits
            return
        torch.cuda.synchronize()
        assert rel(y, y_ref) < 1e-2, (cfg, ks)
        s_hip = st.sum(0).view(-1).cpu()
        assert rel(s_hip[:K], st_ref[:K]) < 2e-2
        assert rel(s_hip[K:], st_ref[K:]) < 2e-2
        outs.append(y.clone())
    assert torch.equal(outs[0], outs[1])
    assert int(hip.ks_tickets.abs().sum()) == 0  # every ticket re-armed by its last arriver


@pytest.mark.parametrize("case", SPLITK_CASES)
@pytest.mark.parametrize("cfg", KS)
@pytest.mark.parametrize("G", [3, 7, 16])
def test_conv_fwd_streamk(hip, ref, case, cfg, G):
    """Stream-K launches (G workgroups share the tiles x k-stages units evenly; a tile spread
    over several workgroups is finished by its last arriver) vs the fp32 reference, bitwise
    equal across two launches, every ticket re-armed."""
    N, H, W, C, K, R, s, p = case
    torch.manual_seed(40 + G)
    P = out_size(H, R, s, p)
    x = bf(torch.randn(N, H, W, C))
    w = bf(torch.randn(K, R, R, C) * (2.0 / (R * R * C)) ** 0.5)
    res = bf(torch.randn(N, P, P, K))
    g = ConvGeom(stride=s, pad_h=p, pad_w=p)
    in_bn = (torch.rand(C) + 0.5, torch.randn(C) * 0.5)
    y_ref = torch.zeros(N, P, P, K)
    st_ref = torch.zeros(2 * K)
    ref.conv_fwd(x.float(), w.float(), y_ref, g, in_bn=in_bn, residual=res.float(), stats=st_ref)
    outs = []
    for _ in range(2):
        y = torch.zeros(N, P, P, K, dtype=torch.bfloat16, device="cuda")
        st = torch.zeros(3, 2, K, device="cuda")
        a = hip.conv_args(x.cuda(), w.cuda(), y, g, residual=res.cuda(), stats=st,
                          in_bn=(in_bn[0].cuda(), in_bn[1].cuda()))
        a.cfg = cfg
        slots = hip.L.drn_conv_sk_slots_cfg(ctypes.byref(a), cfg, G)
        hip._set_ksplit(a, -G)
        rc = hip.L.drn_conv_fwd2(ctypes.byref(a), hip.zero_page.data_ptr(), hip.stream())
        if slots == 0:
            assert rc != 0, (cfg, G)  # more workgroups than units: refused
            return
        assert rc == 0 and 1 <= slots <= G
        torch.cuda.synchronize()
        assert rel(y, y_ref) < 1e-2, (cfg, G)
        s_hip = st.sum(0).view(-1).cpu()
        assert rel(s_hip[:K], st_ref[:K]) < 2e-2
        assert rel(s_hip[K:], st_ref[K:]) < 2e-2
        outs.append(y.clone())
    assert torch.equal(outs[0], outs[1])
    assert int(hip.ks_tickets.abs().sum()) == 0


@pytest.mark.parametrize("G", [2, 3])
def test_conv_fwd_streamk_prologue_finalize_publishes_once(hip, G):
    """A stream-K launch whose workgroups each walk several tiles (G < tiles) with a publishing
    consumer-side BN finalize in the prologue: the moving averages move ONCE (workgroup 0's first
    segment), the output equals the conv reading separately finalized scale / shift."""
    from distributed_resnet_tensorflow_amd.ops.backend import BnCfin
    torch.manual_seed(13)
    N, H, C, K = 2, 14, 128, 256
    x = bf(torch.randn(N, H, H, C) + 0.2).cuda()
    wgt = bf(torch.randn(K, 1, 1, C) * 0.05).cuda()
    gamma, beta = (torch.rand(C) + 0.5).cuda(), (torch.randn(C) * 0.2).cuda()
    xf = x.float().reshape(-1, C)
    M = xf.shape[0]
    st = (torch.stack([xf.sum(0), (xf * xf).sum(0)]).unsqueeze(0) / 4).repeat(4, 1, 1).contiguous()
    sc0, sh0, mu0, is0 = (torch.zeros(C, device="cuda") for _ in range(4))
    hip.bn_finalize(st, 4, M, gamma, beta, None, None, sc0, sh0, mu0, is0, 0.997, 1e-5, update_running=False)
    g = ConvGeom(1, 0, 0)
    want = torch.empty(N, H, H, K, dtype=torch.bfloat16, device="cuda")
    hip.conv_fwd(x, wgt, want, g, in_bn=(sc0, sh0))
    for cfg in KS:
        rm, rv = torch.zeros(C, device="cuda"), torch.ones(C, device="cuda")
        sc, sh, mu, isd = (torch.full((C,), 7.0, device="cuda") for _ in range(4))
        fin = BnCfin(st, float(M), gamma, beta=beta, run_mean=rm, run_var=rv, scale=sc, shift=sh, mean=mu,
                     invstd=isd, publish=True)
        got = torch.empty_like(want)
        a = hip.conv_args(x, wgt, got, g, in_bn=(sc, sh), in_fin=fin)
        a.cfg = cfg
        if hip.L.drn_conv_sk_slots_cfg(ctypes.byref(a), cfg, G) == 0:
            continue
        hip._set_ksplit(a, -G)
        assert hip.L.drn_conv_fwd2(ctypes.byref(a), hip.zero_page.data_ptr(), hip.stream()) == 0, cfg
        torch.cuda.synchronize()
        assert rel(got, want) < 1e-2, cfg
        assert rel(rm, 0.003 * mu0) < 1e-4, cfg  # one update from 0, not two
        assert rel(sc, sc0) < 1e-5, cfg
    assert int(hip.ks_tickets.abs().sum()) == 0


@pytest.mark.parametrize("cfg", [0, 13, 31])
def test_conv_splitk_handoff_stress(hip, ref, cfg):
    """The in-launch partial-tile hand-off under hostile cache state: before every launch the
    partial workspace is poisoned with NaN and read back (its lines warm in some L2s / L1s), and
    launches alternate split-K factors and stream-K grids (different writer / reader placement).
    Any last arriver that reads a stale partial shows up as a NaN or a wrong output."""
    torch.manual_seed(77)
    N, H, W, C, K, R, s, p = 3, 8, 8, 128, 256, 1, 1, 0
    x = bf(torch.randn(N, H, W, C))
    w = bf(torch.randn(K, R, R, C) * (2.0 / (R * R * C)) ** 0.5)
    g = ConvGeom(stride=s, pad_h=p, pad_w=p)
    y_ref = torch.zeros(N, H, W, K)
    ref.conv_fwd(x.float(), w.float(), y_ref, g)
    xc, wc = x.cuda(), w.cuda()
    bad = []
    for it in range(60):
        ks = (2, 3, 4, -3, -5, -7)[it % 6]
        y = torch.zeros(N, H, W, K, dtype=torch.bfloat16, device="cuda")
        a = hip.conv_args(xc, wc, y, g)
        a.cfg = cfg
        hip._set_ksplit(a, ks)
        if ks < 0 and a.ksplit == 0:
            continue
        hip.ks_ws.fill_(float("nan"))
        float(hip.ks_ws.sum())  # warm the poisoned lines
        rc = hip.L.drn_conv_fwd2(ctypes.byref(a), hip.zero_page.data_ptr(), hip.stream())
        if rc != 0:
            continue  # (fewer k-stages than splits for the 32-deep configurations)
        torch.cuda.synchronize()
        if not bool(torch.isfinite(y.float()).all()) or rel(y, y_ref) > 1e-2:
            bad.append((it, ks))
    assert not bad, bad
    assert int(hip.ks_tickets.abs().sum()) == 0


def test_conv_sk_slots(hip):
    """The stream-K slot count bounds how many workgroups one tile's k-stages can touch."""
    a = hip.conv_args(torch.zeros(2, 9, 9, 64, dtype=torch.bfloat16, device="cuda"),
                      torch.zeros(128, 3, 3, 64, dtype=torch.bfloat16, device="cuda"),
                      torch.zeros(2, 9, 9, 128, dtype=torch.bfloat16, device="cuda"), ConvGeom(1, 1, 1))
    # config 0: 128x128 tiles, 64-deep stages -> 2 tiles x 9 stages = 18 units
    for G in range(1, 19):
        starts = [b * 18 // G for b in range(G)] + [18]
        touch = max(sum(1 for b in range(G) if starts[b] < (t + 1) * 9 and starts[b + 1] > t * 9) for t in range(2))
        slots = hip.L.drn_conv_sk_slots_cfg(ctypes.byref(a), 0, G)
        assert slots == touch, (G, touch, slots)
    assert hip.L.drn_conv_sk_slots_cfg(ctypes.byref(a), 0, 18) == 9   # one unit per workgroup
    assert hip.L.drn_conv_sk_slots_cfg(ctypes.byref(a), 0, 19) == 0   # empty ranges refused
    assert hip.L.drn_conv_sk_slots_cfg(ctypes.byref(a), 1, 4) == 0    # not split-capable


NK_CASES = [
    # N, H, W, C, K, R, stride, pad      (narrow-output register-operand kernels, K = 16 / 32)
    (2, 9, 9, 64, 16, 1, 1, 0),          # CIFAR stage-1 1x1 reduce, partial pixel tiles
    (2, 9, 9, 16, 16, 3, 1, 1),          # 3x3 16 -> 16: taps paired per 32-deep k-step
    (3, 8, 8, 16, 32, 3, 1, 1),          # 32 output channels
    (1, 9, 9, 32, 32, 3, 2, 1),          # stride 2
    (2, 8, 8, 128, 16, 1, 1, 0),         # 4 k-steps
    (2, 6, 6, 8, 16, 3, 1, 1),           # C = 8: four taps per k-step
]


@pytest.mark.parametrize("case", NK_CASES)
@pytest.mark.parametrize("i", range(5))
@pytest.mark.parametrize("pro", [False, True])
def test_conv_fwd_nk(hip, ref, case, i, pro):
    """Narrow-output convs (weights + im2col fragments straight to registers, shared epilogue)
    vs the fp32 reference, with the fused BN-apply prologue, residual add and BN statistics;
    configurations whose channel count does not match K are refused."""
    N, H, W, C, K, R, s, p = case
    torch.manual_seed(50 + i)
    P = out_size(H, R, s, p)
    x = bf(torch.randn(N, H, W, C))
    w = bf(torch.randn(K, R, R, C) * (2.0 / (R * R * C)) ** 0.5)
    res = bf(torch.randn(N, P, P, K))
    g = ConvGeom(stride=s, pad_h=p, pad_w=p)
    in_bn = (torch.rand(C) + 0.5, torch.randn(C) * 0.5) if pro else None
    y_ref = torch.zeros(N, P, P, K)
    st_ref = torch.zeros(2 * K)
    ref.conv_fwd(x.float(), w.float(), y_ref, g, in_bn=in_bn, residual=res.float(), stats=st_ref)
    y = torch.zeros(N, P, P, K, dtype=torch.bfloat16, device="cuda")
    st = torch.zeros(3, 2, K, device="cuda")
    a = hip.conv_args(x.cuda(), w.cuda(), y, g, residual=res.cuda(), stats=st,
                      in_bn=None if in_bn is None else (in_bn[0].cuda(), in_bn[1].cuda()))
    a.cfg = hip.L.drn_conv_nk_cfg0() + i
    rc = hip.L.drn_conv_fwd2(ctypes.byref(a), hip.zero_page.data_ptr(), hip.stream())
    mi = (1, 1, 2, 2, 2)[i]
    if K != 16 * mi:
        assert rc != 0
        return
    assert rc == 0
    torch.cuda.synchronize()
    assert rel(y, y_ref) < 1e-2
    s_hip = st.sum(0).view(-1).cpu()
    assert rel(s_hip[:K], st_ref[:K]) < 2e-2
    assert rel(s_hip[K:], st_ref[K:]) < 2e-2


@pytest.mark.parametrize("i", [0, 1])
@pytest.mark.parametrize("R", [1, 3])
def test_conv_nk_bn_bwd_reduce(hip, ref, i, R):
    """Narrow-output data gradient with the fused BN-backward epilogue (ReLU mask, sum g and
    sum g*xhat), as the CIFAR stage-1 backward runs it."""
    torch.manual_seed(13 + R)
    N, H, C, K = 2, 10, 64 if R == 1 else 16, 16
    dy = bf(torch.randn(N, H, H, C))
    wt = bf(torch.randn(K, R, R, C) * 0.1)
    xb = bf(torch.randn(N, H, H, K))
    sc, sh = torch.rand(K) + 0.5, torch.randn(K) * 0.3
    mu, istd = torch.randn(K) * 0.1, torch.rand(K) + 0.5
    g = ConvGeom(1, R // 2, R // 2)
    y_ref = torch.zeros(N, H, H, K)
    st_ref = torch.zeros(2 * K)
    ref.conv_fwd(dy.float(), wt.float(), y_ref, g, stats=st_ref, bn_bwd=(xb.float(), sc, sh, mu, istd))
    y = torch.zeros(N, H, H, K, dtype=torch.bfloat16, device="cuda")
    st = torch.zeros(2, K, device="cuda")
    a = hip.conv_args(dy.cuda(), wt.cuda(), y, g, stats=st,
                      bn_bwd=(xb.cuda(), sc.cuda(), sh.cuda(), mu.cuda(), istd.cuda()))
    a.cfg = hip.L.drn_conv_nk_cfg0() + i
    hip.launch_conv(a)
    torch.cuda.synchronize()
    assert rel(y, y_ref) < 1e-2
    s_hip = st.view(-1).cpu()
    assert rel(s_hip[:K], st_ref[:K]) < 2e-2
    assert rel(s_hip[K:], st_ref[K:]) < 2e-2


def test_conv_glds_out_map(hip, ref):
    """Phase output mapping (stride-2 data-gradient phases) through the LDS-DMA kernel."""
    torch.manual_seed(5)
    N, P, C, K = 2, 5, 64, 64
    x = bf(torch.randn(N, P, P, C))
    w = bf(torch.randn(K, 1, 1, C) * 0.1)
    om = OutMap(P=P, Q=P, stride=2, oh=1, ow=0)
    y_ref = torch.zeros(N, 2 * P, 2 * P, K)
    ref.conv_fwd(x.float(), w.float(), y_ref, ConvGeom(1, 0, 0), out_map=om)
    for cfg in list(range(23)) + sorted(BIG):
        y = torch.zeros(N, 2 * P, 2 * P, K, dtype=torch.bfloat16, device="cuda")
        a = hip.conv_args(x.cuda(), w.cuda(), y, ConvGeom(1, 0, 0), out_map=om)
        a.cfg = cfg
        hip.launch_conv(a)
        torch.cuda.synchronize()
        assert rel(y, y_ref) < 1e-2, cfg


@pytest.mark.parametrize("cfg", [100, 0, 3, 6, 13, 18, 25, 27])
@pytest.mark.parametrize("size", [5, 4])
def test_conv_out_fill(hip, ref, cfg, size):
    """Single-phase strided output (1x1 stride-2 projection data gradient) with out_fill: the
    epilogue writes zeros at the other phase positions of a garbage-filled output (odd and even
    output sizes)."""
    torch.manual_seed(6)
    N, C, K = 2, 64, 64
    H = 2 * size - 1  # odd: the last phase row/column is cut off
    P = (H + 1) // 2
    x = bf(torch.randn(N, P, P, C))
    w = bf(torch.randn(K, 1, 1, C) * 0.1)
    om = OutMap(P=P, Q=P, stride=2, oh=0, ow=0)
    y_ref = torch.full((N, H, H, K), 7.0)
    ref.conv_fwd(x.float(), w.float(), y_ref, ConvGeom(1, 0, 0), out_map=om, out_fill=True)
    assert float(y_ref[:, 1::2].abs().max()) == 0.0
    y = torch.full((N, H, H, K), 7.0, dtype=torch.bfloat16, device="cuda")
    old = hip.forced_cfg
    hip.forced_cfg = cfg
    try:
        hip.conv_fwd(x.cuda(), w.cuda(), y, ConvGeom(1, 0, 0), out_map=om, out_fill=True)
    finally:
        hip.forced_cfg = old
    torch.cuda.synchronize()
    assert rel(y, y_ref) < 1e-2, cfg
    assert float(y.float()[:, :, 1::2].abs().max()) == 0.0


@pytest.mark.parametrize("cfg", [100, 0, 3, 6, 25, 28])
def test_conv_fused_bn_bwd_reduce(hip, ref, cfg):
    """Data-gradient conv with the fused BN-backward epilogue (ReLU mask + sum g, sum g*xhat)."""
    torch.manual_seed(11)
    N, H, C, K = 2, 10, 64, 128
    dy = bf(torch.randn(N, H, H, K))
    wt = bf(torch.randn(C, 3, 3, K) * 0.05)
    xb = bf(torch.randn(N, H, H, C))
    sc, sh = torch.rand(C) + 0.5, torch.randn(C) * 0.3
    mu, istd = torch.randn(C) * 0.1, torch.rand(C) + 0.5
    res = bf(torch.randn(N, H, H, C))
    g = ConvGeom(1, 1, 1)
    y_ref = torch.zeros(N, H, H, C)
    st_ref = torch.zeros(2 * C)
    ref.conv_fwd(dy.float(), wt.float(), y_ref, g, residual=res.float(), stats=st_ref,
                 bn_bwd=(xb.float(), sc, sh, mu, istd))
    y = torch.zeros(N, H, H, C, dtype=torch.bfloat16, device="cuda")
    st = torch.zeros(2, C, device="cuda")
    a = hip.conv_args(dy.cuda(), wt.cuda(), y, g, residual=res.cuda(), stats=st,
                      bn_bwd=(xb.cuda(), sc.cuda(), sh.cuda(), mu.cuda(), istd.cuda()))
    a.cfg = cfg
    hip.launch_conv(a)
    torch.cuda.synchronize()
    assert rel(y, y_ref) < 1e-2
    s_hip = st.view(-1).cpu()
    assert rel(s_hip[:C], st_ref[:C]) < 2e-2
    assert rel(s_hip[C:], st_ref[C:]) < 2e-2


@pytest.mark.parametrize("case", CONV_CASES[:-1])
def test_conv_dgrad_matches_autograd(hip, case):
    N, H, W, C, K, R, s, p = case
    if C == 8:
        pytest.skip("stem has no data gradient")
    torch.manual_seed(1)
    P = out_size(H, R, s, p)
    x = bf(torch.randn(N, H, W, C)).float().requires_grad_(True)
    w = bf(torch.randn(K, R, R, C) * 0.1).float()
    g = ConvGeom(stride=s, pad_h=p, pad_w=p)
    dy = bf(torch.randn(N, P, P, K))
    # autograd oracle through the reference's fixed padding semantics
    xc = x.permute(0, 3, 1, 2)
    pb = (P - 1) * s + R - p - H
    y = F.conv2d(F.pad(xc, (p, pb, p, pb)), w.permute(0, 3, 1, 2), stride=s)
    y.backward(dy.float().permute(0, 3, 1, 2))
    dx_ref = x.grad
    wt = w.flip(1, 2).permute(3, 1, 2, 0).contiguous()  # [C][R][S][K]
    dx = torch.zeros(N, H, W, C, dtype=torch.bfloat16, device="cuda")
    hip.conv_fwd(dy.cuda(), bf(wt).cuda(), dx, dgrad_geom(g, R, R))
    torch.cuda.synchronize()
    assert rel(dx, dx_ref) < 1e-2


@pytest.mark.parametrize("case", CONV_CASES)
@pytest.mark.parametrize("fused", [False, True])
def test_conv_wgrad(hip, ref, case, fused):
    N, H, W, C, K, R, s, p = case
    torch.manual_seed(2)
    P = out_size(H, R, s, p)
    x = bf(torch.randn(N, H, W, C))
    dy = bf(torch.randn(N, P, P, K))
    g = ConvGeom(stride=s, pad_h=p, pad_w=p)
    in_bn = (torch.rand(C) + 0.5, torch.randn(C) * 0.1) if fused else None
    dw_ref = torch.zeros(K, R, R, C)
    ref.conv_wgrad(x.float(), dy.float(), dw_ref, g, in_bn=in_bn)
    dw = torch.zeros(K, R, R, C, device="cuda")
    ws = torch.zeros(max(1, hip.wgrad_ws_elems(N * P * P, K, R, R, C)), device="cuda")
    hip.conv_wgrad(x.cuda(), dy.cuda(), dw, g, in_bn=None if in_bn is None else (in_bn[0].cuda(), in_bn[1].cuda()),
                   ws=ws)
    torch.cuda.synchronize()
    assert rel(dw, dw_ref) < 1e-2


WGRAD_GLDS_CASES = [
    (2, 9, 9, 64, 64, 3, 1, 1),
    (2, 8, 8, 128, 256, 1, 1, 0),
    (3, 13, 13, 64, 128, 3, 2, 1),
    (2, 16, 16, 8, 64, 7, 2, 3),      # stem: Ktot = 392 (partial k tile)
    (2, 7, 7, 256, 72, 3, 1, 1),      # K % BCO != 0
    (1, 6, 6, 32, 16, 3, 1, 1),       # narrow output: 32-channel dY tile, half of it padding
    (2, 16, 16, 16, 16, 3, 1, 1),     # CIFAR stage 1: Ktot = 144 -> 64-deep k tiles (192), K = 16
    (2, 16, 16, 32, 32, 3, 1, 1),     # CIFAR stage 2: Ktot = 288 -> 64-deep k tiles (320), K = 32
    (2, 9, 9, 16, 32, 3, 2, 1),       # narrow, stride 2
    (2, 8, 8, 64, 24, 3, 1, 1),       # narrow, K % 32 != 0
    (3, 7, 7, 128, 256, 1, 1, 0),     # 1x1 stride-1 (uniform-base loader): 147 pixels, partial last stage
    (2, 9, 9, 72, 200, 1, 1, 0),      # 1x1 stride-1, partial k and output-channel tiles
    (8, 14, 14, 256, 128, 1, 1, 0),   # 1x1 stride-1, several pixel splits
]


@pytest.mark.parametrize("case", WGRAD_GLDS_CASES)
@pytest.mark.parametrize("ns", [0, 2, 3, 4, 5, 6, 7, 8])
@pytest.mark.parametrize("fused", [False, True])
def test_conv_wgrad_pipelines(hip, ref, case, ns, fused):
    """Register-staged (ns=0) and LDS-DMA (2/3 stages) weight-gradient kernels vs fp32;
    fused: the patch operand is relu(x * scale + shift) of the raw input, applied in LDS."""
    N, H, W, C, K, R, s, p = case
    torch.manual_seed(7)
    P = out_size(H, R, s, p)
    x = bf(torch.randn(N, H, W, C))
    dy = bf(torch.randn(N, P, P, K))
    g = ConvGeom(stride=s, pad_h=p, pad_w=p)
    in_bn = (torch.rand(C) + 0.5, torch.randn(C) * 0.5) if fused else None
    dw_ref = torch.zeros(K, R, R, C)
    ref.conv_wgrad(x.float(), dy.float(), dw_ref, g, in_bn=in_bn)
    dw = torch.zeros(K, R, R, C, device="cuda")
    ws = torch.zeros(max(1, hip.wgrad_ws_elems(N * P * P, K, R, R, C)), device="cuda")
    old = hip.forced_wgrad_ns
    hip.forced_wgrad_ns = ns
    try:
        run = lambda: hip.conv_wgrad(x.cuda(), dy.cuda(), dw, g, ws=ws,  # noqa: E731
                                     in_bn=None if in_bn is None else (in_bn[0].cuda(), in_bn[1].cuda()))
        if K <= 32 and ns in (4, 5, 6):
            # the narrow 32-channel dY tile needs 64-pixel stages (the autotuner skips these)
            from distributed_resnet_tensorflow_amd.ops._lib import KernelLibraryError
            with pytest.raises(KernelLibraryError):
                run()
            return
        run()
    finally:
        hip.forced_wgrad_ns = old
    torch.cuda.synchronize()
    assert rel(dw, dw_ref) < 1e-2


def test_conv_wgrad_large_splitk(hip, ref):
    N, H, C, K = 16, 28, 64, 64
    torch.manual_seed(3)
    x = bf(torch.randn(N, H, H, C))
    dy = bf(torch.randn(N, H, H, K))
    g = ConvGeom(1, 1, 1)
    dw_ref = torch.zeros(K, 3, 3, C)
    ref.conv_wgrad(x.float(), dy.float(), dw_ref, g)
    dw = torch.zeros(K, 3, 3, C, device="cuda")
    ws = torch.zeros(max(1, hip.wgrad_ws_elems(N * H * H, K, 3, 3, C)), device="cuda")
    hip.conv_wgrad(x.cuda(), dy.cuda(), dw, g, ws=ws)
    torch.cuda.synchronize()
    assert rel(dw, dw_ref) < 1e-2


@pytest.mark.parametrize("n,splits", [(4096, 483), (36864, 103), (25088, 128), (147456, 36), (1048576, 4),
                                      (1024, 7), (64, 1), (8, 300)])
@pytest.mark.parametrize("accumulate", [0, 1])
def test_splitk_reduce(hip, n, splits, accumulate):
    """Deterministic split-K reduction (all three column-tile widths) vs an fp64 sum."""
    torch.manual_seed(11)
    ws = torch.randn(splits, n, device="cuda")
    out0 = torch.randn(n, device="cuda")
    out = out0.clone()
    from distributed_resnet_tensorflow_amd.ops import _lib
    _lib.check(hip.L.drn_splitk_reduce(ws.data_ptr(), out.data_ptr(), n, splits, 0.5, accumulate, hip.stream()),
               "drn_splitk_reduce")
    again = out0.clone()
    _lib.check(hip.L.drn_splitk_reduce(ws.data_ptr(), again.data_ptr(), n, splits, 0.5, accumulate, hip.stream()),
               "drn_splitk_reduce")
    torch.cuda.synchronize()
    want = 0.5 * ws.double().sum(0) + (out0.double() if accumulate else 0)
    assert (out.double() - want).abs().max().item() < 1e-4 * max(1.0, splits ** 0.5)
    assert torch.equal(out, again)  # bitwise reproducible


@pytest.mark.parametrize("C", [16, 64, 256, 2048])
def test_bn_forward_and_backward(hip, ref, C):
    torch.manual_seed(4)
    N, H = 4, 5
    x = bf(torch.randn(N, H, H, C) * 2 + 0.5)
    gamma, beta = torch.rand(C) + 0.5, torch.randn(C) * 0.2
    dy0 = bf(torch.randn(N, H, H, C))
    add0 = bf(torch.randn(N, H, H, C))
    outs = {}
    for be, dev in ((ref, "cpu"), (hip, "cuda")):
        xx = x.to(dev) if dev == "cuda" else x.float()
        G = be.bn_stats_blocks(N * H * H, C)
        part = torch.zeros(G, 2, C, device=dev)
        G = be.bn_stats(xx, part)
        rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
        sc, sh, mu, isd = (torch.zeros(C, device=dev) for _ in range(4))
        be.bn_finalize(part, G, N * H * H, gamma.to(dev), beta.to(dev), rm, rv, sc, sh, mu, isd, 0.997, 1e-5)
        y = torch.zeros_like(xx)
        be.bn_apply(xx, y, sc, sh, relu=True)
        dy = dy0.to(dev) if dev == "cuda" else dy0.float()
        add = add0.to(dev) if dev == "cuda" else add0.float()
        Gb = be.bn_stats_blocks(N * H * H, C)
        partb = torch.zeros(Gb, 2, C, device=dev)
        Gb = be.bn_bwd_reduce(dy, None, 0, xx, sc, sh, mu, isd, partb)
        dg, db, coef = torch.zeros(C, device=dev), torch.zeros(C, device=dev), torch.zeros(3 * C, device=dev)
        be.bn_finalize_bwd(partb, Gb, N * H * H, gamma.to(dev), isd, dg, db, coef)
        dx = torch.zeros_like(xx)
        be.bn_bwd_apply(dy, None, 0, xx, sc, sh, mu, isd, coef, add, dx)
        outs[be.name] = [t.float().cpu() for t in (sc, sh, rm, rv, y, dg, db, dx)]
    for a, b in zip(outs["hip"], outs["ref"]):
        assert rel(a, b) < 1e-2


def test_bn_backward_pool_broadcast(hip, ref):
    """Final-BN backward with dY = dpool / HW broadcast (the global-average-pool gradient)."""
    torch.manual_seed(10)
    N, H, C = 4, 7, 256
    x = bf(torch.randn(N, H, H, C))
    dpool = torch.randn(N, C)
    gamma, beta = torch.rand(C) + 0.5, torch.randn(C) * 0.2
    outs = {}
    for be, dev in ((ref, "cpu"), (hip, "cuda")):
        xx = x.to(dev) if dev == "cuda" else x.float()
        part = torch.zeros(be.bn_stats_blocks(N * H * H, C), 2, C, device=dev)
        G = be.bn_stats(xx, part)
        sc, sh, mu, isd = (torch.zeros(C, device=dev) for _ in range(4))
        be.bn_finalize(part, G, N * H * H, gamma.to(dev), beta.to(dev), None, None, sc, sh, mu, isd, 0.997, 1e-5,
                       update_running=False)
        partb = torch.zeros(be.bn_stats_blocks(N * H * H, C), 2, C, device=dev)
        Gb = be.bn_bwd_reduce(None, dpool.to(dev), H * H, xx, sc, sh, mu, isd, partb)
        dg, db, coef = torch.zeros(C, device=dev), torch.zeros(C, device=dev), torch.zeros(3 * C, device=dev)
        be.bn_finalize_bwd(partb, Gb, N * H * H, gamma.to(dev), isd, dg, db, coef)
        dx = torch.zeros_like(xx)
        be.bn_bwd_apply(None, dpool.to(dev), H * H, xx, sc, sh, mu, isd, coef, None, dx)
        outs[be.name] = [t.float().cpu() for t in (dg, db, dx)]
    for a, b in zip(outs["hip"], outs["ref"]):
        assert rel(a, b) < 1e-2


def test_bn_autograd_oracle(ref):
    """The hand-written BN-ReLU backward equals autograd of batch-norm + relu (CPU oracle)."""
    torch.manual_seed(5)
    N, H, C = 3, 4, 16
    x = torch.randn(N, H, H, C, requires_grad=True)
    gamma = (torch.rand(C) + 0.5).requires_grad_(True)
    beta = (torch.randn(C) * 0.1).requires_grad_(True)
    y = torch.relu(F.batch_norm(x.permute(0, 3, 1, 2), None, None, gamma, beta, training=True, eps=1e-5))
    dy = torch.randn_like(y)
    y.backward(dy)
    xd = x.detach()
    part = torch.zeros(1, 2, C)
    ref.bn_stats(xd, part)
    sc, sh, mu, isd = (torch.zeros(C) for _ in range(4))
    ref.bn_finalize(part, 1, N * H * H, gamma.detach(), beta.detach(), None, None, sc, sh, mu, isd, 0.997, 1e-5,
                    update_running=False)
    dyn = dy.permute(0, 2, 3, 1).contiguous()
    partb = torch.zeros(1, 2, C)
    ref.bn_bwd_reduce(dyn, None, 0, xd, sc, sh, mu, isd, partb)
    dg, db, coef = torch.zeros(C), torch.zeros(C), torch.zeros(3 * C)
    ref.bn_finalize_bwd(partb, 1, N * H * H, gamma.detach(), isd, dg, db, coef)
    dx = torch.zeros_like(xd)
    ref.bn_bwd_apply(dyn, None, 0, xd, sc, sh, mu, isd, coef, None, dx)
    assert torch.allclose(dx, x.grad, atol=1e-4, rtol=1e-3)
    assert torch.allclose(dg, gamma.grad, atol=1e-4, rtol=1e-3)
    assert torch.allclose(db, beta.grad, atol=1e-4, rtol=1e-3)


def test_head(hip, ref):
    torch.manual_seed(6)
    N, H, C, ncls = 8, 7, 2048, 1001
    x = bf(torch.randn(N, H, H, C))
    sc, sh = torch.rand(C) + 0.5, torch.randn(C) * 0.1
    Wd = torch.randn(ncls, C) * 0.02
    b = torch.randn(ncls) * 0.1
    labels = torch.randint(0, ncls, (N,), dtype=torch.int32)
    res = {}
    for be, dev in ((ref, "cpu"), (hip, "cuda")):
        xx = x.cuda() if dev == "cuda" else x.float()
        pooled = torch.zeros(N, C, device=dev)
        be.pool_bnrelu(xx, sc.to(dev), sh.to(dev), pooled)
        logits = torch.zeros(N, ncls, device=dev)
        be.sgemm(0, 1, N, ncls, C, 1.0, pooled, C, Wd.to(dev), C, 0.0, logits, ncls, bias=b.to(dev))
        dl = torch.zeros(N, ncls, device=dev)
        loss = torch.zeros(N, device=dev)
        corr = torch.zeros(N, dtype=torch.int32, device=dev)
        be.softmax_xent(logits, labels.to(dev), 1.0 / N, dl, loss, corr)
        dW = torch.zeros(ncls, C, device=dev)
        be.sgemm(1, 0, ncls, C, N, 1.0, dl, ncls, pooled, C, 0.0, dW, C)
        dpool = torch.zeros(N, C, device=dev)
        be.sgemm(0, 0, N, C, ncls, 1.0, dl, ncls, Wd.to(dev), C, 0.0, dpool, C)
        dbias = torch.zeros(ncls, device=dev)
        be.colsum(dl, dbias)
        res[be.name] = [t.float().cpu() for t in (pooled, logits, dl, loss, corr, dW, dpool, dbias)]
    for a, b2 in zip(res["hip"], res["ref"]):
        assert rel(a, b2) < 2e-3


@pytest.mark.parametrize("H,pad", [(12, 0), (11, 1), (13, 0), (112, 0)])
def test_maxpool(hip, ref, H, pad):
    """3x3/2 max-pool forward (argmax record) and the 2x2-blocked gather backward, even and odd
    sizes, TF 'SAME' padding (pad 0 before) and a symmetric pad."""
    torch.manual_seed(7)
    N, C = 2, 64
    P = (H + 2 * pad - 3) // 2 + 1 if pad else (H + 1) // 2
    x = bf(torch.randn(N, H, H, C))
    dy = bf(torch.randn(N, P, P, C))
    out = {}
    for be, dev in ((ref, "cpu"), (hip, "cuda")):
        xx = x.cuda() if dev == "cuda" else x.float()
        y = torch.zeros(N, P, P, C, dtype=xx.dtype, device=dev)
        arg = torch.zeros(N, P, P, C, dtype=torch.uint8, device=dev)
        st = torch.zeros(3, 2, C, device=dev)  # fused output statistics, 3 atomic replicas
        be.maxpool_fwd(xx, y, arg, 3, 2, pad, pad, stats=st)
        dx = torch.full_like(xx, 3.0)
        be.maxpool_bwd(dy.to(dev) if dev == "cuda" else dy.float(), arg, dx, 3, 2, pad, pad)
        out[be.name] = [y.float().cpu(), arg.cpu(), dx.float().cpu(), st.sum(0).cpu()]
    assert rel(out["hip"][0], out["ref"][0]) < 1e-3
    assert rel(out["hip"][2], out["ref"][2]) < 1e-2
    assert rel(out["hip"][3], out["ref"][3]) < 1e-3


def test_sgd_and_tflip(hip, ref):
    torch.manual_seed(8)
    n = 1000
    w0, m0, g0 = torch.randn(n), torch.randn(n), torch.randn(n)
    res = {}
    for be, dev in ((ref, "cpu"), (hip, "cuda")):
        w, m, g = w0.clone().to(dev), m0.clone().to(dev), g0.clone().to(dev)
        wb = torch.zeros(n, dtype=torch.bfloat16 if dev == "cuda" else torch.float32, device=dev)
        lr = torch.tensor([0.1], device=dev)
        be.sgd_momentum(w, m, g, wb, lr, 0.9, 2e-4, 0.5)
        res[be.name] = [w.cpu(), m.cpu(), wb.float().cpu()]
    for a, b in zip(res["hip"], res["ref"]):
        assert rel(a, b) < 4e-3
    # transpose-flip
    o1 = 16 * 9 * 8
    o2 = o1 + 32 * 16
    o3 = o2 + 16 * 2 * 8
    descs = [tflip_desc(0, 0, 16, 3, 3, 8), tflip_desc(o1, o1, 32, 1, 1, 16),
             tflip_desc(0, o2, 16, 3, 3, 8, Ru=2, Sv=1, r0=2, s0=1, dr=-2, ds=-2),
             tflip_desc(o3, o3, 136, 3, 3, 200),  # partial 64-wide tiles on both axes
             tflip_desc(o3, o3 + 136 * 9 * 200, 136, 3, 3, 200, Ru=1, Sv=2, r0=1, s0=2, dr=-2, ds=-2)]
    tot = o3 + 136 * 9 * 200 + 136 * 2 * 200
    wflat = torch.randn(tot)
    table, nt, total = tflip_table(descs)
    out_ref = torch.zeros(tot)
    ref.weight_tflip(wflat, out_ref, table, nt, total)
    out_hip = torch.zeros(tot, dtype=torch.bfloat16, device="cuda")
    hip.weight_tflip(bf(wflat).cuda(), out_hip, table.cuda(), nt, total)
    torch.cuda.synchronize()
    assert torch.equal(out_hip.float().cpu(), bf(out_ref).float())


def test_cifar_augment(hip, ref):
    torch.manual_seed(9)
    N = 4
    raw = torch.randint(0, 256, (N, 32, 32, 3), dtype=torch.uint8)
    params = torch.tensor([[0, 0, 0], [8, 8, 1], [3, 5, 1], [4, 4, 0]], dtype=torch.int32)
    o_ref = torch.zeros(N, 32, 32, 8)
    ref.cifar_augment(raw, params, o_ref, 4)
    o = torch.zeros(N, 32, 32, 8, dtype=torch.bfloat16, device="cuda")
    hip.cifar_augment(raw.cuda(), params.cuda(), o, 4)
    torch.cuda.synchronize()
    assert rel(o, o_ref) < 1e-2


@pytest.mark.parametrize("cfg", [100, 0, 3, 10, 15, 17, "nk"])
@pytest.mark.parametrize("bwd", [False, True])
def test_conv_fused_bn_finalize(hip, ref, cfg, bwd):
    """The last-arriving workgroup of each channel column finalizes the BN (forward: scale /
    shift / mean / invstd + moving averages; backward: dgamma, dbeta, coef) inside the conv,
    matching the separate finalize; the arrival counters are re-armed for the next launch."""
    from distributed_resnet_tensorflow_amd.ops.backend import BnFin
    torch.manual_seed(12)
    N, H, C, K = 8, 28, 64, 320          # K = 320: partial channel columns for BC = 128 / 256
    if cfg == "nk":                      # narrow-output kernel: 16 -> 16 channels, one column
        C, K, cfg = 16, 16, hip.L.drn_conv_nk_cfg0() + 1
    x = bf(torch.randn(N, H, H, C))
    w = bf(torch.randn(K, 3, 3, C) * 0.05)
    g = ConvGeom(1, 1, 1)
    count = float(N * H * H)
    xb = bf(torch.randn(N, H, H, K))
    sc, sh = torch.rand(K) + 0.5, torch.randn(K) * 0.3
    mu, istd = torch.randn(K) * 0.1, torch.rand(K) + 0.5
    gamma, beta = torch.rand(K) + 0.5, torch.randn(K) * 0.1
    rm0, rv0 = torch.randn(K) * 0.1, torch.rand(K) + 0.5

    def run(be, dev, dt):
        t = lambda v: v.to(dev)
        y = torch.zeros(N, H, H, K, dtype=dt, device=dev)
        rep = getattr(be, "stats_replicas", 1)
        st = torch.zeros(rep, 2, K, device=dev)
        outs = {k: torch.zeros(K, device=dev) for k in ("scale", "shift", "mean", "invstd", "dgamma", "dbeta")}
        outs["coef"] = torch.zeros(3 * K, device=dev)
        outs["run_mean"], outs["run_var"] = t(rm0.clone()), t(rv0.clone())
        cnt = torch.zeros(64, dtype=torch.int32, device=dev)
        if bwd:
            fin = BnFin(cnt, count, t(gamma), dgamma=outs["dgamma"], dbeta=outs["dbeta"], coef=outs["coef"])
            bb = (t(xb) if dev == "cuda" else xb.float(), t(sc), t(sh), t(mu), t(istd))
        else:
            fin = BnFin(cnt, count, t(gamma), beta=t(beta), run_mean=outs["run_mean"], run_var=outs["run_var"],
                        scale=outs["scale"], shift=outs["shift"], mean=outs["mean"], invstd=outs["invstd"])
            bb = None
        xx, ww = (x.cuda(), w.cuda()) if dev == "cuda" else (x.float(), w.float())
        if dev == "cuda":
            a = be.conv_args(xx, ww, y, g, stats=st, bn_bwd=bb, bn_fin=fin)
            a.cfg = cfg
            for _ in range(2):   # second launch: the counters must have been re-armed
                st.zero_()       # (the executor clears the statistics arena once per step)
                be.launch_conv(a)
            torch.cuda.synchronize()
            assert int(cnt.abs().sum()) == 0, "arrival counters not re-armed"
        else:
            for _ in range(2):
                be.conv_fwd(xx, ww, y, g, stats=st, bn_bwd=bb, bn_fin=fin)
        return {k: v.float().cpu() for k, v in outs.items()}

    got = run(hip, "cuda", torch.bfloat16)
    exp = run(ref, "cpu", torch.float32)   # (the reference finalize clears its accumulator itself)
    keys = ("dgamma", "dbeta", "coef") if bwd else ("scale", "shift", "mean", "invstd", "run_mean", "run_var")
    for k in keys:
        assert rel(got[k], exp[k]) < 2e-2, (k, rel(got[k], exp[k]))


@pytest.mark.parametrize("C,G", [(64, 8), (256, 8), (1024, 2), (2048, 1)])
@pytest.mark.parametrize("relu_bwd", [True, False])
def test_bn_consumer_finalize(hip, ref, C, G, relu_bwd):
    """Consumer-side BN finalize (BnCfin): the materialising apply and the backward apply derive
    the BN parameters from G statistics replicas in their prologue and publish them (moving
    averages, dgamma/dbeta); compared with the separate finalize + apply of the fp32 reference."""
    from distributed_resnet_tensorflow_amd.ops.backend import BnCfin
    torch.manual_seed(11)
    N, H = 4, 6
    x = bf(torch.randn(N, H, H, C) * 1.5 + 0.3)
    dy0, add0 = bf(torch.randn(N, H, H, C)), bf(torch.randn(N, H, H, C))
    gamma, beta = torch.rand(C) + 0.5, torch.randn(C) * 0.2
    M = N * H * H
    xf = x.float().reshape(M, C)
    # the same sums split over G replicas (as the atomic-spreading producers leave them)
    tot = torch.stack([xf.sum(0), (xf * xf).sum(0)])
    w = torch.rand(G, 1, 1)
    w = w / w.sum()
    parts = (tot.unsqueeze(0) * w).contiguous()
    outs = {}
    for be, dev in ((ref, "cpu"), (hip, "cuda")):
        xx = x.to(dev) if dev == "cuda" else x.float()
        st = parts.to(dev) if dev == "cuda" else parts.sum(0, keepdim=True).clone()
        rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
        sc, sh, mu, isd = (torch.zeros(C, device=dev) for _ in range(4))
        fin = BnCfin(st, float(M), gamma.to(dev), beta=beta.to(dev), run_mean=rm, run_var=rv, scale=sc, shift=sh,
                     mean=mu, invstd=isd, publish=True)
        y = torch.zeros_like(xx)
        be.bn_apply_fin(xx, y, fin, relu=True)
        dy = dy0.to(dev) if dev == "cuda" else dy0.float()
        add = add0.to(dev) if dev == "cuda" else add0.float()
        # backward sums (sum g, sum g*xhat) of the masked gradient, again split over replicas
        g = dy.float().reshape(M, C) * ((xx.float().reshape(M, C) * sc + sh) > 0).float() if relu_bwd \
            else dy.float().reshape(M, C)
        xh = (xx.float().reshape(M, C) - mu) * isd
        btot = torch.stack([g.sum(0), (g * xh).sum(0)])
        bst = (btot.unsqueeze(0) * w.to(btot.device)).contiguous() if dev == "cuda" else btot.unsqueeze(0).clone()
        dg, db = torch.zeros(C, device=dev), torch.zeros(C, device=dev)
        bfin = BnCfin(bst, float(M), gamma.to(dev), mean=mu, invstd=isd, dgamma=dg, dbeta=db, publish=True)
        dx = torch.zeros_like(xx)
        be.bn_bwd_apply_fin(dy, None, 0, xx, sc, sh, bfin, add, dx, relu=relu_bwd)
        outs[be.name] = [t.float().cpu() for t in (sc, sh, mu, isd, rm, rv, y, dg, db, dx)]
    for name, a, b in zip("sc sh mu isd rm rv y dg db dx".split(), outs["hip"], outs["ref"]):
        assert rel(a, b) < 1e-2, name


@pytest.mark.parametrize("C", [256, 1024])
def test_bn_bwd_apply_fin_non_publishing(hip, C):
    """A non-publishing backward apply (fused prologue finalize below BN_FIN_SPLIT_C channels,
    separate finalize launch into scratch at and above it) leaves dgamma / dbeta untouched and
    computes the same dx as the publishing one."""
    from distributed_resnet_tensorflow_amd.ops.backend import BnCfin
    torch.manual_seed(13)
    N, H = 4, 6
    M = N * H * H
    x = bf(torch.randn(N, H, H, C)).cuda()
    dy = bf(torch.randn(N, H, H, C)).cuda()
    sc, sh = (torch.rand(C) + 0.5).cuda(), (torch.randn(C) * 0.3).cuda()
    mu, isd = (torch.randn(C) * 0.1).cuda(), (torch.rand(C) + 0.5).cuda()
    bst = torch.randn(4, 2, C).cuda()
    gamma = (torch.rand(C) + 0.5).cuda()
    res = {}
    for pub in (True, False):
        dg, db = torch.full((C,), 7.0, device="cuda"), torch.full((C,), 7.0, device="cuda")
        dx = torch.zeros_like(x)
        hip.bn_bwd_apply_fin(dy, None, 0, x, sc, sh, BnCfin(bst, float(M), gamma, mean=mu, invstd=isd, dgamma=dg,
                                                           dbeta=db, publish=pub), None, dx, relu=True)
        res[pub] = (dx.float().cpu(), dg.cpu(), db.cpu())
    assert torch.equal(res[True][0], res[False][0])
    assert bool((res[False][1] == 7.0).all()) and bool((res[False][2] == 7.0).all())
    assert not bool((res[True][1] == 7.0).all())


@pytest.mark.parametrize("M,C", [(100352, 128), (25088 + 7, 256), (391, 2048)])
@pytest.mark.parametrize("fin", [True, False])
@pytest.mark.parametrize("add", [False, True])
def test_bn_bwd_apply_batches(hip, M, C, fin, add):
    """The backward applies' 4-vector batches (loads issued before the coefficient prologue, the
    last batch partial, clamped loads past the end) on tensors of several batches per thread,
    against the affine form dx = A*g + B*x + D (+ add) computed in fp32 by PyTorch."""
    from distributed_resnet_tensorflow_amd.ops.backend import BnCfin
    torch.manual_seed(21)
    x = bf(torch.randn(M, C) * 1.5 + 0.2).cuda()
    dy = bf(torch.randn(M, C)).cuda()
    a = bf(torch.randn(M, C)).cuda() if add else None
    sc, sh = (torch.rand(C) + 0.5).cuda(), (torch.randn(C) * 0.3).cuda()
    mu, isd = (torch.randn(C) * 0.1).cuda(), (torch.rand(C) + 0.5).cuda()
    gamma = (torch.rand(C) + 0.5).cuda()
    bst = (torch.randn(3, 2, C) * M ** 0.5).cuda()
    sg, sgx = bst[:, 0].sum(0), bst[:, 1].sum(0)
    k1, k2, k3 = gamma * isd, sg / M, sgx / M
    dx = torch.full_like(x, float("nan"))
    if fin:
        dg, db = torch.zeros(C, device="cuda"), torch.zeros(C, device="cuda")
        hip.bn_bwd_apply_fin(dy, None, 0, x, sc, sh, BnCfin(bst, float(M), gamma, mean=mu, invstd=isd, dgamma=dg,
                                                           dbeta=db, publish=True), a, dx, relu=True)
        assert rel(dg, sgx) < 1e-5 and rel(db, sg) < 1e-5
    else:
        coef = torch.cat([k1, k2, k3])
        hip.bn_bwd_apply(dy, None, 0, x, sc, sh, mu, isd, coef, a, dx, relu=True)
    xf = x.float()
    g = dy.float() * ((xf * sc + sh) > 0).float()
    want = k1 * (g - k2 - (xf - mu) * isd * k3)
    if add:
        want = want + a.float()
    assert bool(torch.isfinite(dx.float()).all())   # every element written (the tail included)
    assert rel(dx.float(), want) < 1e-2


@pytest.mark.parametrize("publish", [True, False])
@pytest.mark.parametrize("nk", [False, True])
def test_conv_prologue_finalize(hip, ref, publish, nk):
    """A fused-prologue 1x1 conv finalizing its input BN from the statistics replicas equals the
    conv reading separately finalized scale/shift; only a publishing launch writes them out
    (nk: the narrow-output register-operand kernel, 16 output channels)."""
    from distributed_resnet_tensorflow_amd.ops.backend import BnCfin
    torch.manual_seed(12)
    N, H, C, K = 2, 14, 128, 16 if nk else 256
    old_forced = hip.forced_cfg
    hip.forced_cfg = hip.L.drn_conv_nk_cfg0() + 1 if nk else old_forced
    try:
        _prologue_finalize_case(hip, publish, N, H, C, K)
    finally:
        hip.forced_cfg = old_forced


def _prologue_finalize_case(hip, publish, N, H, C, K):
    from distributed_resnet_tensorflow_amd.ops.backend import BnCfin
    x = bf(torch.randn(N, H, H, C) + 0.2).cuda()
    wgt = bf(torch.randn(K, 1, 1, C) * 0.05).cuda()
    gamma, beta = (torch.rand(C) + 0.5).cuda(), (torch.randn(C) * 0.2).cuda()
    xf = x.float().reshape(-1, C)
    st = (torch.stack([xf.sum(0), (xf * xf).sum(0)]).unsqueeze(0) / 4).repeat(4, 1, 1).contiguous()
    sc0, sh0, mu0, is0 = (torch.zeros(C, device="cuda") for _ in range(4))
    hip.bn_finalize(st, 4, xf.shape[0], gamma, beta, None, None, sc0, sh0, mu0, is0, 0.997, 1e-5, update_running=False)
    want = torch.empty(N, H, H, K, dtype=torch.bfloat16, device="cuda")
    hip.conv_fwd(x, wgt, want, ConvGeom(1, 0, 0), in_bn=(sc0, sh0))
    sc, sh, mu, isd = (torch.full((C,), 7.0, device="cuda") for _ in range(4))
    fin = BnCfin(st, float(xf.shape[0]), gamma, beta=beta, scale=sc, shift=sh, mean=mu, invstd=isd, publish=publish)
    got = torch.empty_like(want)
    hip.conv_fwd(x, wgt, got, ConvGeom(1, 0, 0), in_bn=(sc, sh), in_fin=fin)
    torch.cuda.synchronize()
    assert rel(got, want) < 1e-2
    if publish:
        assert rel(sc, sc0) < 1e-5 and rel(sh, sh0) < 1e-4 and rel(isd, is0) < 1e-5
    else:
        assert bool((sc == 7.0).all())


@pytest.mark.parametrize("case", [(4, 16, 16, 16, 3, 1, 1), (4, 24, 64, 32, 1, 1, 0), (4, 33, 32, 64, 3, 2, 1)])
@pytest.mark.parametrize("ns", [0, 2, 5, 7])
def test_wgrad_atomic_split_k(hip, ref, case, ns):
    """Split-K weight gradient accumulated with fp32 atomics straight into the (pre-zeroed)
    gradient instead of partial slabs + drn_splitk_reduce."""
    N, H, C, K, R, s, p = case
    torch.manual_seed(31 + ns)
    P = (H + 2 * p - R) // s + 1
    x = bf(torch.randn(N, H, H, C))
    dy = bf(torch.randn(N, P, P, K))
    g = ConvGeom(s, p, p)
    dw_ref = torch.zeros(K, R, R, C)
    ref.conv_wgrad(x.float(), dy.float(), dw_ref, g)
    dw = torch.zeros(K, R, R, C, device="cuda")
    xd, dyd = x.cuda(), dy.cuda()   # (the launch arguments hold raw pointers: keep the tensors alive)
    a = hip.wgrad_args(xd, dyd, dw, g, target_blocks=4096, atomic=True)
    assert a.splits > 1 and a.atomic_out == 1
    if K <= 32 and ns in (4, 5, 6):  # narrow 32-channel dY tiles: 64-pixel stages only
        assert hip.L.drn_conv_wgrad2(ctypes.byref(a), hip.zero_page.data_ptr(), ns, hip.stream()) != 0
        return
    hip._wgrad_full(a, ns, dw, hip.stream())
    torch.cuda.synchronize()
    assert rel(dw, dw_ref) < 1e-2


@pytest.mark.parametrize("N,H,pad", [(2, 224, 3), (3, 64, 3), (2, 96, 3)])
def test_fused_stem_conv_pool(hip, ref, N, H, pad):
    """Fused ImageNet stem (csrc/kernels/stem_pool.hip stem_conv_pool_kernel): packed 7x7/2 conv +
    3x3/2 max-pool + the pooled BN statistics in one kernel equals the two-kernel path (packed conv
    with the tuned configuration, then maxpool_fwd) -- pooled values, first-max taps, statistics --
    and the fp32 reference (conv, bf16 rounding, ceil-mode 3x3/2 max-pool)."""
    import torch.nn.functional as F
    torch.manual_seed(H + N)
    K, R = 64, 7
    # pad 3: the reference's conv2d_fixed_padding (explicit 3 + 3, what the executor runs)
    P = (H + 2 * pad - R) // 2 + 1
    PP = (P + 1) // 2
    x = torch.zeros(N, H, H, 8)
    x[..., :3] = torch.randn(N, H, H, 3)
    x = bf(x)
    w = torch.zeros(K, R, R, 8)
    w[..., :3] = torch.randn(K, R, R, 3) * (2.0 / (R * R * 3)) ** 0.5
    w = bf(w)
    n_xp = N * H * (H + 2) * 4
    buf = torch.zeros(n_xp + 64, dtype=torch.bfloat16, device="cuda")
    xp = buf[:n_xp].view(N, H, H + 2, 4)
    hip.stem_pack_input(x.cuda(), xp)
    w4 = torch.zeros(K, R, 8, 4, dtype=torch.bfloat16, device="cuda")
    hip.stem_pack_weights(w.cuda(), w4)
    g4 = ConvGeom(stride=2, pad_h=pad, pad_w=pad - 1)
    # two-kernel path
    y = torch.zeros(N, P, P, K, dtype=torch.bfloat16, device="cuda")
    hip.conv_fwd(xp, w4, y, g4)
    yp_ref = torch.zeros(N, PP, PP, K, dtype=torch.bfloat16, device="cuda")
    arg_ref = torch.zeros(N, PP, PP, K, dtype=torch.uint8, device="cuda")
    st_ref = torch.zeros(2, 2, K, device="cuda")
    hip.maxpool_fwd(y, yp_ref, arg_ref, 3, 2, 0, 0, stats=st_ref)
    # fused
    yp = torch.full((N, PP, PP, K), float("nan"), dtype=torch.bfloat16, device="cuda")
    arg = torch.full((N, PP, PP, K), 77, dtype=torch.uint8, device="cuda")
    st = torch.zeros(3, 2, K, device="cuda")
    hip.stem_conv_pool(xp, w4, yp, arg, g4, H, H, P, P, stats=st)
    torch.cuda.synchronize()
    assert bool(torch.isfinite(yp.float()).all())
    diff = (yp.float() - yp_ref.float()).abs()
    # same bf16 conv outputs up to the MFMA summation order: nearly all pooled values identical
    assert (diff > 0).float().mean().item() < 1e-3, (diff > 0).float().mean().item()
    assert diff.max().item() <= 0.05 * yp_ref.float().abs().max().item()
    same = diff == 0
    assert (arg[same] == arg_ref[same]).float().mean().item() > 0.999
    assert int(arg.max()) <= 8
    s1, s0 = st.sum(0).view(-1).cpu(), st_ref.sum(0).view(-1).cpu()
    assert rel(s1[:K], s0[:K]) < 1e-3 and rel(s1[K:], s0[K:]) < 1e-3
    # the fp32 reference
    y32 = torch.zeros(N, P, P, K)
    ref.conv_fwd(x.float(), w.float(), y32, ConvGeom(stride=2, pad_h=pad, pad_w=pad))
    yb = bf(y32).float().permute(0, 3, 1, 2)
    p32 = F.max_pool2d(yb, 3, 2, ceil_mode=True).permute(0, 2, 3, 1)
    assert tuple(p32.shape) == (N, PP, PP, K)
    assert rel(yp.float().cpu(), p32) < 1e-2
    # refused geometry: output width not a multiple of 16
    a_bad = hip.L.drn_stem_conv_pool(xp.data_ptr(), w4.data_ptr(), yp.data_ptr(), arg.data_ptr(), None, 1, N, H, H,
                                     P, P - 8, PP, (P - 8 + 1) // 2, K, pad, 1, hip.stream())
    assert a_bad != 0


@pytest.mark.parametrize("N,H", [(2, 16), (3, 30), (2, 224)])
def test_packed_stem(hip, ref, N, H):
    """Packed stem (csrc/kernels/stem.hip): the 7x7/2 conv over a 4-channel, column-padded copy of
    the 8-channel images with tap-pair weights equals the fp32 reference of the original conv --
    forward with BN statistics under every applicable LDS-DMA configuration, and the weight
    gradient (every pipeline) mapped back to the [K,7,7,8] layout, padding channels exactly 0."""
    torch.manual_seed(H)
    K, R = 64, 7
    P = out_size(H, R, 2, 3)
    x = torch.zeros(N, H, H, 8)
    x[..., :3] = torch.randn(N, H, H, 3)
    x = bf(x)
    w = torch.zeros(K, R, R, 8)
    w[..., :3] = torch.randn(K, R, R, 3) * (2.0 / (R * R * 3)) ** 0.5
    w = bf(w)
    g8 = ConvGeom(stride=2, pad_h=3, pad_w=3)
    g4 = ConvGeom(stride=2, pad_h=3, pad_w=2)
    y_ref = torch.zeros(N, P, P, K)
    st_ref = torch.zeros(2 * K)
    ref.conv_fwd(x.float(), w.float(), y_ref, g8, stats=st_ref)
    xd = x.cuda()
    n_xp = N * H * (H + 2) * 4
    buf = torch.zeros(n_xp + 64, dtype=torch.bfloat16, device="cuda")
    xp = buf[:n_xp].view(N, H, H + 2, 4)
    hip.stem_pack_input(xd, xp)
    w4 = torch.zeros(K, R, 8, 4, dtype=torch.bfloat16, device="cuda")
    hip.stem_pack_weights(w.cuda(), w4)
    torch.cuda.synchronize()
    # layout: interior = channels 0-3 of the images, pad columns and the tap-8 weights zero
    assert torch.equal(xp[:, :, 1:H + 1, :].cpu(), x[..., :4])
    assert xp[:, :, 0].abs().max().item() == 0 and xp[:, :, H + 1].abs().max().item() == 0
    assert torch.equal(w4[:, :, :7, :].cpu(), w[..., :4]) and w4[:, :, 7].abs().max().item() == 0
    ran = 0
    for cfg in range(hip.L.drn_conv_glds_num_cfgs()):
        y = torch.zeros(N, P, P, K, dtype=torch.bfloat16, device="cuda")
        st = torch.zeros(2, 2, K, device="cuda")
        a = hip.conv_args(xp, w4, y, g4, stats=st)
        a.cfg = cfg
        if hip.L.drn_conv_fwd2(ctypes.byref(a), hip.zero_page.data_ptr(), hip.stream()) != 0:
            continue
        torch.cuda.synchronize()
        assert rel(y, y_ref) < 1e-2, cfg
        s_hip = st.sum(0).view(-1).cpu()
        assert rel(s_hip[:K], st_ref[:K]) < 2e-2 and rel(s_hip[K:], st_ref[K:]) < 2e-2, cfg
        ran += 1
    assert ran >= 10  # the 64-deep one-tile configurations
    a = hip.conv_args(xp, w4, y, g4)
    a.cfg = 100  # the packed layout exists on the LDS-DMA path only: loud refusal elsewhere
    assert hip.L.drn_conv_fwd2(ctypes.byref(a), hip.zero_page.data_ptr(), hip.stream()) != 0
    # weight gradient
    dy = bf(torch.randn(N, P, P, K))
    dw_ref = torch.zeros(K, R, R, 8)
    ref.conv_wgrad(x.float(), dy.float(), dw_ref, g8)
    ws = torch.zeros(max(1, hip.wgrad_ws_elems(N * P * P, K, R, 8, 4)), device="cuda")
    old = hip.forced_wgrad_ns
    try:
        # 9 / 10: the input-halo kernel (conv_wgrad.hip stem_wgrad_halo_kernel: half output rows,
        # so an even output width; an odd one is refused)
        for ns in (2, 3, 4, 5, 6) + ((9, 10) if P % 2 == 0 else ()):
            hip.forced_wgrad_ns = ns
            dw4 = torch.zeros(K, R, 8, 4, device="cuda")
            hip.conv_wgrad(xp, dy.cuda(), dw4, g4, ws=ws)
            dw = torch.full((K, R, R, 8), 7.0, device="cuda")
            hip.stem_unpack_grad(dw4, dw)
            torch.cuda.synchronize()
            assert rel(dw, dw_ref) < 1e-2, ns
            assert dw[..., 4:].abs().max().item() == 0, ns
    finally:
        hip.forced_wgrad_ns = old
