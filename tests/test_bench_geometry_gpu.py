"""Bench-geometry correctness: every distinct convolution of the ResNet-50 v2 training step at the
benchmark shape (batch 128, 224 x 224) runs with the kernel configuration the
autotuner (or the tuning database) chose for it -- forward and data-gradient launches including
split-K / stream-K tiles, and weight-gradient launches with their split counts -- and is
compared with the fp32 reference of the same op (ops.backend.RefBackend on the GPU: test oracle
only) on fresh bf16-rounded random operands.

The launches are recorded from one real autotuned forward + backward of the executor at collection
time (pytest_generate_tests: one test id per distinct launch, no unused parametrised slots), so the
test covers exactly the (geometry, configuration) pairs bench.py times."""
import ctypes

import pytest
import torch

from distributed_resnet_tensorflow_amd.models.spec import build_spec
from distributed_resnet_tensorflow_amd.ops.backend import BnCfin, ConvGeom, HipBackend, OutMap, RefBackend
from distributed_resnet_tensorflow_amd.runtime.executor import Executor

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not torch.cuda.is_available(), reason="no GPU")]

BATCH = 128
_REC = {}


def _rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / b.norm().clamp_min(1e-12)).item()


def _record():
    """One autotuned ResNet-50 step; returns {key: ('fwd', args copy)} and {key: ('wgrad', ...)}."""
    if _REC:
        return _REC
    be = HipBackend("cuda")
    ex = Executor(build_spec("imagenet", 50), BATCH, be, "cuda", seed=0, weight_decay=1e-4)
    be.synthetic_images(ex.images, seed=3)
    ex.autotune()
    fwd, wg = {}, {}
    launch, wgrad = be.launch_conv, be.conv_wgrad

    def rec_launch(a):
        key = be.conv_key(a)
        if key not in fwd:
            c = type(a)()
            ctypes.memmove(ctypes.addressof(c), ctypes.addressof(a), ctypes.sizeof(a))
            fwd[key] = c
        return launch(a)

    def rec_wgrad(x, dy, out, g, in_bn=None, relu_in=True, ws=None):
        k = (tuple(x.shape), tuple(dy.shape), tuple(out.shape), g.stride, g.pad_h, g.pad_w, in_bn is not None)
        wg.setdefault(k, (g, relu_in))
        return wgrad(x, dy, out, g, in_bn=in_bn, relu_in=relu_in, ws=ws)

    be.launch_conv, be.conv_wgrad = rec_launch, rec_wgrad
    ex.forward(train=True)
    ex.backward()
    torch.cuda.synchronize()
    be.launch_conv, be.conv_wgrad = launch, wgrad
    _REC.update(be=be, ex=ex, fwd=fwd, wgrad=wg)
    return _REC


def _conv_id(k) -> str:
    N, H, W, C, K, R, S, P, Q, st, ph, pw, dil, pro, ost, res, bwd, stats = k[:18]
    tags = "".join(t for t, on in (("p", pro), ("r", res), ("b", bwd), ("s", stats), ("m", ost)) if on)
    return f"{H}x{W}x{C}-{K}-{R}x{S}s{st}d{dil}" + (f"-{tags}" if tags else "")


def _wgrad_id(k) -> str:
    xs, dys, outs, st, ph, pw, pro = k
    return f"{xs[1]}x{xs[2]}x{xs[3]}-{outs[0]}-{outs[1]}x{outs[2]}s{st}" + ("-p" if pro else "")


def pytest_generate_tests(metafunc):
    """One test per distinct launch of the recorded step (ids name the geometry)."""
    kinds = {"test_bench_geometry_conv": ("fwd", _conv_id), "test_bench_geometry_wgrad": ("wgrad", _wgrad_id)}
    if metafunc.function.__name__ not in kinds:
        return
    kind, idf = kinds[metafunc.function.__name__]
    keys = sorted(_record()[kind], key=str) if torch.cuda.is_available() else []
    metafunc.parametrize("key", keys, ids=[f"{i:02d}-{idf(k)}" for i, k in enumerate(keys)])


def test_bench_geometry_records_the_step():
    r = _record()
    assert len(r["fwd"]) > 0 and len(r["wgrad"]) > 0, (len(r["fwd"]), len(r["wgrad"]))


def test_bench_geometry_conv(key):
    r = _record()
    be, keys = r["be"], sorted(r["fwd"], key=str)
    i = keys.index(key)
    a0 = r["fwd"][keys[i]]
    N, H, W, C, K, R, S, P, Q = a0.N, a0.H, a0.W, a0.C, a0.K, a0.R, a0.S, a0.P, a0.Q
    torch.manual_seed(i)
    dev = "cuda"
    C_store = C
    x = torch.randn(N, H, W, C_store, device=dev).bfloat16()
    if C == 4:  # packed stem input: 4 channels, the 4th a zero pad (RGB)
        x[..., 3] = 0
    w = (torch.randn(K, R, S, C_store, device=dev) * (2.0 / (R * S * C_store)) ** 0.5).bfloat16()
    mapped = a0.out_stride != 0
    oH, oW = (a0.out_H, a0.out_W) if mapped else (P, Q)
    om = OutMap(P, Q, a0.out_stride, a0.out_oh, a0.out_ow) if mapped else None
    g = ConvGeom(a0.stride, a0.pad_h, a0.pad_w, a0.dil)
    in_bn = (torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev) * 0.3) if a0.in_scale else None
    fin = None
    G = keys[i][-1]  # the recorded launch finalized its input BN in the prologue from G replicas
    if G:
        # replica sums of a known per-channel mean / variance (all in replica 0); the reference
        # applies the scale / shift they finalize to
        n = float(N * H * W)
        mu, var = torch.randn(C, device=dev) * 0.3, torch.rand(C, device=dev) + 0.5
        gamma, beta = torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev) * 0.3
        stats = torch.zeros(G, 2, C, device=dev)
        stats[0, 0], stats[0, 1] = mu * n, (var + mu * mu) * n
        fin = BnCfin(stats, n, gamma, beta=beta, publish=False)
        sc = gamma / torch.sqrt(var + fin.eps)
        in_bn = (sc, beta - mu * sc)
    res = torch.randn(N, oH, oW, K, device=dev).bfloat16() if a0.residual else None
    bb = None
    if a0.bn_x:
        bb = (torch.randn(N, oH, oW, K, device=dev).bfloat16(), torch.rand(K, device=dev) + 0.5,
              torch.randn(K, device=dev) * 0.3, torch.randn(K, device=dev) * 0.1, torch.rand(K, device=dev) + 0.5)
    rep = max(1, a0.stats_rep)
    st = torch.zeros(rep, 2, K, device=dev) if a0.stats else None
    y = torch.zeros(N, oH, oW, K, device=dev, dtype=torch.bfloat16)
    if res is not None and mapped:
        y.copy_(res)            # accumulating phase launch: residual == output
        res = y
    a = be.conv_args(x, w, y, g, in_bn=in_bn, residual=res, stats=st, out_map=om, bn_bwd=bb, in_fin=fin)
    assert be.conv_key(a) == keys[i]
    cfg = be.conv_cfg.get(keys[i])
    assert cfg is not None, "the benchmark launch was not tuned"
    res_ref = None if res is None else res.float().clone()
    be.launch_conv(a)
    torch.cuda.synchronize()
    ref = RefBackend(dev)
    y_ref = torch.zeros(N, oH, oW, K, device=dev)
    if res_ref is not None and mapped:
        y_ref.copy_(res_ref)
    st_ref = torch.zeros(2 * K, device=dev) if st is not None else None
    ref.conv_fwd(x.float(), w.float(), y_ref, g, in_bn=in_bn, residual=res_ref, stats=st_ref, out_map=om,
                 bn_bwd=None if bb is None else (bb[0].float(),) + bb[1:])
    assert _rel(y, y_ref) < 1e-2, (keys[i], cfg)
    if st is not None:
        s = st.sum(0).view(-1)
        tol = 3e-2 if bb is not None else 2e-2
        assert _rel(s[:K], st_ref[:K]) < tol and _rel(s[K:], st_ref[K:]) < tol, (keys[i], cfg)


def test_bench_geometry_wgrad(key):
    r = _record()
    be, ex = r["be"], r["ex"]
    keys = sorted(r["wgrad"], key=str)
    i = keys.index(key)
    k = key
    xs, dys, outs, _, _, _, pro = k
    g, relu_in = r["wgrad"][k]
    torch.manual_seed(1000 + i)
    dev = "cuda"
    x = torch.randn(*xs, device=dev).bfloat16()
    dy = torch.randn(*dys, device=dev).bfloat16()
    C = xs[-1]
    in_bn = (torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev) * 0.3) if pro else None
    out = torch.zeros(*outs, device=dev)
    be.conv_wgrad(x, dy, out, g, in_bn=in_bn, relu_in=relu_in, ws=ex.wgrad_ws)
    torch.cuda.synchronize()
    out_ref = torch.zeros(*outs, device=dev)
    RefBackend(dev).conv_wgrad(x.float(), dy.float(), out_ref, g, in_bn=in_bn, relu_in=relu_in)
    assert _rel(out, out_ref) < 1e-2, (k, be.wgrad_ns.get(be.wgrad_key(be.wgrad_args(x, dy, out, g, in_bn))))
