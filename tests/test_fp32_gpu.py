"""Reference-precision (fp32) learner path on the GPU.

Kernel level: every fp32 conv (fwd / dgrad / wgrad, all ResNet-18 CIFAR
shapes at batch 32 -- i.e. the real launch plans incl. split-K and the
parity-decomposed stride-2 dgrad -- plus ragged odd shapes) is pinned against
plain PyTorch F.conv2d / conv2d_input / conv2d_weight computed in fp64 on the
host, at relative error <= 1e-5; BatchNorm, head and gather against the
host reference ops.

Model level: the fp32 ResNet-18 training step vs an independent torch.nn
ResNet-18 (tests/torch_resnet_ref.py) -- loss and EVERY per-tensor gradient
at relative error <= 1e-4, BN running statistics after the step -- and a
300-step loss trajectory where bf16 must land within 3% of fp32.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _rel(a, b):
    a, b = a.double().cpu().flatten(), b.double().cpu().flatten()
    return float((a - b).norm() / (b.norm() + 1e-300))


RESNET_SHAPES = [  # N, H, W, C, Co, k, stride
    (32, 32, 32, 8, 64, 3, 1),      # stem
    (32, 32, 32, 64, 64, 3, 1),
    (32, 32, 32, 64, 128, 3, 2),
    (32, 32, 32, 64, 128, 1, 2),
    (32, 16, 16, 128, 128, 3, 1),
    (32, 16, 16, 128, 256, 3, 2),
    (32, 16, 16, 128, 256, 1, 2),
    (32, 8, 8, 256, 256, 3, 1),
    (32, 8, 8, 256, 512, 3, 2),
    (32, 8, 8, 256, 512, 1, 2),
    (32, 4, 4, 512, 512, 3, 1),
]
ODD_SHAPES = [
    (3, 7, 7, 12, 20, 3, 1),
    (2, 9, 9, 8, 16, 3, 2),    # odd dX dims: masked (non-parity) stride-2 dgrad
    (5, 6, 10, 4, 36, 1, 1),
    (4, 10, 6, 16, 8, 1, 2),
]


@pytest.fixture(autouse=True)
def _exact_after():
    yield
    from metisfl_amd.ops import nn as K
    K.set_conv_products("exact")


@pytest.fixture(params=["exact", "bf16x3"])
def products(request):
    """Both fp32 convolution product modes (ops/nn.py set_conv_products)."""
    from metisfl_amd.ops import nn as K
    K.set_conv_products(request.param)
    yield request.param
    K.set_conv_products("exact")


def _shape(t):
    from metisfl_amd.ops.nn import ConvShape
    N, H, W, C, Co, k, s = t
    return ConvShape(N, H, W, C, Co, k, k, s, k // 2)


def _ws(shp):
    from metisfl_amd.ops import nn as K
    n = max(K.conv_plan(m, shp, torch.device(DEV), torch.float32).workspace for m in (0, 1))
    return torch.zeros(max(4, n), dtype=torch.float32, device=DEV)


@pytest.mark.parametrize("t", RESNET_SHAPES + ODD_SHAPES, ids=lambda t: "x".join(map(str, t)))
def test_conv32_forward_matches_fp64(t, products):
    from metisfl_amd.ops import nn as K
    shp = _shape(t)
    g = torch.Generator().manual_seed(hash(t) & 0xFFFF)
    x = torch.randn(shp.N, shp.H, shp.W, shp.C, generator=g)
    w = torch.randn(shp.Co, shp.R, shp.S, shp.C, generator=g) / (shp.R * shp.S * shp.C) ** 0.5
    ref = F.conv2d(x.double().permute(0, 3, 1, 2), w.double().permute(0, 3, 1, 2), stride=shp.stride,
                   padding=shp.pad).permute(0, 2, 3, 1)
    y = torch.zeros(ref.shape, dtype=torch.float32, device=DEV)
    stats = torch.zeros(2 * shp.Co, dtype=torch.float64, device=DEV)
    ws = _ws(shp)
    K.conv_forward(x.to(DEV), w.to(DEV), y, shp, ws, stats)
    torch.cuda.synchronize()
    assert _rel(y, ref) <= 1e-5
    r2 = ref.reshape(-1, shp.Co)
    if products == "exact":
        assert _rel(stats[:shp.Co], r2.sum(0)) <= 1e-5
    else:  # a channel sum cancels: bound the error by the sum of magnitudes
        err = (stats[:shp.Co].cpu() - r2.sum(0)).norm() / r2.abs().sum(0).norm()
        assert err <= 1e-5, float(err)
    assert _rel(stats[shp.Co:], (r2 * r2).sum(0)) <= 1e-5
    # the split-K counters re-arm: a second launch gives the same bits
    y2 = torch.zeros_like(y)
    K.conv_forward(x.to(DEV), w.to(DEV), y2, shp, ws, None)
    torch.cuda.synchronize()
    assert torch.equal(y, y2)


@pytest.mark.parametrize("t", [s for s in RESNET_SHAPES if s[3] != 8] + ODD_SHAPES,
                         ids=lambda t: "x".join(map(str, t)))
def test_conv32_backward_pair_matches_fp64(t, products):
    """The paired dgrad + wgrad launch (conv32_bwd_pair_kernel, or its
    two-launch fallback for shapes that do not pair) vs fp64 references."""
    from metisfl_amd.ops import nn as K
    shp = _shape(t)
    g = torch.Generator().manual_seed(11 + (hash(t) & 0xFFFF))
    x = torch.randn(shp.N, shp.H, shp.W, shp.C, generator=g)
    dy = torch.randn(shp.N, shp.P, shp.Q, shp.Co, generator=g)
    w = torch.randn(shp.Co, shp.R, shp.S, shp.C, generator=g) / (shp.R * shp.S * shp.C) ** 0.5
    ref_dx = torch.nn.grad.conv2d_input((shp.N, shp.C, shp.H, shp.W), w.double().permute(0, 3, 1, 2),
                                        dy.double().permute(0, 3, 1, 2), stride=shp.stride,
                                        padding=shp.pad).permute(0, 2, 3, 1)
    ref_dw = torch.nn.grad.conv2d_weight(x.double().permute(0, 3, 1, 2), (shp.Co, shp.C, shp.R, shp.S),
                                         dy.double().permute(0, 3, 1, 2), stride=shp.stride,
                                         padding=shp.pad).permute(0, 2, 3, 1)
    dx = torch.zeros(ref_dx.shape, dtype=torch.float32, device=DEV)
    dw = torch.zeros(ref_dw.shape, dtype=torch.float32, device=DEV)
    K.conv_backward_pair(x.to(DEV), dy.to(DEV), dw, w.to(DEV), dx, shp, _ws(shp), accumulate=False)
    torch.cuda.synchronize()
    assert _rel(dx, ref_dx) <= 1e-5
    assert _rel(dw, ref_dw) <= 1e-5


@pytest.mark.parametrize("t", [s for s in RESNET_SHAPES if s[3] != 8], ids=lambda t: "x".join(map(str, t)))
def test_conv32_pair_ring2_matches_ring3(t):
    """The 2-stage LDS ring of the paired launches (set_conv32_pair_ring,
    the co-located throughput setting) changes the pipelining only: dX and
    the forward outputs bitwise, dW to the order of its split-K atomics."""
    from metisfl_amd.ops import nn as K
    from metisfl_amd.ops._native import ops
    K.set_conv_products("bf16x3")
    shp = _shape(t)
    g = torch.Generator().manual_seed(5 + (hash(t) & 0xFFFF))
    x = torch.randn(shp.N, shp.H, shp.W, shp.C, generator=g).to(DEV)
    dy = torch.randn(shp.N, shp.P, shp.Q, shp.Co, generator=g).to(DEV)
    w = (torch.randn(shp.Co, shp.R, shp.S, shp.C, generator=g) / (shp.R * shp.S * shp.C) ** 0.5).to(DEV)
    out = []
    try:
        for ns in (3, 2):
            ops().set_conv32_pair_ring(ns)
            dx = torch.zeros(shp.N, shp.H, shp.W, shp.C, device=DEV)
            dw = torch.zeros_like(w)
            K.conv_backward_pair(x, dy, dw, w, dx, shp, _ws(shp), accumulate=False)
            fw = None
            if shp.R == 3 and shp.stride == 2:
                s2 = _shape((shp.N, shp.H, shp.W, shp.C, shp.Co, 1, 2))
                w2 = w[:, 1:2, 1:2, :].contiguous()
                y1 = torch.zeros_like(dy)
                y2 = torch.zeros_like(dy)
                K.conv_forward_pair(x, w, y1, _ws(shp), None, w2, y2, _ws(s2), None, shp)
                fw = (y1, y2)
            torch.cuda.synchronize()
            out.append((dx, dw, fw))
    finally:
        ops().set_conv32_pair_ring(0)
    (dx3, dw3, f3), (dx2, dw2, f2) = out
    assert torch.equal(dx3, dx2)
    assert _rel(dw2, dw3) <= 1e-6
    if f3 is not None:
        assert torch.equal(f3[0], f2[0]) and torch.equal(f3[1], f2[1])


@pytest.mark.parametrize("t", RESNET_SHAPES + ODD_SHAPES, ids=lambda t: "x".join(map(str, t)))
def test_conv32_dgrad_matches_fp64(t, products):
    from metisfl_amd.ops import nn as K
    shp = _shape(t)
    g = torch.Generator().manual_seed(7 + (hash(t) & 0xFFFF))
    dy = torch.randn(shp.N, shp.P, shp.Q, shp.Co, generator=g)
    w = torch.randn(shp.Co, shp.R, shp.S, shp.C, generator=g) / (shp.R * shp.S * shp.Co) ** 0.5
    ref = torch.nn.grad.conv2d_input((shp.N, shp.C, shp.H, shp.W), w.double().permute(0, 3, 1, 2),
                                     dy.double().permute(0, 3, 1, 2), stride=shp.stride,
                                     padding=shp.pad).permute(0, 2, 3, 1)
    ws = _ws(shp)
    dx = torch.zeros(ref.shape, dtype=torch.float32, device=DEV)
    K.conv_dgrad(dy.to(DEV), w.to(DEV), dx, shp, ws, accumulate=False)
    torch.cuda.synchronize()
    assert _rel(dx, ref) <= 1e-5
    # accumulate: dx += dgrad
    base = torch.randn(ref.shape, generator=g)
    dx2 = base.to(DEV)
    K.conv_dgrad(dy.to(DEV), w.to(DEV), dx2, shp, ws, accumulate=True)
    torch.cuda.synchronize()
    assert _rel(dx2, ref + base.double()) <= 1e-5


def test_conv32_dgrad_fused_bn_reductions(products):
    from metisfl_amd.ops import nn as K
    shp = _shape((32, 16, 16, 128, 128, 3, 1))
    g = torch.Generator().manual_seed(11)
    dy = torch.randn(shp.N, shp.P, shp.Q, shp.Co, generator=g)
    w = torch.randn(shp.Co, 3, 3, shp.C, generator=g) / (9 * shp.Co) ** 0.5
    z = torch.randn(shp.N, shp.H, shp.W, shp.C, generator=g)
    yv = torch.relu(torch.randn(shp.N, shp.H, shp.W, shp.C, generator=g))
    mean = torch.randn(shp.C, generator=g)
    invstd = torch.rand(shp.C, generator=g) + 0.5
    acc_c = torch.zeros(2 * shp.C, dtype=torch.float64)
    dx_c = torch.zeros(shp.N, shp.H, shp.W, shp.C)
    K.conv_dgrad(dy, w, dx_c, shp, None, False, K.BnBwdTarget(z, yv, mean, invstd, acc_c))
    acc_g = torch.zeros(2 * shp.C, dtype=torch.float64, device=DEV)
    dx_g = torch.zeros(shp.N, shp.H, shp.W, shp.C, device=DEV)
    K.conv_dgrad(dy.to(DEV), w.to(DEV), dx_g, shp, _ws(shp), False,
                 K.BnBwdTarget(z.to(DEV), yv.to(DEV), mean.to(DEV), invstd.to(DEV), acc_g))
    torch.cuda.synchronize()
    assert _rel(dx_g, dx_c) <= 1e-5
    assert _rel(acc_g, acc_c) <= 1e-5


@pytest.mark.parametrize("t", RESNET_SHAPES + ODD_SHAPES, ids=lambda t: "x".join(map(str, t)))
def test_conv32_wgrad_matches_fp64(t, products):
    from metisfl_amd.ops import nn as K
    shp = _shape(t)
    g = torch.Generator().manual_seed(3 + (hash(t) & 0xFFFF))
    x = torch.randn(shp.N, shp.H, shp.W, shp.C, generator=g)
    dy = torch.randn(shp.N, shp.P, shp.Q, shp.Co, generator=g)
    ref = torch.nn.grad.conv2d_weight(x.double().permute(0, 3, 1, 2).contiguous(),
                                      (shp.Co, shp.C, shp.R, shp.S),
                                      dy.double().permute(0, 3, 1, 2).contiguous(), stride=shp.stride,
                                      padding=shp.pad).permute(0, 2, 3, 1)
    dw = torch.full(ref.shape, 123.0, dtype=torch.float32, device=DEV)  # overwritten
    K.conv_wgrad(x.to(DEV), dy.to(DEV), dw, shp, accumulate=False)
    torch.cuda.synchronize()
    assert _rel(dw, ref) <= 1e-5
    dw2 = torch.ones(ref.shape, dtype=torch.float32, device=DEV)  # accumulate onto 1
    K.conv_wgrad(x.to(DEV), dy.to(DEV), dw2, shp, accumulate=True)
    torch.cuda.synchronize()
    assert _rel(dw2, ref + 1.0) <= 1e-5


@pytest.mark.parametrize("res,relu,train", [(False, True, True), (True, True, True), (False, False, True),
                                            (True, True, False)])
def test_bn32_apply_and_backward_match_host(res, relu, train):
    from metisfl_amd.ops import nn as K
    g = torch.Generator().manual_seed(5)
    M, C = 4096, 128
    x = torch.randn(M, C, generator=g) * 2 + 0.5
    r = torch.randn(M, C, generator=g) if res else None
    gamma = torch.rand(C, generator=g) + 0.5
    beta = torch.randn(C, generator=g)
    out = {}
    for dev in ("cpu", DEV):
        acc = torch.zeros(2 * C, dtype=torch.float64, device=dev)
        K.bn_stats(x.to(dev), C, acc)
        mean = torch.zeros(C, device=dev)
        invstd = torch.zeros(C, device=dev)
        rm = torch.full((C,), 0.1, device=dev)
        rv = torch.full((C,), 1.5, device=dev)
        y = torch.zeros(M, C, device=dev)
        K.bn_apply(x.to(dev), C, acc, gamma.to(dev), beta.to(dev), mean, invstd, rm, rv, y,
                   r.to(dev) if res else None, relu, train)
        dy = torch.randn(M, C, generator=torch.Generator().manual_seed(9)).to(dev)
        accb = torch.zeros(2 * C, dtype=torch.float64, device=dev)
        dg = torch.zeros(C, device=dev)
        db = torch.zeros(C, device=dev)
        dx = torch.zeros(M, C, device=dev)
        dym = torch.zeros(M, C, device=dev) if relu else None
        if train:
            K.bn_backward(dy, x.to(dev), y if relu else None, C, gamma.to(dev), mean, invstd, accb, dg, db,
                          dx, dym)
        out[dev] = [t.cpu() for t in (acc, mean, invstd, rm, rv, y, dg, db, dx) + ((dym,) if relu else ())]
    for a, b in zip(out["cpu"], out[DEV]):
        assert _rel(b, a) <= 1e-5


@pytest.mark.parametrize("t", [(8, 16, 16, 128, 128, 3, 1), (8, 16, 16, 64, 128, 3, 2), (8, 16, 16, 64, 128, 1, 2),
                               (8, 32, 32, 8, 64, 3, 1)], ids=lambda t: "x".join(map(str, t)))
def test_packed_dy_path_is_bit_identical(t):
    """bf16x3: the BN backward writes dz as packed hi|lo splits (dx_packed)
    and the layer's dgrad / wgrad / paired launch decode it (dy_packed) -- the
    same products as splitting an fp32 dY in the k-loop, so bit-identical
    outputs; and the packed BN output is exactly split_pack of the fp32 one."""
    from metisfl_amd.ops import nn as K
    from metisfl_amd.ops import optim as O
    prev = K.conv_products()
    K.set_conv_products("bf16x3")
    try:
        N, H, W_, C, Co, R, st = t
        shp = K.ConvShape(N, H, W_, C, Co, R, R, st, R // 2)
        g = torch.Generator().manual_seed(21)
        x = torch.randn(N, H, W_, C, generator=g).to(DEV)
        w = (torch.randn(Co, R, R, C, generator=g) / (R * R * C) ** 0.5).to(DEV)
        M = N * shp.P * shp.Q
        # the BN backward producing dz, fp32 and packed
        z = torch.randn(M, Co, generator=g).to(DEV)
        yv = torch.relu(torch.randn(M, Co, generator=g)).to(DEV)
        dout = torch.randn(M, Co, generator=g).to(DEV)
        gamma = (torch.rand(Co, generator=g) + 0.5).to(DEV)
        mean = z.mean(0)
        invstd = 1.0 / z.var(0, unbiased=False).add(1e-5).sqrt()
        dz32 = torch.zeros(M, Co, device=DEV)
        dzp = torch.zeros(M, Co, device=DEV)
        for out, pk in ((dz32, False), (dzp, True)):
            acc = torch.zeros(2 * Co, dtype=torch.float64, device=DEV)
            K.bn_backward(dout, z, yv, Co, gamma, mean, invstd, acc, None, None, out, dx_packed=pk)
        ref_pack = torch.zeros(M * Co, dtype=torch.int32, device=DEV)
        O.split_pack(dz32.reshape(-1), ref_pack)
        torch.cuda.synchronize()
        assert torch.equal(dzp.view(torch.int32).reshape(-1), ref_pack)
        dz32 = dz32.reshape(N, shp.P, shp.Q, Co)
        dzp = dzp.reshape(N, shp.P, shp.Q, Co)
        res = {}
        for pk, dz in ((False, dz32), (True, dzp)):
            dx = torch.zeros(N, H, W_, C, device=DEV)
            dw = torch.zeros(Co, R, R, C, device=DEV)
            dx2 = torch.zeros_like(dx)
            dw2 = torch.zeros_like(dw)
            if C % 32 == 0:
                K.conv_backward_pair(x, dz, dw, w, dx, shp, _ws(shp), accumulate=False, dy_packed=pk)
                K.conv_dgrad(dz, w, dx2, shp, _ws(shp), accumulate=False, dy_packed=pk)
            K.conv_wgrad(x, dz, dw2, shp, accumulate=False, dy_packed=pk)
            torch.cuda.synchronize()
            res[pk] = (dx, dw, dx2, dw2)
        # dx: deterministic split-K (slices summed in order) -> bit-identical;
        # dw: split-K slices meet in fp32 atomics, whose order varies run to run
        assert torch.equal(res[False][0], res[True][0]) and torch.equal(res[False][2], res[True][2])
        for a, b in ((res[False][1], res[True][1]), (res[False][3], res[True][3])):
            assert _rel(b, a) <= 1e-6
        # activations: the packed mirror a BN apply writes (yp) feeds the
        # forward / wgrad as xp -- same bits as packing x on the fly
        xp = torch.zeros(x.shape, dtype=torch.int32, device=DEV)
        O.split_pack(x.reshape(-1), xp.view(-1))
        y1 = torch.zeros(N, shp.P, shp.Q, Co, device=DEV)
        y2 = torch.zeros_like(y1)
        K.conv_forward(x, w, y1, shp, _ws(shp))
        K.conv_forward(x, w, y2, shp, _ws(shp), xp=xp)
        dwa = torch.zeros(Co, R, R, C, device=DEV)
        dwb = torch.zeros_like(dwa)
        K.conv_wgrad(x, dzp, dwa, shp, accumulate=False, dy_packed=True)
        K.conv_wgrad(x, dzp, dwb, shp, accumulate=False, dy_packed=True, xp=xp)
        C2 = Co
        zz = torch.randn(M, C2, generator=g).to(DEV)
        acc = torch.zeros(2 * C2, dtype=torch.float64, device=DEV)
        K.bn_stats(zz, C2, acc)
        yb = torch.zeros(M, C2, device=DEV)
        ybp = torch.zeros(M, C2, dtype=torch.int32, device=DEV)
        K.bn_apply(zz, C2, acc, gamma, gamma - 1, torch.zeros(C2, device=DEV), torch.zeros(C2, device=DEV),
                   torch.zeros(C2, device=DEV), torch.ones(C2, device=DEV), yb, relu=True, yp=ybp)
        ref_y = torch.zeros(M * C2, dtype=torch.int32, device=DEV)
        O.split_pack(yb.reshape(-1), ref_y)
        torch.cuda.synchronize()
        assert torch.equal(y1, y2)
        assert _rel(dwb, dwa) <= 1e-6
        assert torch.equal(ybp.reshape(-1), ref_y)
    finally:
        K.set_conv_products(prev)


def test_head32_and_gather32_match_host():
    from metisfl_amd.ops import nn as K
    g = torch.Generator().manual_seed(1)
    B, HW, C, NC = 32, 16, 512, 10
    x = torch.randn(B, HW, C, generator=g)
    W = torch.randn(NC, C, generator=g) * 0.05
    b = torch.randn(NC, generator=g) * 0.1
    lab = torch.randint(0, NC, (B,), generator=g, dtype=torch.int32)
    res = {}
    for dev in ("cpu", DEV):
        feat = torch.zeros(B * C, device=dev)
        dl = torch.zeros(B * NC, device=dev)
        dx = torch.zeros(B, HW, C, device=dev)
        st = torch.zeros(4, device=dev)
        dW = torch.zeros(NC, C, device=dev)
        db = torch.zeros(NC, device=dev)
        K.head_forward_backward(x.to(dev), B, HW, C, W.to(dev), b.to(dev), lab.to(dev), feat, dl, dx, st,
                                True, dW, db)
        res[dev] = [t.cpu() for t in (feat, dl, dx, st[:3], dW, db)]
    for a, c in zip(res["cpu"], res[DEV]):
        assert _rel(c, a) <= 1e-5
    # gather: fp32 rows through the permutation at the device step counter
    shard = torch.randn(64, 32, 32, 8, generator=g)
    labels = torch.randint(0, 10, (64,), generator=g, dtype=torch.int32)
    perm = torch.randperm(64, generator=g).to(torch.int32)
    step = torch.tensor([3], dtype=torch.int32)
    xb = torch.zeros(16, 32, 32, 8, device=DEV)
    yb = torch.zeros(16, dtype=torch.int32, device=DEV)
    K.gather_batch(shard.to(DEV), labels.to(DEV), perm.to(DEV), step.to(DEV), 4, 16, xb, yb)
    torch.cuda.synchronize()
    idx = perm[(3 % 4) * 16:(3 % 4 + 1) * 16].long()
    assert torch.equal(xb.cpu(), shard[idx]) and torch.equal(yb.cpu(), labels[idx])


# ---------------------------------------------------------------------------
def _x8(x):
    return F.pad(torch.as_tensor(x), (0, 5))


@pytest.mark.parametrize("conv_products", ["exact", "bf16x3", "bf16x3_halo_dgrad", "bf16x3_coloc"])
def test_fp32_resnet18_step_matches_torch_nn(conv_products, monkeypatch):
    """The whole fp32 training step (gather -> 20 conv/BN layers -> head ->
    backward) vs an independent torch.nn ResNet-18 in fp64, for both fp32
    convolution product modes (and the opt-in halo dgrad backward, and the
    co-located regime's kernel choices: models/colocated.py configure_regime
    -- fewer split-K slices for the input gradients, im2col at 4x4x512)."""
    from metisfl_amd.models import layers as L
    from metisfl_amd.models.colocated import CoLocatedLearners
    from metisfl_amd.models.resnet import ResNet18
    from metisfl_amd.ops._native import ops
    coloc = conv_products.endswith("_coloc")
    if conv_products.endswith("_halo_dgrad"):
        monkeypatch.setattr(L, "HALO_DGRAD", True)
    if coloc:
        monkeypatch.setattr(L, "HCONV_SKIP", {4})
        ops().set_conv32_plan_overrides(CoLocatedLearners.plans)
    try:
        _step_vs_torch_nn(conv_products.split("_")[0])
    finally:
        if coloc:
            ops().set_conv32_plan_overrides("")


def _step_vs_torch_nn(conv_products):
    from metisfl_amd.models.resnet import ResNet18
    from metisfl_amd.ops.optim import OptimizerSpec
    from tests.torch_resnet_ref import reference_step
    rng = np.random.default_rng(0)
    B = 32
    x = rng.standard_normal((B, 32, 32, 3)).astype(np.float32)
    y = rng.integers(0, 10, B)
    net = ResNet18(batch_size=B, device=DEV, optimizer=OptimizerSpec("vanilla_sgd", 0.0), seed=4,
                   conv_products=conv_products)
    assert net.compute_dtype == torch.float32
    values = net.state.to_numpy()
    ds = net.make_dataset(x, y, shuffle=False)
    net.zero_grad_in_optimizer = False
    net.reset_train_stats()
    net._train_body(ds)
    torch.cuda.synchronize()
    loss = net.train_stats()["loss"]
    # ReLU masks pinned to the executor's own (tests/torch_resnet_ref._relu):
    # with 2.5M ReLU'd elements per step a handful sit within fp32 rounding of
    # zero, and a flipped mask element moves its whole upstream gradient --
    # e.g. ONE flipped element of layer3.1's output put 1e-4 into every
    # gradient below it.  The flip count itself is bounded.
    masks = {n: (l.y > 0).permute(0, 3, 1, 2).cpu()
             for n, l in [("stem", net.stem)] + [(c.name, c) for b in net.blocks for c in (b.c1, b.c2)]}
    flips = [0]
    ref_loss, ref_g, ref_run = reference_step(values, _x8(x), torch.as_tensor(y), relu_masks=masks, flips=flips)
    # bf16x3 products carry ~15x the exact mode's per-element error, so
    # proportionally more near-zero pre-activations flip sign
    assert flips[0] <= (8 if conv_products == "exact" else 160), flips
    assert abs(loss - ref_loss) <= 1e-5 * max(1.0, abs(ref_loss)), (loss, ref_loss)
    worst = []
    for name, rg in ref_g.items():
        err = _rel(net.state.grad(name), rg)
        worst.append((err, name))
        assert err <= 1e-4, (name, err)
    worst.sort(reverse=True)
    print(f"mask flips {flips[0]}; worst per-tensor gradient rel err:", worst[:4])
    for name, rv in ref_run.items():
        assert _rel(net.state.view(name), rv) <= 1e-5, name


def test_bf16_resnet18_step_tracks_torch_nn():
    """The mixed-precision option against the same fp32-exact oracle: cosine
    of the whole gradient and of every conv weight gradient."""
    from metisfl_amd.models.resnet import ResNet18
    from metisfl_amd.ops.optim import OptimizerSpec
    from tests.torch_resnet_ref import reference_step
    rng = np.random.default_rng(1)
    B = 32
    x = rng.standard_normal((B, 32, 32, 3)).astype(np.float32)
    y = rng.integers(0, 10, B)
    net = ResNet18(batch_size=B, device=DEV, optimizer=OptimizerSpec("vanilla_sgd", 0.0), seed=4, dtype="bf16")
    values = net.state.to_numpy()
    ds = net.make_dataset(x, y, shuffle=False)
    net.zero_grad_in_optimizer = False
    net._train_body(ds)
    torch.cuda.synchronize()
    _, ref_g, _ = reference_step(values, _x8(x), torch.as_tensor(y))
    # floor: the exact oracle fed only bf16-ROUNDED inputs and weights -- the
    # perturbation bf16 storage alone introduces, before any bf16 arithmetic
    vb = {k: (torch.as_tensor(v).to(torch.bfloat16).double().numpy() if k.endswith("conv.weight") else v)
          for k, v in values.items()}
    _, flo_g, _ = reference_step(vb, _x8(x).to(torch.bfloat16).double(), torch.as_tensor(y))

    def cos(a, b):
        a, b = a.double().cpu().flatten(), b.double().cpu().flatten()
        return float(a @ b / (a.norm() * b.norm() + 1e-300))

    def cos_all(g):
        return cos(torch.cat([g[n].flatten().cpu() for n in ref_g]), torch.cat([ref_g[n].flatten() for n in ref_g]))

    ours = {n: net.state.grad(n) for n in ref_g}
    c_all, c_floor = cos_all(ours), cos_all(flo_g)
    per = sorted((cos(ours[n], ref_g[n]), n) for n in ref_g if n.endswith("conv.weight"))
    print(f"bf16 gradient cosine {c_all:.5f} (bf16-rounded-input oracle {c_floor:.5f}); lowest {per[:3]}")
    # at random init the net amplifies input rounding (the floor itself is
    # well below 1); the bf16 kernels may add at most as much again
    assert c_all >= min(0.99, c_floor - (1 - c_floor))


def test_loss_trajectory_bf16_within_3pct_of_fp32():
    """300 local updates on a learnable synthetic task: the bf16 final loss
    lands within 3% (or 0.02 absolute) of the fp32 one."""
    from metisfl_amd.models.resnet import ResNet18
    from metisfl_amd.ops.optim import OptimizerSpec
    rng = np.random.default_rng(0)
    n = 960
    x = rng.standard_normal((n, 32, 32, 3)).astype(np.float32)
    y = rng.integers(0, 10, n)
    x[np.arange(n), :, :, y % 3] += ((y[:, None, None] // 3) - 1.5) * 0.6
    final = {}
    for dt in ("fp32", "bf16"):
        net = ResNet18(batch_size=32, device=DEV, optimizer=OptimizerSpec("momentum_sgd", 0.01, momentum=0.75),
                       seed=7, dtype=dt)
        ds = net.make_dataset(x, y, seed=1)
        spe = ds.steps_per_epoch
        curve = []
        for ep in range(10):  # 10 x 30 = 300 updates
            net.reset_train_stats()
            net.train_steps(ds, spe, ep * spe)
            curve.append(net.train_stats()["loss"])
        final[dt] = curve[-1]
        print(dt, [round(c, 4) for c in curve])
    assert final["fp32"] < 1.0  # the task was learned
    assert abs(final["bf16"] - final["fp32"]) <= max(0.03 * final["fp32"], 0.02), final


def test_bf16x3_weight_mirror_tracks_master():
    """The packed bf16x3 weight mirror (hi << 16 | lo, written by the fused
    optimizer and read by the fwd / dgrad convolutions) equals the split of
    the fp32 master after training steps, bit for bit, and after an external
    write of the master (refresh_bf16)."""
    from metisfl_amd.models.resnet import ResNet18
    from metisfl_amd.ops import optim as opt_ops
    from metisfl_amd.ops.optim import OptimizerSpec
    net = ResNet18(batch_size=8, device=DEV, seed=3, conv_products="bf16x3",
                   optimizer=OptimizerSpec("momentum_sgd", 0.01, momentum=0.9))
    assert net.state.psplit is not None
    g = torch.Generator(device=DEV).manual_seed(0)
    x = torch.randn((64, 32, 32, 3), generator=g, device=DEV)
    y = torch.randint(0, 10, (64,), generator=g, device=DEV)
    net.train_steps(net.make_dataset(x, y), 3)
    torch.cuda.synchronize()

    def ref():
        r = torch.zeros(net.state.n_params, dtype=torch.int32)
        opt_ops.split_pack(net.state.params32.cpu(), r)
        return r
    assert torch.equal(net.state.psplit.cpu(), ref())
    net.state.params32.mul_(0.5)
    net.state.refresh_bf16()
    torch.cuda.synchronize()
    assert torch.equal(net.state.psplit.cpu(), ref())


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("B,HW,C", [(32, 16, 512), (8, 16, 256), (512, 16, 512)])
def test_split_head_matches_one_launch_head(dtype, B, HW, C, monkeypatch):
    """The split head (head.hip head_split_*: B x C/128 workgroups, two
    launches) against the one-launch head on the same inputs: the BN apply
    (y, published mean / invstd / running statistics) bit-identical, pooled
    features / logits-derived outputs to fp32 summation order."""
    from metisfl_amd.ops import nn as K
    K_ = 10
    g = torch.Generator(device="cpu").manual_seed(5)

    def mk(*shape, scale=1.0):
        return (torch.randn(*shape, generator=g) * scale).to(DEV)
    z, res = mk(B, HW, C).to(dtype), mk(B, HW, C).to(dtype)
    W, bias = mk(K_, C, scale=0.05), mk(K_, scale=0.1)
    labels = torch.randint(0, K_, (B,), generator=g).to(torch.int32).to(DEV)
    acc = torch.zeros(8 * 2 * C, dtype=torch.float64, device=DEV)
    acc[: 2 * C] = torch.cat([z.double().reshape(-1, C).sum(0), (z.double().reshape(-1, C) ** 2).sum(0)]).to(DEV)
    outs = {}
    for split in ("0", "1"):
        monkeypatch.setenv("MFL_HEAD_SPLIT", split)
        bn = K.BnParams(acc.clone(), torch.ones(C, device=DEV) * 1.1, torch.full((C,), 0.05, device=DEV),
                        torch.zeros(C, device=DEV), torch.zeros(C, device=DEV), torch.zeros(C, device=DEV),
                        torch.ones(C, device=DEV), 0.1, 1e-5)
        y = torch.empty_like(z)
        feat = torch.zeros(B * C, device=DEV)
        dlog = torch.zeros(B * K_, device=DEV)
        dx = torch.empty_like(z)
        stats = torch.zeros(4, device=DEV)
        dW, db = torch.zeros(K_, C, device=DEV), torch.zeros(K_, device=DEV)
        acc_b = torch.zeros(8 * 2 * C, dtype=torch.float64, device=DEV)
        K.head_forward_backward_bn(B, HW, C, W, bias, labels, feat, dlog, dx, stats, True, dW, db, z, res, bn,
                                   True, y, acc_b)
        torch.cuda.synchronize()
        outs[split] = dict(y=y, feat=feat, dlog=dlog, dx=dx, stats=stats, dW=dW, db=db, acc_b=acc_b,
                           mean=bn.mean, invstd=bn.invstd, rm=bn.run_mean, rv=bn.run_var)
    a, b = outs["0"], outs["1"]
    for k in ("y", "mean", "invstd", "rm", "rv"):
        assert torch.equal(a[k], b[k]), k
    for k in ("feat", "dlog", "dx", "dW", "db", "acc_b"):
        ref = a[k].double()
        rel = float((b[k].double() - ref).abs().max() / max(1e-30, float(ref.abs().max())))
        # bf16 dx: a summation-order difference can flip one bf16 rounding (2^-8)
        tol = 2e-5 if (dtype == torch.float32 or k != "dx") else 8e-3
        assert rel <= tol, (k, rel)
    assert torch.allclose(a["stats"], b["stats"], rtol=1e-5, atol=1e-3)
