"""Halo-tiled fp32 convolution with the producer's BatchNorm fused into the
operand fill (kernels/hconv.hip) on the GPU.

Every ResNet-18 3x3 / stride-1 stage at batch 32, each residual kind (none,
fp32 tensor, BN of a projection shortcut), train and eval:
* the output is pinned against F.conv2d in fp64 of the reference activation
  at relative error <= 1e-5 (bf16x3 products, like conv32's c32s);
* the activation the owner tiles write (y, packed yp) and the published
  BatchNorm statistics / running averages are BIT-identical to the fp32
  BatchNorm apply (bn32_apply) the fill replaces;
* the output's BN sums match the fp64 sums of the reference output.
"""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda"
STAGES = [(32, 32, 64), (16, 16, 128), (8, 8, 256), (4, 4, 512)]


def _rel(a, b):
    a, b = a.double().cpu().flatten(), b.double().cpu().flatten()
    return float((a - b).norm() / (b.norm() + 1e-300))


def _bn(C, g, z, reps=8):
    from metisfl_amd.ops import nn as K
    zf = z.reshape(-1, C).double()
    acc = torch.zeros(reps, 2, C, dtype=torch.float64)
    # spread the sums over the replicas like the producing epilogue does
    acc[0, 0] = zf[0::2].sum(0)
    acc[0, 1] = (zf[0::2] ** 2).sum(0)
    acc[reps - 1, 0] = zf[1::2].sum(0)
    acc[reps - 1, 1] = (zf[1::2] ** 2).sum(0)
    return K.BnParams(acc.reshape(-1).to(DEV),
                      (0.5 + torch.rand(C, generator=g)).to(DEV), (0.2 * torch.randn(C, generator=g)).to(DEV),
                      torch.zeros(C, device=DEV), torch.zeros(C, device=DEV),
                      (0.1 * torch.randn(C, generator=g)).to(DEV), (0.5 + torch.rand(C, generator=g)).to(DEV))


def _clone(b):
    from metisfl_amd.ops import nn as K
    return K.BnParams(b.acc, b.gamma, b.beta, b.mean.clone(), b.invstd.clone(), b.run_mean.clone(),
                      b.run_var.clone(), b.momentum, b.eps)


@pytest.mark.parametrize("train", [True, False], ids=["train", "eval"])
@pytest.mark.parametrize("rk", [0, 1, 2], ids=["nores", "res", "bnres"])
@pytest.mark.parametrize("st", STAGES, ids=lambda s: f"{s[0]}x{s[1]}x{s[2]}")
def test_hconv_forward_fused_bn(st, rk, train):
    from metisfl_amd.ops import nn as K
    from metisfl_amd.ops.optim import split_pack
    H, W, C = st
    N = 32
    shp = K.ConvShape(N, H, W, C, C, 3, 3, 1, 1)
    ws_n = K.hconv_workspace(shp, torch.device(DEV))
    assert ws_n >= 0
    g = torch.Generator().manual_seed(1000 * H + 10 * rk + int(train))
    z = (torch.randn(N, H, W, C, generator=g) * 1.5 + 0.3).to(DEV)
    w = (torch.randn(C, 3, 3, C, generator=g) / (9 * C) ** 0.5).to(DEV)
    wp = torch.zeros(w.numel(), dtype=torch.int32, device=DEV)
    split_pack(w.reshape(-1), wp)
    bn = _bn(C, g, z.cpu())
    res = zr = bnr = None
    if rk == 1:
        res = torch.randn(N, H, W, C, generator=g).to(DEV)
    elif rk == 2:
        zr = (torch.randn(N, H, W, C, generator=g) - 0.2).to(DEV)
        bnr = _bn(C, g, zr.cpu())
    # reference: the BatchNorm apply(s) the fill replaces (bn32_apply)
    bn_ref, bnr_ref = _clone(bn), (_clone(bnr) if bnr is not None else None)
    r = res
    if rk == 2:
        r = torch.empty_like(zr)
        K.bn_apply(zr, C, bnr_ref.acc, bnr_ref.gamma, bnr_ref.beta, bnr_ref.mean, bnr_ref.invstd,
                   bnr_ref.run_mean, bnr_ref.run_var, r, relu=False, train=train)
    y_ref = torch.empty_like(z)
    yp_ref = torch.empty(z.shape, dtype=torch.int32, device=DEV)
    K.bn_apply(z, C, bn_ref.acc, bn_ref.gamma, bn_ref.beta, bn_ref.mean, bn_ref.invstd, bn_ref.run_mean,
               bn_ref.run_var, y_ref, residual=r, relu=True, train=train, yp=yp_ref)
    out_ref = F.conv2d(y_ref.double().cpu().permute(0, 3, 1, 2), w.double().cpu().permute(0, 3, 1, 2),
                       padding=1).permute(0, 2, 3, 1)
    # the fused launch
    out = torch.zeros(N, H, W, C, device=DEV)
    y = torch.zeros_like(z)
    yp = torch.zeros(z.shape, dtype=torch.int32, device=DEV)
    stats = torch.zeros(8 * 2 * C, dtype=torch.float64, device=DEV) if train else None
    ws = torch.zeros(max(4, ws_n), device=DEV)
    K.hconv_forward(z, wp, w, out, shp, bn, train, True, ws=ws, stats=stats, res=res, zr=zr, bnr=bnr, y=y, yp=yp)
    torch.cuda.synchronize()
    assert _rel(out, out_ref) <= 1e-5
    assert torch.equal(y, y_ref)
    assert torch.equal(yp, yp_ref)
    for a, b in [(bn, bn_ref)] + ([(bnr, bnr_ref)] if bnr is not None else []):
        for f in ("mean", "invstd", "run_mean", "run_var"):
            assert torch.equal(getattr(a, f), getattr(b, f)), f
    if train:
        s = stats.reshape(8, 2, C).sum(0).cpu()
        o2 = out_ref.reshape(-1, C)
        err = (s[0] - o2.sum(0)).norm() / o2.abs().sum(0).norm()
        assert err <= 1e-5, float(err)
        assert _rel(s[1], (o2 * o2).sum(0)) <= 1e-5
    # split-K tickets re-arm: a second launch gives the same bits
    out2 = torch.zeros_like(out)
    K.hconv_forward(z, wp, w, out2, shp, _clone(bn), train, True, ws=ws, res=res, zr=zr,
                    bnr=_clone(bnr) if bnr is not None else None)
    torch.cuda.synchronize()
    assert torch.equal(out, out2)


@pytest.mark.parametrize("mode", ["mask_bnb", "mask_accum_bnb", "plain"])
@pytest.mark.parametrize("st", STAGES, ids=lambda s: f"{s[0]}x{s[1]}x{s[2]}")
def test_hconv_dgrad_fused_bn_backward(st, mode):
    """dx (+)= conv3x3^T(BN_bwd(dy [* mask]), W) in one launch vs the fp32
    BatchNorm backward (bn32) it replaces + an fp64 transposed convolution:
    dx <= 1e-5, the packed dz (wgrad operand), the masked gradient and
    dgamma / dbeta bit-identical, the consumer-BN sums <= 1e-5."""
    from metisfl_amd.ops import nn as K
    from metisfl_amd.ops.optim import split_pack
    H, W, C = st
    N = 32
    mask, accum, bnb_on = "mask" in mode, "accum" in mode, "bnb" in mode
    shp = K.ConvShape(N, H, W, C, C, 3, 3, 1, 1)
    ws_n = K.hconv_workspace(shp, torch.device(DEV))
    g = torch.Generator().manual_seed(7 * H + len(mode))
    dy = torch.randn(N, H, W, C, generator=g).to(DEV)
    z = (torch.randn(N, H, W, C, generator=g) * 1.3 + 0.2).to(DEV)
    ym = torch.randn(N, H, W, C, generator=g).clamp_min(0).to(DEV) if mask else None
    w = (torch.randn(C, 3, 3, C, generator=g) / (9 * C) ** 0.5).to(DEV)
    wp = torch.zeros(w.numel(), dtype=torch.int32, device=DEV)
    split_pack(w.reshape(-1), wp)
    mean = (0.1 * torch.randn(C, generator=g)).to(DEV)
    invstd = (0.5 + torch.rand(C, generator=g)).to(DEV)
    gamma = (0.5 + torch.rand(C, generator=g)).to(DEV)
    # complete sums of g and g * xhat, spread over two of 8 replicas
    gd = (dy * (ym > 0) if mask else dy).reshape(-1, C).double().cpu()
    xh = ((z - mean) * invstd).reshape(-1, C).double().cpu()
    acc = torch.zeros(8, 2, C, dtype=torch.float64)
    acc[0, 0], acc[0, 1] = gd[0::2].sum(0), (gd[0::2] * xh[0::2]).sum(0)
    acc[7, 0], acc[7, 1] = gd[1::2].sum(0), (gd[1::2] * xh[1::2]).sum(0)
    acc = acc.reshape(-1).to(DEV)
    bn = K.BnParams(acc, gamma, torch.zeros(C, device=DEV), mean, invstd, None, None)
    # reference: bn32's backward apply (fp32 dz, packed dz, masked g)
    dz_ref = torch.empty_like(z)
    dres_ref = torch.empty_like(z) if mask else None
    dg_ref, db_ref = torch.zeros(C, device=DEV), torch.zeros(C, device=DEV)
    K.bn_backward(dy, z, ym, C, gamma, mean, invstd, acc, dg_ref, db_ref, dz_ref, dy_masked=dres_ref, presummed=True)
    dzp_ref = torch.empty(z.shape, dtype=torch.int32, device=DEV)
    K.bn_backward(dy, z, ym, C, gamma, mean, invstd, acc, None, None, dzp_ref, presummed=True, dx_packed=True)
    out0 = torch.randn(N, H, W, C, generator=g).to(DEV) if accum else torch.zeros(N, H, W, C, device=DEV)
    out_ref = F.conv_transpose2d(dz_ref.double().cpu().permute(0, 3, 1, 2), w.double().cpu().permute(0, 3, 1, 2),
                                 padding=1).permute(0, 2, 3, 1) + out0.double().cpu()
    bnb = None
    if bnb_on:
        zp = torch.randn(N, H, W, C, generator=g).to(DEV)
        yp_ = torch.randn(N, H, W, C, generator=g).clamp_min(0).to(DEV)
        bnb = K.BnBwdTarget(zp, yp_, (0.1 * torch.randn(C, generator=g)).to(DEV),
                            (0.5 + torch.rand(C, generator=g)).to(DEV),
                            torch.zeros(8 * 2 * C, dtype=torch.float64, device=DEV))
    # the fused launch
    out = out0.clone()
    dzp = torch.zeros(z.shape, dtype=torch.int32, device=DEV)
    dres = torch.zeros_like(z) if mask else None
    dgam, dbet = torch.zeros(C, device=DEV), torch.zeros(C, device=DEV)
    ws = torch.zeros(max(4, ws_n), device=DEV)
    K.hconv_dgrad(dy, ym, z, wp, w, out, shp, bn, dgamma=dgam, dbeta=dbet, ws=ws, dres=dres, dzp=dzp,
                  accumulate=accum, bnb=bnb)
    torch.cuda.synchronize()
    assert _rel(out, out_ref) <= 1e-5
    assert torch.equal(dzp, dzp_ref)
    if mask:
        assert torch.equal(dres, dres_ref)
    assert torch.equal(dgam, dg_ref) and torch.equal(dbet, db_ref)
    if bnb_on:
        o2 = out_ref.reshape(-1, C)
        gk = o2 * (bnb.y.double().cpu().reshape(-1, C) > 0)
        xk = ((bnb.z.double().cpu() - bnb.mean.double().cpu()) * bnb.invstd.double().cpu()).reshape(-1, C)
        s = bnb.acc.reshape(8, 2, C).sum(0).cpu()
        assert (s[0] - gk.sum(0)).norm() / gk.abs().sum(0).norm() <= 1e-5
        assert (s[1] - (gk * xk).sum(0)).norm() / (gk * xk).abs().sum(0).norm() <= 1e-5
    # split-K tickets re-arm: a second launch gives the same bits
    out2 = out0.clone()
    K.hconv_dgrad(dy, ym, z, wp, w, out2, shp, bn, ws=ws, accumulate=accum)
    torch.cuda.synchronize()
    assert torch.equal(out, out2)


@pytest.mark.parametrize("rk", [0, 1, 2], ids=["nores", "res", "bnres"])
@pytest.mark.parametrize("st", STAGES, ids=lambda s: f"{s[0]}x{s[1]}x{s[2]}")
def test_hconv_forward_bf16_option(st, rk):
    """The bf16 option's halo conv (bf16 activations / weights / output, one
    bf16 product): against a plain PyTorch reference of the same op -- the
    BatchNorm (+ residual) + ReLU in fp32 from the fp64 sums, rounded to bf16,
    then the convolution in fp64 of the bf16 operands."""
    from metisfl_amd.ops import nn as K
    H, W, C = st
    N = 32
    shp = K.ConvShape(N, H, W, C, C, 3, 3, 1, 1)
    ws_n = K.hconv_workspace(shp, torch.device(DEV))
    assert ws_n >= 0
    g = torch.Generator().manual_seed(7000 + 1000 * H + rk)
    z = (torch.randn(N, H, W, C, generator=g) * 1.5 + 0.3).to(torch.bfloat16).to(DEV)
    w = (torch.randn(C, 3, 3, C, generator=g) / (9 * C) ** 0.5).to(torch.bfloat16).to(DEV)
    bn = _bn(C, g, z.float().cpu())
    res = zr = bnr = None
    if rk == 1:
        res = torch.randn(N, H, W, C, generator=g).to(torch.bfloat16).to(DEV)
    elif rk == 2:
        zr = (torch.randn(N, H, W, C, generator=g) - 0.2).to(torch.bfloat16).to(DEV)
        bnr = _bn(C, g, zr.float().cpu())
    M = N * H * W

    def coef(b, x):
        acc = b.acc.cpu().reshape(-1, 2, C).sum(0)
        mu = acc[0] / M
        var = (acc[1] / M - mu * mu).clamp_min(0)
        isd = 1.0 / torch.sqrt(var + b.eps)
        gm, bt = b.gamma.cpu().double(), b.beta.cpu().double()
        sc, sh = (gm * isd).float(), (bt - mu * gm * isd).float()
        return x.float().cpu() * sc + sh, mu, isd

    v, mu, isd = coef(bn, z)
    if rk == 1:
        v = v + res.float().cpu()
    elif rk == 2:
        v = v + coef(bnr, zr)[0]
    y_ref = v.clamp_min(0).to(torch.bfloat16)
    out_ref = F.conv2d(y_ref.double().permute(0, 3, 1, 2), w.double().cpu().permute(0, 3, 1, 2),
                       padding=1).permute(0, 2, 3, 1)
    out = torch.zeros(N, H, W, C, dtype=torch.bfloat16, device=DEV)
    y = torch.zeros_like(z)
    stats = torch.zeros(2 * C, dtype=torch.float64, device=DEV)
    ws = torch.zeros(max(4, ws_n), device=DEV)
    K.hconv_forward(z, None, w, out, shp, bn, True, True, ws=ws, stats=stats, res=res, zr=zr, bnr=bnr, y=y)
    torch.cuda.synchronize()
    # bf16 output rounding: ~2^-9 per element
    assert _rel(out, out_ref) <= 3e-3, _rel(out, out_ref)
    assert _rel(y, y_ref) <= 2e-3
    assert _rel(bn.mean, mu) <= 1e-6 and _rel(bn.invstd, isd) <= 1e-6
    o2 = out.double().cpu().reshape(-1, C)  # the sums are of the stored (rounded) output
    s = stats.reshape(2, C).cpu()
    assert (s[0] - o2.sum(0)).norm() / o2.abs().sum(0).norm() <= 1e-5
    assert _rel(s[1], (o2 * o2).sum(0)) <= 1e-5
    out2 = torch.zeros_like(out)
    K.hconv_forward(z, None, w, out2, shp, _clone(bn), True, True, ws=ws, res=res, zr=zr,
                    bnr=_clone(bnr) if bnr is not None else None)
    torch.cuda.synchronize()
    assert torch.equal(out, out2)
