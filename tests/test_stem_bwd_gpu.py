"""Fused stem backward (bn32.hip stem_bwd32_kernel): the stem's BatchNorm(+ReLU)
backward and its 3x3 weight gradient in one launch.  Pinned against the same
math in fp64 on the host (dw at relative error <= 1e-5: exact fp32 products,
fp32 partial sums) and against the two-launch GPU path it replaces
(bn32_bwd_apply + conv32 wgrad); dgamma / dbeta come from the same replica
sums and must be bit-identical to bn32_bwd_apply's."""
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _rel(a, b):
    a, b = a.double().cpu().flatten(), b.double().cpu().flatten()
    return float((a - b).norm() / (b.norm() + 1e-300))


def _case(N, seed=0, reps=8, zero_pad_channels=True):
    g = torch.Generator().manual_seed(seed)
    H = W = 32
    Ci, Co = 8, 64
    x = torch.randn(N, H, W, Ci, generator=g)
    if zero_pad_channels:
        x[..., 3:] = 0  # the stem's zero-padded RGB input
    z = torch.randn(N, H, W, Co, generator=g) * 1.7 + 0.3
    mean = z.reshape(-1, Co).mean(0)
    invstd = 1.0 / (z.reshape(-1, Co).var(0, unbiased=False) + 1e-5).sqrt()
    gamma = torch.rand(Co, generator=g) + 0.5
    beta = torch.randn(Co, generator=g) * 0.1
    y = torch.relu((z - mean) * invstd * gamma + beta)
    dy = torch.randn(N, H, W, Co, generator=g) * 1e-2
    # the presummed backward sums (g = dy [y > 0]), split over `reps` replicas
    gm = torch.where(y > 0, dy, torch.zeros(())).reshape(-1, Co).double()
    xh = ((z - mean) * invstd).reshape(-1, Co).double()
    tot = torch.stack([gm.sum(0), (gm * xh).sum(0)])  # [2][Co]
    parts = torch.rand(reps, 1, Co, generator=g, dtype=torch.float64)
    parts = parts / parts.sum(0, keepdim=True)
    acc = (parts * tot).reshape(-1)
    return dict(x=x, z=z, y=y, dy=dy, gamma=gamma, mean=mean, invstd=invstd, acc=acc, tot=tot)


def _ref_dw(c):
    """fp64 host reference: dz = gamma invstd (g - mean g - xhat mean(g xhat)),
    dw = conv2d_weight(x, dz)."""
    Co = c["z"].shape[-1]
    M = c["z"].numel() // Co
    g = torch.where(c["y"] > 0, c["dy"], torch.zeros(())).double()
    xh = ((c["z"] - c["mean"]) * c["invstd"]).double()
    k1 = (c["gamma"] * c["invstd"]).double()
    dz = k1 * (g - c["tot"][0] / M - xh * (c["tot"][1] / M))
    xn = c["x"].double().permute(0, 3, 1, 2).contiguous()
    dzn = dz.permute(0, 3, 1, 2).contiguous()
    dw = torch.nn.grad.conv2d_weight(xn, (Co, xn.shape[1], 3, 3), dzn, stride=1, padding=1)
    return dw.permute(0, 2, 3, 1).contiguous()  # KRSC


@pytest.mark.parametrize("N", [32, 8, 3])
def test_stem_backward_fused_matches_fp64(N):
    from metisfl_amd.ops import nn as K
    c = _case(N, seed=N)
    shp = K.ConvShape(N, 32, 32, 8, 64, 3, 3, 1, 1)
    assert K.stem_backward_ok(shp, torch.device(DEV))
    d = {k: v.to(DEV) for k, v in c.items()}
    dw = torch.zeros(64, 3, 3, 8, device=DEV)
    dgamma = torch.zeros(64, device=DEV)
    dbeta = torch.zeros(64, device=DEV)
    K.stem_backward(d["dy"], d["z"], d["y"], d["x"], shp, d["gamma"], d["mean"], d["invstd"], d["acc"], dgamma,
                    dbeta, dw)
    torch.cuda.synchronize()
    ref = _ref_dw(c)
    assert _rel(dw, ref) <= 1e-5, _rel(dw, ref)
    assert dw[..., 3:].abs().max().item() == 0.0  # zero-padded input channels get no gradient

    # the two-launch path it replaces: bn32_bwd_apply (fp32 dz) + exact conv32 wgrad
    prev = K.conv_products()
    K.set_conv_products("exact")
    dz = torch.empty_like(d["z"])
    dg2 = torch.zeros(64, device=DEV)
    db2 = torch.zeros(64, device=DEV)
    K.bn_backward(d["dy"], d["z"], d["y"], 64, d["gamma"], d["mean"], d["invstd"], d["acc"].clone(), dg2, db2, dz,
                  presummed=True)
    dw2 = torch.zeros(64, 3, 3, 8, device=DEV)
    K.conv_wgrad(d["x"], dz, dw2, shp, accumulate=True)
    torch.cuda.synchronize()
    assert torch.equal(dgamma, dg2) and torch.equal(dbeta, db2)
    assert _rel(dw, dw2) <= 1e-5, _rel(dw, dw2)
    K.set_conv_products(prev)


def test_stem_backward_accumulates_and_rejects_other_shapes():
    from metisfl_amd.ops import nn as K
    c = _case(4, seed=11, reps=1, zero_pad_channels=False)
    shp = K.ConvShape(4, 32, 32, 8, 64, 3, 3, 1, 1)
    d = {k: v.to(DEV) for k, v in c.items()}
    base = torch.randn(64, 3, 3, 8, device=DEV)
    dw = base.clone()
    K.stem_backward(d["dy"], d["z"], d["y"], d["x"], shp, d["gamma"], d["mean"], d["invstd"], d["acc"], None, None,
                    dw)
    torch.cuda.synchronize()
    ref = _ref_dw(c)
    assert _rel(dw - base, ref) <= 1e-5
    dev = torch.device(DEV)
    assert not K.stem_backward_ok(K.ConvShape(4, 32, 32, 16, 64, 3, 3, 1, 1), dev)  # Cin
    assert not K.stem_backward_ok(K.ConvShape(4, 16, 16, 8, 64, 3, 3, 1, 1), dev)   # 16-pixel rows
    assert not K.stem_backward_ok(K.ConvShape(4, 32, 32, 8, 64, 3, 3, 2, 1), dev)   # stride 2



def test_stem_backward_fused_bf16_option():
    """The bf16 option's tensors (dy, z, y, x bf16) through the same launch:
    against the fp64 reference of the bf16-rounded inputs (dz and the products
    stay fp32 inside the kernel)."""
    from metisfl_amd.ops import nn as K
    N = 32
    c = _case(N, seed=77)
    for k in ("x", "z", "y", "dy"):
        c[k] = c[k].to(torch.bfloat16).float()  # what the kernel sees
    shp = K.ConvShape(N, 32, 32, 8, 64, 3, 3, 1, 1)
    d = {k: (v.to(torch.bfloat16) if k in ("x", "z", "y", "dy") else v).to(DEV) for k, v in c.items()}
    dw = torch.zeros(64, 3, 3, 8, device=DEV)
    dgamma = torch.zeros(64, device=DEV)
    dbeta = torch.zeros(64, device=DEV)
    K.stem_backward(d["dy"], d["z"], d["y"], d["x"], shp, d["gamma"], d["mean"], d["invstd"], d["acc"], dgamma,
                    dbeta, dw)
    torch.cuda.synchronize()
    ref = _ref_dw(c)
    assert _rel(dw, ref) <= 1e-5, _rel(dw, ref)
    assert _rel(dbeta, c["tot"][0]) <= 1e-6 and _rel(dgamma, c["tot"][1]) <= 1e-6
