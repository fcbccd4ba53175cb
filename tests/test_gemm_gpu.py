"""K7b large-tile GEMM (gemm_big.hip) vs fp32 PyTorch references on the
BERT-base projection shapes, all three layouts (fwd NT + epilogue, dgrad
NN, wgrad TN into fp32), and agreement with the conv-core GEMM path."""
import pytest
import torch

pytestmark = pytest.mark.gpu

SHAPES = [(512, 768, 768), (1024, 3072, 768), (512, 768, 3072), (256, 2304, 768),
          (2560, 2112, 768)]  # ragged N (the MLM decoder's vocabulary is 30,528 wide)


def _ops():
    from metisfl_amd.ops._native import ops
    return ops()


def _rel(a, b):
    return float((a.float() - b.float()).norm() / (b.float().norm() + 1e-12))


@pytest.fixture(autouse=True)
def big_on():
    _ops().set_gemm_big(True)
    yield
    _ops().set_gemm_big(True)


@pytest.mark.parametrize("M,N,K", SHAPES)
def test_fwd_bias_resid_gelu(M, N, K):
    g = torch.Generator(device="cuda").manual_seed(M + N + K)
    x = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    w = (torch.randn(N, K, device="cuda", generator=g) * 0.05).bfloat16()
    bias = torch.randn(N, device="cuda", generator=g)
    resid = torch.randn(M, N, device="cuda", generator=g).bfloat16()
    y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    act = torch.empty_like(y)
    _ops().gemm_fwd(x, w, y, bias, resid, act, M, N, K)
    ref = x.float() @ w.float().t() + bias + resid.float()
    assert _rel(y, ref) < 1e-2
    assert _rel(act, torch.nn.functional.gelu(y.float())) < 1e-2
    # plain forward, no epilogue
    _ops().gemm_fwd(x, w, y, None, None, None, M, N, K)
    assert _rel(y, x.float() @ w.float().t()) < 1e-2


@pytest.mark.parametrize("M,N,K", SHAPES)
def test_dgrad_accumulate(M, N, K):
    g = torch.Generator(device="cuda").manual_seed(7 * M + N)
    dy = torch.randn(M, N, device="cuda", generator=g).bfloat16()
    w = (torch.randn(N, K, device="cuda", generator=g) * 0.05).bfloat16()
    dx = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    base = dx.float().clone()
    _ops().gemm_dgrad(dy, w, dx, M, N, K, True)
    assert _rel(dx, base + dy.float() @ w.float()) < 1e-2
    _ops().gemm_dgrad(dy, w, dx, M, N, K, False)
    assert _rel(dx, dy.float() @ w.float()) < 1e-2


@pytest.mark.parametrize("M,N,K", SHAPES)
def test_wgrad_fp32_accumulate(M, N, K):
    g = torch.Generator(device="cuda").manual_seed(3 * M + K)
    x = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    dy = torch.randn(M, N, device="cuda", generator=g).bfloat16()
    dw = torch.randn(N, K, device="cuda", generator=g)
    base = dw.clone()
    _ops().gemm_wgrad(x, dy, dw, M, N, K, True, False)
    ref = dy.float().t() @ x.float()
    assert _rel(dw - base, ref) < 2e-3
    _ops().gemm_wgrad(x, dy, dw, M, N, K, False, False)
    assert _rel(dw, ref) < 2e-3


def test_big_and_conv_paths_agree():
    M, N, K = 1024, 768, 3072
    g = torch.Generator(device="cuda").manual_seed(11)
    x = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    w = (torch.randn(N, K, device="cuda", generator=g) * 0.05).bfloat16()
    outs = []
    for on in (True, False):
        _ops().set_gemm_big(on)
        y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        _ops().gemm_fwd(x, w, y, None, None, None, M, N, K)
        dw = torch.zeros(N, K, device="cuda")
        _ops().gemm_wgrad(x, y, dw, M, N, K, False, False)
        outs.append((y.float(), dw))
    assert _rel(outs[0][0], outs[1][0]) < 1e-2
    assert _rel(outs[0][1], outs[1][1]) < 1e-2


@pytest.mark.parametrize("on", [True, False])
def test_dgrad_gelu_fused_epilogue(on):
    """FFN1 backward in one launch: dz = (dy W) * gelu'(z), dbias += colsum(dz);
    large-tile fused epilogue (on) and the dgrad + gelu_bwd fallback (off)."""
    from metisfl_amd.ops import bert as BO
    _ops().set_gemm_big(on)
    M, N, K = 1024, 768, 3072
    g = torch.Generator(device="cuda").manual_seed(21)
    dy = torch.randn(M, N, device="cuda", generator=g).bfloat16()
    w = (torch.randn(N, K, device="cuda", generator=g) * 0.05).bfloat16()
    z = (torch.randn(M, K, device="cuda", generator=g) * 2).bfloat16()
    dz = torch.empty(M, K, device="cuda", dtype=torch.bfloat16)
    db = torch.full((K,), 0.25, device="cuda")
    BO.gemm_dgrad_gelu(dy, w, dz, z, M, N, K, dbias=db)
    dh = dy.float() @ w.float()
    ref = dh * BO.gelu_grad_ref(z.float())
    assert _rel(dz, ref) < 1e-2
    assert _rel(db - 0.25, ref.sum(0)) < 1e-2


@pytest.mark.parametrize("width", ["192", "256"])
@pytest.mark.parametrize("M,N,K", [(512, 768, 768), (768, 2304, 1536), (2560, 2112, 768)])
def test_pp_tile_widths(width, M, N, K, monkeypatch):
    """The ping-pong kernel's 256x192 and 256x256 tiles, forced (MFL_GB_WIDTH),
    on all three layouts -- including the transposing-read B1 half-tile of
    the 192-wide tile (dgrad / wgrad) and a ragged M."""
    monkeypatch.setenv("MFL_GB_WIDTH", width)
    test_fwd_bias_resid_gelu(M, N, K)
    test_dgrad_accumulate(M, N, K)
    test_wgrad_fp32_accumulate(M, N, K)


@pytest.mark.parametrize("M", [16384, 2048, 1024])
def test_grouped_wgrad_pair(M):
    """The BERT attention-output + QKV weight gradients in one grouped launch
    (gemm_pp_group_kernel, split-K slabs) against fp32 references."""
    H = 768
    g = torch.Generator(device="cuda").manual_seed(M)
    x0 = torch.randn(M, H, device="cuda", generator=g).bfloat16()
    dy0 = torch.randn(M, H, device="cuda", generator=g).bfloat16()
    x1 = torch.randn(M, H, device="cuda", generator=g).bfloat16()
    dy1 = torch.randn(M, 3 * H, device="cuda", generator=g).bfloat16()
    dw0 = torch.zeros(H, H, device="cuda")
    dw1 = torch.zeros(3 * H, H, device="cuda")
    grouped = _ops().gemm_wgrad2(x0, dy0, dw0, H, H, x1, dy1, dw1, 3 * H, H, M)
    assert grouped
    assert _rel(dw0, dy0.float().t() @ x0.float()) < 2e-3
    assert _rel(dw1, dy1.float().t() @ x1.float()) < 2e-3
    # deterministic (slabs summed in slice order)
    dw0b, dw1b = torch.zeros_like(dw0), torch.zeros_like(dw1)
    _ops().gemm_wgrad2(x0, dy0, dw0b, H, H, x1, dy1, dw1b, 3 * H, H, M)
    assert torch.equal(dw0, dw0b) and torch.equal(dw1, dw1b)


def test_dgrad_split_k_uneven_slices():
    """A split-K dgrad whose slice count does not divide the k-tiles: a
    32,000-word vocabulary at M = 512, K = 768 gives 31 slices of 17 k-tiles
    over 500, so a 31st slice would own none.  The launch must use only the
    slices that hold tiles; the workspace is poisoned with NaN first (the
    caching allocator hands the freed block back), so a slab left unwritten
    shows up in dx."""
    M, N, K = 512, 32000, 768
    g = torch.Generator(device="cuda").manual_seed(5)
    dy = torch.randn(M, N, device="cuda", generator=g).bfloat16()
    w = (torch.randn(N, K, device="cuda", generator=g) * 0.05).bfloat16()
    dx = torch.empty(M, K, device="cuda", dtype=torch.bfloat16)
    poison = torch.full((40 * M * K,), float("nan"), device="cuda")
    del poison
    _ops().gemm_dgrad(dy, w, dx, M, N, K, False)
    assert torch.isfinite(dx.float()).all()
    assert _rel(dx, dy.float() @ w.float()) < 1e-2


@pytest.mark.parametrize("M,N,K", SHAPES + [(512, 32000, 768)])
def test_dgrad_resid_equals_accumulate_into_copy(M, N, K):
    """dx = dy w + resid (the BERT backward's residual-branch gradient read in
    the output stage, models/bert.py) is bitwise the old two-step form: a copy
    of resid accumulated into -- on the plain large-tile path, the split-K
    slab path (the 32,000-word decoder shape) and the conv-core path."""
    g = torch.Generator(device="cuda").manual_seed(13 * M + K)
    dy = torch.randn(M, N, device="cuda", generator=g).bfloat16()
    w = (torch.randn(N, K, device="cuda", generator=g) * 0.05).bfloat16()
    resid = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    for big in (True, False):
        _ops().set_gemm_big(big)
        acc = resid.clone()
        _ops().gemm_dgrad(dy, w, acc, M, N, K, True)
        dx = torch.empty_like(resid)
        _ops().gemm_dgrad(dy, w, dx, M, N, K, False, resid)
        assert torch.equal(dx, acc), big
        assert _rel(dx, resid.float() + dy.float() @ w.float()) < 1e-2
    with pytest.raises(RuntimeError):
        _ops().gemm_dgrad(dy, w, dx, M, N, K, True, resid)


@pytest.mark.parametrize("big", [True, False])
def test_stored_gelu_derivative(big):
    """FFN1's forward may store gelu'(z) in place of z (act_grad) and the FFN2
    dgrad multiply by it (pre) instead of evaluating erf / exp in its output
    stage (models/bert.py GELU_GRAD).  gelu(z) is unchanged bitwise; the stored
    derivative is gelu' of the same bf16 pre-activation; the fused backward
    agrees with the one that evaluates gelu'(z) to bf16 rounding."""
    _ops().set_gemm_big(big)
    M, F, H = 1024, 3072, 768
    g = torch.Generator(device="cuda").manual_seed(17)
    a = torch.randn(M, H, device="cuda", generator=g).bfloat16()
    w1 = (torch.randn(F, H, device="cuda", generator=g) * 0.05).bfloat16()
    b1 = torch.randn(F, device="cuda", generator=g) * 0.1
    z, h = torch.empty(M, F, device="cuda", dtype=torch.bfloat16), torch.empty(M, F, device="cuda", dtype=torch.bfloat16)
    gp, h2 = torch.empty_like(z), torch.empty_like(h)
    _ops().gemm_fwd(a, w1, z, b1, None, h, M, F, H)
    _ops().gemm_fwd(a, w1, gp, b1, None, h2, M, F, H, True)
    assert torch.equal(h, h2)
    from metisfl_amd.ops.bert import gelu_grad_ref
    assert _rel(gp, gelu_grad_ref(z.float())) < 4e-3
    # backward: dz = (dy w2) * gelu'(z)
    dy = torch.randn(M, H, device="cuda", generator=g).bfloat16()
    w2 = (torch.randn(H, F, device="cuda", generator=g) * 0.05).bfloat16()
    dz0, dz1 = torch.empty_like(z), torch.empty_like(z)
    db0, db1 = torch.zeros(F, device="cuda"), torch.zeros(F, device="cuda")
    _ops().gemm_dgrad_gelu(dy, w2, dz0, z, db0, M, H, F)
    _ops().gemm_dgrad_gelu(dy, w2, dz1, gp, db1, M, H, F, True)
    ref = (dy.float() @ w2.float()) * gelu_grad_ref(z.float())
    assert _rel(dz0, ref) < 1e-2 and _rel(dz1, ref) < 1e-2
    assert _rel(dz1, dz0) < 8e-3
    assert _rel(db1, db0) < 8e-3
    _ops().set_gemm_big(True)


def test_grouped_wgrad_ffn_pair():
    """The BERT FFN2 + FFN1 weight gradients in one grouped launch (768 x 3072
    and 3072 x 768 outputs, 72 tiles, one merged slab reduce) against fp32
    references and the two single launches."""
    M, H, F = 4096, 768, 3072
    g = torch.Generator(device="cuda").manual_seed(23)
    h = torch.randn(M, F, device="cuda", generator=g).bfloat16()
    dfo = torch.randn(M, H, device="cuda", generator=g).bfloat16()
    a = torch.randn(M, H, device="cuda", generator=g).bfloat16()
    dz = torch.randn(M, F, device="cuda", generator=g).bfloat16()
    dw2, dw1 = torch.zeros(H, F, device="cuda"), torch.zeros(F, H, device="cuda")
    assert _ops().gemm_wgrad2(h, dfo, dw2, H, F, a, dz, dw1, F, H, M)
    assert _rel(dw2, dfo.float().t() @ h.float()) < 2e-3
    assert _rel(dw1, dz.float().t() @ a.float()) < 2e-3
    s2, s1 = torch.zeros_like(dw2), torch.zeros_like(dw1)
    _ops().gemm_wgrad(h, dfo, s2, M, H, F, False, True)
    _ops().gemm_wgrad(a, dz, s1, M, F, H, False, True)
    assert _rel(dw2, s2) < 1e-5 and _rel(dw1, s1) < 1e-5
