"""BERT-base ops: Linear-layer GEMMs + encoder kernels (csrc/kernels/bert.hip,
gemm.hip).  Device tensors always run the HIP kernels (``_native.ops`` raises
if the extension is missing); CPU tensors run the fp32 PyTorch reference of
the same op, which the GPU numerics tests compare against and the CPU model
tests train with.

Shape conventions: activations are row-major ``[M][width]`` bf16, Linear
weights ``[N_out][K_in]`` (K-contiguous, the layout the MFMA GEMM reads for
all three training GEMMs), LayerNorm / bias parameters and all gradients
fp32.  Batch records for the masked-LM path are int32 rows
``[tokens T | mlm positions P | mlm label ids P | inverse map T]``.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

from metisfl_amd.ops._native import ops

BF = torch.bfloat16


def _b(t):
    return t.float()


def _put(dst, val):
    dst.copy_(val.reshape(dst.shape).to(dst.dtype))


# ---- Linear -----------------------------------------------------------------
def gemm_fwd(x, w, y, M, N, K, bias=None, resid=None, act_out=None, act_grad=False) -> None:
    """y = x w^T (+bias) (+resid); act_out = gelu(y) (exact erf).  ``act_grad``
    (with act_out): y holds gelu'(z) of the bf16 pre-activation z instead of z,
    for a backward that multiplies by it (gemm_dgrad_gelu ``pre``)."""
    if x.is_cuda:
        ops().gemm_fwd(x, w, y, bias, resid, act_out, M, N, K, act_grad)
        return
    v = _b(x).reshape(M, K) @ _b(w).reshape(N, K).t()
    if bias is not None:
        v = v + bias.reshape(-1)[:N]
    if resid is not None:
        v = v + _b(resid).reshape(M, N)
    _put(y, v)
    if act_out is not None:
        z = _b(y).reshape(M, N)
        _put(act_out, F.gelu(z))
        if act_grad:
            _put(y, gelu_grad_ref(z))


def gemm_dgrad(dy, w, dx, M, N, K, accumulate=False, resid=None) -> None:
    """dx (+)= dy w; with ``resid``: dx = dy w + resid (a residual branch's
    gradient added in the output stage, instead of accumulating into a copy)."""
    if dy.is_cuda:
        ops().gemm_dgrad(dy, w, dx, M, N, K, accumulate, resid)
        return
    v = _b(dy).reshape(M, N) @ _b(w).reshape(N, K)
    if accumulate:
        v = v + _b(dx).reshape(M, K)
    if resid is not None:
        v = v + _b(resid).reshape(M, K)
    _put(dx, v)


def gemm_dgrad_gelu(dy, w, dz, z, M, N, K, dbias=None, pre=False) -> None:
    """dz = (dy w) * gelu'(z) (exact erf), dbias += column sums of dz: the
    FFN1 backward GEMM with the GELU backward fused into its epilogue.
    ``pre``: z holds gelu'(z) already (the forward's act_grad)."""
    if dy.is_cuda:
        ops().gemm_dgrad_gelu(dy, w, dz, z, dbias, M, N, K, pre)
        return
    v = _b(dy).reshape(M, N) @ _b(w).reshape(N, K)
    zz = _b(z).reshape(M, K)
    g = (v * (zz if pre else gelu_grad_ref(zz))).to(BF)
    _put(dz, g)
    if dbias is not None:
        dbias.add_(g.float().sum(0).reshape(dbias.shape))


def gemm_wgrad(x, dy, dw, M, N, K, accumulate=False, zeroed=False) -> None:
    """dw (+)= dy^T x  (fp32).  ``zeroed``: dw is already zero (skips the
    pre-zeroing of split-K plans; the training step's gradient buffer)."""
    if x.is_cuda:
        ops().gemm_wgrad(x, dy, dw, M, N, K, accumulate, zeroed)
        return
    v = _b(dy).reshape(M, N).t() @ _b(x).reshape(M, K)
    if accumulate:
        dw.add_(v.reshape(dw.shape))
    else:
        dw.copy_(v.reshape(dw.shape))


def gemm_wgrad2(x0, dy0, dw0, N0, K0, x1, dy1, dw1, N1, K1, M) -> bool:
    """dw0 = dy0^T x0 and dw1 = dy1^T x1 (fp32, both zero on entry) over the
    same M rows in ONE grouped launch on the GPU (gemm_big.hip
    gemm_pp_group_kernel) -> whether it was grouped."""
    if x0.is_cuda:
        return bool(ops().gemm_wgrad2(x0, dy0, dw0, N0, K0, x1, dy1, dw1, N1, K1, M))
    gemm_wgrad(x0, dy0, dw0, M, N0, K0)
    gemm_wgrad(x1, dy1, dw1, M, N1, K1)
    return False


# ---- LayerNorm ----------------------------------------------------------------
def _ln_ref(x, gamma, beta, eps):
    mean = x.mean(-1)
    var = ((x - mean[:, None]) ** 2).mean(-1)
    rstd = torch.rsqrt(var + eps)
    return (x - mean[:, None]) * rstd[:, None] * gamma + beta, mean, rstd


def ln_fwd(x, gamma, beta, y, mean, rstd, M, H, eps) -> None:
    if x.is_cuda:
        ops().ln_fwd(x, gamma, beta, y, mean, rstd, M, H, eps)
        return
    out, m, r = _ln_ref(_b(x).reshape(M, H), gamma.reshape(H), beta.reshape(H), eps)
    _put(y, out)
    mean[:M].copy_(m)
    rstd[:M].copy_(r)


def _emb_sum(rec, rec_stride, B, T, word, pos, type_, H):
    tok = rec.reshape(B, rec_stride)[:, :T].long()
    x = _b(word).reshape(-1, H)[tok] + _b(pos).reshape(-1, H)[:T][None] + _b(type_).reshape(-1, H)[0]
    return x.reshape(B * T, H).to(BF)


def emb_ln_fwd(rec, rec_stride, B, T, word, pos, type_, xsave, gamma, beta, y, mean, rstd, H, eps) -> None:
    if y.is_cuda:
        ops().emb_ln_fwd(rec, rec_stride, B, T, word, pos, type_, xsave, gamma, beta, y, mean, rstd, H, eps)
        return
    xs = _emb_sum(rec, rec_stride, B, T, word, pos, type_, H)
    _put(xsave, xs)
    ln_fwd(xs, gamma, beta, y, mean, rstd, B * T, H, eps)


def _ln_bwd_ref(dy, x, mean, rstd, gamma, M, H):
    dy, x = _b(dy).reshape(M, H), _b(x).reshape(M, H)
    xh = (x - mean[:M, None]) * rstd[:M, None]
    g = dy * gamma.reshape(H)
    dx = rstd[:M, None] * (g - g.mean(-1, keepdim=True) - xh * (g * xh).mean(-1, keepdim=True))
    return dx, (dy * xh).sum(0), dy.sum(0)


def ln_bwd(dy, x, mean, rstd, gamma, dx, dgamma, dbeta, M, H, dx2=None, dbias_prev=None) -> None:
    """dx (and dx2) = LN backward; dgamma, dbeta, dbias_prev (+= colsum dx) accumulate."""
    if dy.is_cuda:
        ops().ln_bwd(dy, x, mean, rstd, gamma, dx, dx2, dgamma, dbeta, dbias_prev, M, H)
        return
    d, dg, db = _ln_bwd_ref(dy, x, mean, rstd, gamma, M, H)
    dq = d.to(BF)
    _put(dx, dq)
    if dx2 is not None:
        _put(dx2, dq)
    dgamma.add_(dg.reshape(dgamma.shape))
    dbeta.add_(db.reshape(dbeta.shape))
    if dbias_prev is not None:
        dbias_prev.add_(d.sum(0).reshape(dbias_prev.shape))


class EmbGradScratch:
    """Device scratch of the sorted (contention-free) word-embedding gradient:
    fp32 dx rows [M][H], (token, row) pairs + their sorted copies, hipCUB
    radix-sort temp storage."""

    def __init__(self, M: int, H: int, V: int, device):
        self.demb = torch.empty(M * H, dtype=torch.float32, device=device)
        self.idx = torch.empty(4 * M, dtype=torch.int32, device=device)
        nbytes = int(ops().emb_sort_temp_bytes(M, V)) if torch.device(device).type == "cuda" else 1
        self.tmp = torch.empty(max(1, nbytes), dtype=torch.uint8, device=device)


def emb_ln_bwd(dy, xsave, mean, rstd, gamma, rec, rec_stride, B, T, dword, dpos, dtype, dgamma, dbeta, H,
               scratch: EmbGradScratch | None = None) -> None:
    if dy.is_cuda:
        if scratch is not None:
            ops().emb_ln_bwd(dy, xsave, mean, rstd, gamma, rec, rec_stride, B, T, dword, dpos, dtype, dgamma,
                             dbeta, H, scratch.demb, scratch.idx, scratch.tmp)
        else:
            ops().emb_ln_bwd(dy, xsave, mean, rstd, gamma, rec, rec_stride, B, T, dword, dpos, dtype, dgamma,
                             dbeta, H)
        return
    M = B * T
    d, dg, db = _ln_bwd_ref(dy, xsave, mean, rstd, gamma, M, H)
    dgamma.add_(dg.reshape(dgamma.shape))
    dbeta.add_(db.reshape(dbeta.shape))
    tok = rec.reshape(B, rec_stride)[:, :T].reshape(-1).long()
    dword.reshape(-1, H).index_add_(0, tok, d)
    dpos.reshape(-1, H)[:T].add_(d.reshape(B, T, H).sum(0))
    dtype.reshape(-1)[:H].add_(d.sum(0))


# ---- GELU / bias gradients ----------------------------------------------------
def gelu_grad_ref(z):
    return 0.5 * (1.0 + torch.erf(z / math.sqrt(2.0))) + z * torch.exp(-0.5 * z * z) / math.sqrt(2 * math.pi)


def gelu_bwd(dh, z, dz, M, N, dbias=None) -> None:
    if dh.is_cuda:
        ops().gelu_bwd(dh, z, dz, dbias, M, N)
        return
    g = (_b(dh).reshape(M, N) * gelu_grad_ref(_b(z).reshape(M, N))).to(BF)
    _put(dz, g)
    if dbias is not None:
        dbias.add_(g.float().sum(0).reshape(dbias.shape))


def colsum(dy, dbias, M, N) -> None:
    if dy.is_cuda:
        ops().colsum(dy, dbias, M, N)
        return
    dbias.add_(_b(dy).reshape(M, N).sum(0).reshape(dbias.shape))


# ---- attention (seq 128, head dim 64) -----------------------------------------
SEQ, HEAD_DIM = 128, 64


def _split_qkv(qkv, B, heads):
    H = heads * HEAD_DIM
    t = _b(qkv).reshape(B, SEQ, 3, heads, HEAD_DIM).permute(2, 0, 3, 1, 4)  # 3, B, h, T, d
    return t[0], t[1], t[2], H


def attn_fwd(qkv, ctx, lse, B, heads, scale) -> None:
    if qkv.is_cuda:
        ops().attn_fwd(qkv, ctx, lse, B, heads, scale)
        return
    q, k, v, H = _split_qkv(qkv, B, heads)
    s = (q @ k.transpose(-1, -2)) * scale
    L = torch.logsumexp(s, -1)
    p = torch.exp(s - L[..., None]).to(BF).float()
    o = p @ v
    _put(ctx, o.permute(0, 2, 1, 3).reshape(B * SEQ, H))
    lse.reshape(-1)[: B * heads * SEQ].copy_(L.reshape(-1))


def attn_bwd(qkv, ctx, lse, dctx, dqkv, B, heads, scale, dbias=None) -> None:
    if qkv.is_cuda:
        ops().attn_bwd(qkv, ctx, lse, dctx, dqkv, dbias, B, heads, scale)
        return
    q, k, v, H = _split_qkv(qkv, B, heads)
    L = lse.reshape(-1)[: B * heads * SEQ].reshape(B, heads, SEQ)
    do = _b(dctx).reshape(B, SEQ, heads, HEAD_DIM).permute(0, 2, 1, 3)
    o = _b(ctx).reshape(B, SEQ, heads, HEAD_DIM).permute(0, 2, 1, 3)
    s = (q @ k.transpose(-1, -2)) * scale
    p = torch.exp(s - L[..., None])
    dp = do @ v.transpose(-1, -2)
    D = (do * o).sum(-1, keepdim=True)
    ds = p * (dp - D)
    dq = (ds @ k) * scale
    dk = (ds.transpose(-1, -2) @ q) * scale
    dv = p.transpose(-1, -2) @ do
    g = torch.stack([dq, dk, dv], 0).permute(1, 3, 0, 2, 4).reshape(B * SEQ, 3 * H)
    _put(dqkv, g)
    if dbias is not None:
        dbias.add_(g.sum(0).reshape(dbias.shape))


# ---- masked-LM head plumbing ----------------------------------------------------
def _rec(rec, rec_stride, B):
    return rec.reshape(-1)[: B * rec_stride].reshape(B, rec_stride)


def mlm_gather(x, rec, rec_stride, B, T, P, out, H) -> None:
    if x.is_cuda:
        ops().mlm_gather(x, rec, rec_stride, B, T, P, out, H)
        return
    pos = _rec(rec, rec_stride, B)[:, T:T + P].long()
    xs = x.reshape(B, T, H)
    _put(out, torch.gather(xs, 1, pos[..., None].expand(B, P, H)))


def mlm_scatter(dsel, rec, rec_stride, B, T, P, dx, H) -> None:
    if dx.is_cuda:
        ops().mlm_scatter(dsel, rec, rec_stride, B, T, P, dx, H)
        return
    inv = _rec(rec, rec_stride, B)[:, T + 2 * P:T + 2 * P + T].long()
    src = dsel.reshape(B, P, H)
    out = torch.zeros(B, T, H, dtype=dsel.dtype)
    m = inv >= 0
    out[m] = torch.gather(src, 1, inv.clamp(min=0)[..., None].expand(B, T, H))[m]
    _put(dx, out)


def vocab_xent(logits, rec, rec_stride, B, T, P, V, Vp, stats, dlogits=None) -> None:
    """Softmax CE over V of Vp columns; dlogits = (softmax - onehot) / (B*P)."""
    if logits.is_cuda:
        ops().vocab_xent(logits, dlogits, rec, rec_stride, B, T, P, V, Vp, stats)
        return
    R = B * P
    z = _b(logits).reshape(R, Vp)[:, :V]
    y = _rec(rec, rec_stride, B)[:, T + P:T + 2 * P].reshape(R).long()
    valid = (y >= 0) & (y < V)
    lse = torch.logsumexp(z, -1)
    yc = y.clamp(0, V - 1)
    loss = (lse - z.gather(1, yc[:, None])[:, 0])[valid].sum()
    correct = (z.argmax(-1) == y)[valid].float().sum()
    stats[0] += loss
    stats[1] += correct
    stats[2] += float(valid.sum())
    if dlogits is not None:
        g = torch.softmax(z, -1)
        g[torch.arange(R), yc] -= 1.0
        g = g * valid[:, None].float() / R
        full = torch.zeros(R, Vp)
        full[:, :V] = g
        _put(dlogits, full)
