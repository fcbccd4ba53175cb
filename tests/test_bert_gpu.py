"""BERT-path HIP kernels (bert.hip, gemm.hip) vs the fp32 CPU reference ops,
and the BERT-tiny training step GPU vs CPU."""
import math
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"
BF = torch.bfloat16


def rel(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return float((a - b).norm() / (b.norm() + 1e-12))


def _native():
    from metisfl_amd.ops._native import ops
    ops()


@pytest.mark.parametrize("M,N,K", [(512, 768, 256), (4096, 2304, 768), (640, 1000, 256), (200, 136, 72)])
def test_linear_gemms(M, N, K):
    from metisfl_amd.ops import bert as BO
    _native()
    torch.manual_seed(0)
    x = torch.randn(M, K).to(BF)
    w = (torch.randn(N, K) * 0.05).to(BF)
    b = torch.randn(N)
    r = torch.randn(M, N).to(BF)
    outs = {}
    for dev in ("cpu", DEV):
        y, h = torch.empty(M, N, dtype=BF, device=dev), torch.empty(M, N, dtype=BF, device=dev)
        BO.gemm_fwd(x.to(dev), w.to(dev), y, M, N, K, bias=b.to(dev), resid=r.to(dev), act_out=h)
        dy = (torch.randn(M, N, generator=torch.Generator().manual_seed(1))).to(BF).to(dev)
        dx = x.clone().to(dev)
        BO.gemm_dgrad(dy, w.to(dev), dx, M, N, K, accumulate=True)
        dw = torch.ones(N, K, device=dev)
        BO.gemm_wgrad(x.to(dev), dy, dw, M, N, K, accumulate=True)
        dw2 = torch.full((N, K), 7.0, device=dev)
        BO.gemm_wgrad(x.to(dev), dy, dw2, M, N, K, accumulate=False)
        outs[dev] = (y, h, dx, dw, dw2)
    for a, c in zip(outs[DEV], outs["cpu"]):
        assert rel(a, c) < 1e-2


@pytest.mark.parametrize("accumulate", [False, True])
def test_split_k_dgrad_long_reduction(accumulate):
    """A dgrad whose output tiles cannot fill the chip but whose reduction is
    long (the MLM decoder: 2,560 x 768 over the vocabulary) runs split-K
    through fp32 slabs and one bf16 reduce."""
    from metisfl_amd.ops import bert as BO
    from metisfl_amd.ops._native import ops
    _native()
    M, N, K = 512, 8192, 768
    assert ops().gemm_dgrad_workspace(M, N, K) > 0  # the split plan is taken
    assert ops().gemm_dgrad_workspace(16384, 768, 768) == 0  # full-chip shapes are not split
    g = torch.Generator().manual_seed(3)
    dy = torch.randn(M, N, generator=g).to(BF)
    w = (torch.randn(N, K, generator=g) * 0.05).to(BF)
    dx0 = torch.randn(M, K, generator=g).to(BF)
    ref = dy.float() @ w.float() + (dx0.float() if accumulate else 0.0)
    dx = dx0.clone().to(DEV)
    BO.gemm_dgrad(dy.to(DEV), w.to(DEV), dx, M, N, K, accumulate=accumulate)
    assert rel(dx.cpu(), ref) < 1e-2


@pytest.mark.parametrize("H", [256, 768])
def test_layernorm_fwd_bwd(H):
    from metisfl_amd.ops import bert as BO
    _native()
    torch.manual_seed(1)
    M = 300
    x = (torch.randn(M, H) * 2 + 0.5).to(BF)
    gam, bet = torch.rand(H) + 0.5, torch.randn(H)
    dy = torch.randn(M, H).to(BF)
    res = {}
    for dev in ("cpu", DEV):
        y = torch.empty(M, H, dtype=BF, device=dev)
        mean, rstd = torch.zeros(M, device=dev), torch.zeros(M, device=dev)
        BO.ln_fwd(x.to(dev), gam.to(dev), bet.to(dev), y, mean, rstd, M, H, 1e-12)
        dx, dx2 = torch.empty(M, H, dtype=BF, device=dev), torch.empty(M, H, dtype=BF, device=dev)
        dg, db, dbp = (torch.zeros(H, device=dev) for _ in range(3))
        BO.ln_bwd(dy.to(dev), x.to(dev), mean, rstd, gam.to(dev), dx, dg, db, M, H, dx2=dx2, dbias_prev=dbp)
        res[dev] = (y, mean, rstd, dx, dx2, dg, db, dbp)
    for a, c in zip(res[DEV], res["cpu"]):
        assert rel(a, c) < 1e-2


@pytest.mark.parametrize("sorted_grad", [False, True])
def test_embedding_layernorm_fwd_bwd(sorted_grad):
    """Embedding LN forward / backward vs CPU; ``sorted_grad``: the word-table
    gradient by token sort + segmented sum (B = 32 puts [CLS] rows and ~640
    [MASK] rows in long segments that cross many 64-row chunks)."""
    from metisfl_amd.datasets import synthetic_mlm
    from metisfl_amd.ops import bert as BO
    _native()
    torch.manual_seed(2)
    B, T, P, H, V = (32 if sorted_grad else 3), 128, (20 if sorted_grad else 8), 256, 500
    rec = torch.as_tensor(synthetic_mlm(B, T, P, V, seed=1))
    stride = rec.shape[1]
    word, pos, typ = (torch.randn(V, H) * 0.1).to(BF), (torch.randn(T, H) * 0.1).to(BF), (torch.randn(2, H) * 0.1).to(BF)
    gam, bet = torch.rand(H) + 0.5, torch.randn(H)
    dy = torch.randn(B * T, H).to(BF)
    res = {}
    for dev in ("cpu", DEV):
        M = B * T
        xs, y = torch.empty(M, H, dtype=BF, device=dev), torch.empty(M, H, dtype=BF, device=dev)
        mean, rstd = torch.zeros(M, device=dev), torch.zeros(M, device=dev)
        r = rec.to(dev)
        BO.emb_ln_fwd(r, stride, B, T, word.to(dev), pos.to(dev), typ.to(dev), xs, gam.to(dev), bet.to(dev), y,
                      mean, rstd, H, 1e-12)
        dw, dp, dt = torch.zeros(V, H, device=dev), torch.zeros(T, H, device=dev), torch.zeros(2, H, device=dev)
        dg, db = torch.zeros(H, device=dev), torch.zeros(H, device=dev)
        scr = BO.EmbGradScratch(M, H, V, dev) if (sorted_grad and dev != "cpu") else None
        if scr is not None:
            dw.fill_(0.5)  # the sorted path adds into the buffer (tied decoder grads land there too)
        BO.emb_ln_bwd(dy.to(dev), xs, mean, rstd, gam.to(dev), r, stride, B, T, dw, dp, dt, dg, db, H,
                      scratch=scr)
        if scr is not None:
            dw.sub_(0.5)
        res[dev] = (xs, y, dw, dp, dt, dg, db)
    for a, c in zip(res[DEV], res["cpu"]):
        assert rel(a, c) < 1e-2


def test_gelu_bwd_and_colsum():
    from metisfl_amd.ops import bert as BO
    _native()
    torch.manual_seed(3)
    M, N = 333, 3072
    dh, z = torch.randn(M, N).to(BF), (torch.randn(M, N) * 2).to(BF)
    res = {}
    for dev in ("cpu", DEV):
        dz = torch.empty(M, N, dtype=BF, device=dev)
        db, cs = torch.zeros(N, device=dev), torch.zeros(N, device=dev)
        BO.gelu_bwd(dh.to(dev), z.to(dev), dz, M, N, dbias=db)
        BO.colsum(dh.to(dev), cs, M, N)
        res[dev] = (dz, db, cs)
    for a, c in zip(res[DEV], res["cpu"]):
        assert rel(a, c) < 1e-2


@pytest.mark.parametrize("heads", [4, 12])
def test_attention_fwd_bwd(heads):
    from metisfl_amd.ops import bert as BO
    _native()
    torch.manual_seed(4)
    B, T, H = 2, 128, heads * 64
    qkv = (torch.randn(B * T, 3 * H) * 1.5).to(BF)
    dctx = torch.randn(B * T, H).to(BF)
    scale = 1.0 / math.sqrt(64)
    res = {}
    for dev in ("cpu", DEV):
        ctx = torch.empty(B * T, H, dtype=BF, device=dev)
        lse = torch.zeros(B * heads * T, device=dev)
        BO.attn_fwd(qkv.to(dev), ctx, lse, B, heads, scale)
        dqkv = torch.empty(B * T, 3 * H, dtype=BF, device=dev)
        db = torch.zeros(3 * H, device=dev)
        BO.attn_bwd(qkv.to(dev), ctx, lse, dctx.to(dev), dqkv, B, heads, scale, dbias=db)
        res[dev] = (ctx, lse, dqkv, db)
    for nm, a, c in zip(("ctx", "lse", "dqkv", "dbias"), res[DEV], res["cpu"]):
        assert rel(a, c) < 2e-2, nm
    # against autograd of plain fp32 attention
    q = qkv.float().reshape(B, T, 3, heads, 64).permute(2, 0, 3, 1, 4).requires_grad_(True)
    o = torch.softmax(q[0] @ q[1].transpose(-1, -2) * scale, -1) @ q[2]
    o.permute(0, 2, 1, 3).reshape(B * T, H).backward(dctx.float())
    g = q.grad.permute(1, 3, 0, 2, 4).reshape(B * T, 3 * H)
    assert rel(res[DEV][2], g) < 2e-2


def test_mlm_gather_scatter_and_vocab_xent():
    from metisfl_amd.datasets import synthetic_mlm
    from metisfl_amd.ops import bert as BO
    _native()
    torch.manual_seed(5)
    B, T, P, H, V, Vp = 4, 128, 20, 256, 30522, 30528
    rec = torch.as_tensor(synthetic_mlm(B, T, P, V, seed=3))
    stride = rec.shape[1]
    x = torch.randn(B * T, H).to(BF)
    logits = (torch.randn(B * P, Vp) * 3).to(BF)
    res = {}
    for dev in ("cpu", DEV):
        r = rec.to(dev)
        sel = torch.empty(B * P, H, dtype=BF, device=dev)
        BO.mlm_gather(x.to(dev), r, stride, B, T, P, sel, H)
        back = torch.empty(B * T, H, dtype=BF, device=dev)
        BO.mlm_scatter(sel, r, stride, B, T, P, back, H)
        st = torch.zeros(4, device=dev)
        dl = torch.empty(B * P, Vp, dtype=BF, device=dev)
        BO.vocab_xent(logits.to(dev), r, stride, B, T, P, V, Vp, st, dlogits=dl)
        res[dev] = (sel, back, st[:3], dl)
    for a, c in zip(res[DEV], res["cpu"]):
        assert rel(a, c) < 1e-2
    assert float(res[DEV][3][:, V:].float().abs().sum()) == 0.0


def test_bert_tiny_step_gpu_vs_cpu():
    from metisfl_amd.datasets import synthetic_mlm
    from metisfl_amd.models.bert import BERT_TINY, BertMLM
    from metisfl_amd.ops.optim import OptimizerSpec
    _native()
    nets = {}
    c = BERT_TINY
    rec = synthetic_mlm(4, c.seq, c.max_pred, c.vocab, seed=7, rec_stride=c.rec_stride)
    for dev in ("cpu", DEV):
        n = BertMLM(batch_size=4, device=dev, seed=2, config=c, optimizer=OptimizerSpec("vanilla_sgd", 0.0))
        n.zero_grad_in_optimizer = False
        n._train_body(n.make_dataset(rec, shuffle=False))
        nets[dev] = n
    torch.cuda.synchronize()
    a, b = nets["cpu"].state.grad32.double(), nets[DEV].state.grad32.double().cpu()
    cos = float(a @ b / (a.norm() * b.norm()))
    assert cos > 0.98, cos
    la = float(nets["cpu"].stats[0]) / float(nets["cpu"].stats[2])
    lb = float(nets[DEV].stats[0].cpu()) / float(nets[DEV].stats[2].cpu())
    assert abs(la - lb) < 0.02 * la


def test_bert_tiny_step_tracks_torch_nn_oracle():
    """The bf16 HIP BERT step vs an independent fp32 torch.nn BERT
    (tests/torch_bert_ref.py) on the same master weights and records: loss
    and the gradient of EVERY parameter tensor (cosine similarity; bf16
    activations / GEMM operands bound the agreement)."""
    import sys
    sys.path.insert(0, os.path.dirname(__file__))
    from torch_bert_ref import TorchBertMLM

    from metisfl_amd.datasets import synthetic_mlm
    from metisfl_amd.models.bert import BERT_TINY, BertMLM
    from metisfl_amd.ops.optim import OptimizerSpec
    _native()
    c = BERT_TINY
    rec = synthetic_mlm(8, c.seq, c.max_pred, c.vocab, seed=5, rec_stride=c.rec_stride)
    net = BertMLM(batch_size=8, device=DEV, seed=4, config=c, optimizer=OptimizerSpec("vanilla_sgd", 0.0))
    net.zero_grad_in_optimizer = False
    net._train_body(net.make_dataset(rec, shuffle=False))
    torch.cuda.synchronize()
    loss_gpu = float(net.stats[0].cpu()) / float(net.stats[2].cpu())
    ref = TorchBertMLM(c)
    ref.load_from_flat(net.state)
    loss_ref = ref(torch.as_tensor(rec[:8]))
    loss_ref.backward()
    g_ref = ref.grads_like_flat()
    num = den_a = den_b = 0.0
    worst = []
    for name, gr in g_ref.items():
        gg = net.state.grad(name).detach().double().cpu().reshape(gr.shape)
        gr = gr.double()
        if name == "emb.word":  # rows of tokens that never occur get zero in both
            gr, gg = gr[: c.vocab], gg[: c.vocab]
        num += float((gg * gr).sum())
        den_a += float((gg * gg).sum())
        den_b += float((gr * gr).sum())
        cs = float((gg * gr).sum() / (gg.norm() * gr.norm() + 1e-30))
        worst.append((cs, name))
    worst.sort()
    cos = num / (den_a ** 0.5 * den_b ** 0.5)
    print(f"bf16 BERT-tiny: loss {loss_gpu:.5f} vs torch.nn fp32 {float(loss_ref):.5f}; "
          f"gradient cosine {cos:.5f}; lowest {worst[:3]}")
    assert abs(loss_gpu - float(loss_ref)) < 0.01 * float(loss_ref)
    assert cos > 0.99, (cos, worst[:5])
    assert worst[0][0] > 0.95, worst[:5]


def test_bert_base_graph_step_runs():
    """Full BERT-base (110M) training steps through the captured hipGraph."""
    from metisfl_amd.datasets import synthetic_mlm
    from metisfl_amd.models.bert import BertMLM
    _native()
    net = BertMLM(batch_size=8, device=DEV, seed=0)
    c = net.cfg
    ds = net.make_dataset(synthetic_mlm(32, c.seq, c.max_pred, c.vocab, seed=1, rec_stride=c.rec_stride))
    net.reset_train_stats()
    net.train_steps(ds, 3)
    assert int(net.state.step.cpu()) == 3  # the optimizer launch's fused step tick
    s = net.train_stats()
    assert np.isfinite(s["loss"]) and abs(s["loss"] - math.log(c.vocab)) < 1.5, s


def test_attention_bwd_persistent_matches_per_item_launch(monkeypatch):
    """The persistent attention backward (next item's tiles prefetched into
    registers, 576 items over <= 256 workgroups) computes exactly what the
    one-item-per-workgroup launch does: D = rowsum(dO * O) is summed in a
    different order (8-lane tree vs 2 x 32 sequential), so dq/dk/dv agree up
    to that fp32 rounding (bf16 outputs: nearly all bits equal)."""
    from metisfl_amd.ops import bert as BO
    _native()
    torch.manual_seed(9)
    B, heads = 48, 12
    T, H = 128, heads * 64
    qkv = (torch.randn(B * T, 3 * H) * 1.5).to(BF).to(DEV)
    dctx = torch.randn(B * T, H).to(BF).to(DEV)
    scale = 1.0 / math.sqrt(64)
    ctx = torch.empty(B * T, H, dtype=BF, device=DEV)
    lse = torch.zeros(B * heads * T, device=DEV)
    BO.attn_fwd(qkv, ctx, lse, B, heads, scale)
    out = {}
    for mode in ("0", "1"):
        monkeypatch.setenv("MFL_ATTN_BWD_PERSIST", mode)
        dqkv = torch.empty(B * T, 3 * H, dtype=BF, device=DEV)
        db = torch.zeros(3 * H, device=DEV)
        BO.attn_bwd(qkv, ctx, lse, dctx, dqkv, B, heads, scale, dbias=db)
        torch.cuda.synchronize()
        out[mode] = (dqkv, db)
    a, b = out["1"][0], out["0"][0]
    assert rel(a, b) < 1e-3
    assert (a == b).float().mean().item() > 0.99
    assert rel(out["1"][1], out["0"][1]) < 1e-4


def test_attention_fwd_persistent_matches_per_item_launch(monkeypatch):
    """The persistent attention forward (a workgroup walks items with the next
    item's K / V slices in flight, 1152 items over <= 512 workgroups) runs the
    per-item arithmetic unchanged: context and lse bitwise equal to the
    one-item-per-workgroup launch."""
    from metisfl_amd.ops import bert as BO
    _native()
    torch.manual_seed(10)
    B, heads = 96, 12
    T, H = 128, heads * 64
    qkv = (torch.randn(B * T, 3 * H) * 1.5).to(BF).to(DEV)
    scale = 1.0 / math.sqrt(64)
    out = {}
    for mode in ("0", "1"):
        monkeypatch.setenv("MFL_ATTN_FWD_PERSIST", mode)
        ctx = torch.full((B * T, H), float("nan"), dtype=BF, device=DEV)
        lse = torch.full((B * heads * T,), float("nan"), device=DEV)
        BO.attn_fwd(qkv, ctx, lse, B, heads, scale)
        torch.cuda.synchronize()
        out[mode] = (ctx, lse)
    assert torch.equal(out["1"][0], out["0"][0])
    assert torch.equal(out["1"][1], out["0"][1])
