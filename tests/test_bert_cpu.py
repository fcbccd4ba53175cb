"""BERT masked-LM learner on the CPU reference ops: the hand-written backward
(fused bias / LN / attention gradients, tied decoder) against torch.autograd
of an independent functional BERT built from the same weights."""
import math

import numpy as np
import torch
import torch.nn.functional as F

from metisfl_amd.datasets import synthetic_mlm
from metisfl_amd.models.bert import BERT_TINY, BertMLM
from metisfl_amd.ops.optim import OptimizerSpec


def _ref_loss(net, rec):
    c = net.cfg
    B, T, H, P, V = net.B, c.seq, c.hidden, c.max_pred, c.vocab
    st = net.state
    leaves = {}

    def w(name):  # matrices the kernels read as bf16
        if name not in leaves:
            leaves[name] = st.bf16(name).float().clone().requires_grad_(True)
        return leaves[name]

    def p(name):  # fp32 LN / bias parameters
        if name not in leaves:
            leaves[name] = st.view(name).float().clone().requires_grad_(True)
        return leaves[name]

    def ln(x, pre):
        return F.layer_norm(x, (H,), p(pre + ".gamma"), p(pre + ".beta"), c.eps)

    r = torch.as_tensor(rec).long()
    tok = r[:, :T]
    x = w("emb.word")[tok] + w("emb.pos")[:T][None] + w("emb.type")[0]
    x = ln(x.reshape(B * T, H), "emb.ln")
    for i in range(c.layers):
        q = f"layer{i}."
        qkv = x @ w(q + "qkv.w").t() + p(q + "qkv.b")
        t = qkv.reshape(B, T, 3, c.heads, 64).permute(2, 0, 3, 1, 4)
        s = t[0] @ t[1].transpose(-1, -2) / math.sqrt(64)
        ctx = (torch.softmax(s, -1) @ t[2]).permute(0, 2, 1, 3).reshape(B * T, H)
        a = ln(ctx @ w(q + "out.w").t() + p(q + "out.b") + x, q + "ln1")
        h = F.gelu(a @ w(q + "ffn1.w").t() + p(q + "ffn1.b"))
        x = ln(h @ w(q + "ffn2.w").t() + p(q + "ffn2.b") + a, q + "ln2")
    pos = r[:, T:T + P]
    hm = x.reshape(B, T, H)[torch.arange(B)[:, None], pos].reshape(B * P, H)
    u = ln(F.gelu(hm @ w("head.w").t() + p("head.b")), "head.ln")
    logits = (u @ w("emb.word").t() + p("head.dec.b"))[:, :V]
    ids = r[:, T + P:T + 2 * P].reshape(-1)
    loss = F.cross_entropy(logits, ids)
    loss.backward()
    return float(loss.detach()), {k: v.grad for k, v in leaves.items()}


def test_bert_tiny_grads_match_autograd():
    net = BertMLM(batch_size=2, device="cpu", seed=3, config=BERT_TINY,
                  optimizer=OptimizerSpec("vanilla_sgd", 0.0))
    net.zero_grad_in_optimizer = False
    c = net.cfg
    rec = synthetic_mlm(2, c.seq, c.max_pred, c.vocab, seed=5, rec_stride=c.rec_stride)
    ds = net.make_dataset(rec, shuffle=False)
    net._train_body(ds)
    loss = float(net.stats[0]) / float(net.stats[2])
    ref_loss, ref = _ref_loss(net, rec)
    assert abs(loss - ref_loss) < 0.02 * ref_loss, (loss, ref_loss)
    assert abs(ref_loss - math.log(c.vocab)) < 1.0  # random init: ~uniform prediction
    bad = []
    for name, gref in ref.items():
        got = net.state.grad(name).double().reshape(-1)
        g = gref.double().reshape(-1)
        if name == "emb.type":
            g, got = g[: c.hidden], got[: c.hidden]  # only type id 0 is used
        cos = float(got @ g / (got.norm() * g.norm() + 1e-30))
        if cos < 0.98:
            bad.append((name, cos))
    assert not bad, bad


def test_bert_tiny_learns():
    net = BertMLM(batch_size=8, device="cpu", seed=1, config=BERT_TINY,
                  optimizer=OptimizerSpec("adam_weight_decay", 1e-3, weight_decay=0.01, epsilon=1e-6))
    c = net.cfg
    rec = synthetic_mlm(64, c.seq, c.max_pred, c.vocab, seed=2, rec_stride=c.rec_stride)
    ds = net.make_dataset(rec)
    losses = []
    for k in range(8):
        net.reset_train_stats()
        net.train_steps(ds, 4, step_offset=4 * k)
        losses.append(net.train_stats()["loss"])
    assert np.isfinite(losses[-1]) and losses[-1] < losses[0] - 1.0, losses


def test_bert_base_parameter_count():
    from metisfl_amd.models.bert import BERT_BASE
    n = BERT_BASE.param_count()
    assert 108e6 < n < 111e6, n  # BERT-base MLM without the NSP / pooler head
