"""BERT-base masked-LM learner on the HIP kernels.

The reference has no transformer model; SURVEY §2.10 sizes its kernels for a
BERT-base config (110M parameters, bf16) as the GEMM-heavy federated
workload of the new build, and §5.7 asks for a fused attention kernel.  This
is that learner: a post-LN encoder (Devlin et al. layout: embeddings + LN,
12 x [QKV -> attention -> out-proj + residual -> LN -> FFN(GELU) + residual ->
LN], masked-LM head with the decoder tied to the word embeddings), trained
with the fused flat-buffer optimizer (AdamW by default).  The sentence-pair
(NSP) head and dropout are not modelled: the benchmark is MLM throughput.

Step = ONE hipGraph replay: batch gather -> embeddings+LN -> 12 layers ->
gather of the masked positions -> head -> vocab CE -> backward (every
weight gradient by the wgrad GEMM straight into the flat fp32 gradient
buffer, bias / LN gradients fused into the kernels that produce the
activations' gradients) -> one optimizer launch -> step tick.

Per layer 7 forward launches (QKV GEMM+bias, attention, out-proj
GEMM+bias+residual, LN, FFN-1 GEMM+bias+GELU, FFN-2 GEMM+bias+residual, LN)
and 12 backward launches.
"""
from __future__ import annotations

import os

from dataclasses import dataclass

import numpy as np
import torch

from metisfl_amd.models.flat import FlatState, VarSpec
from metisfl_amd.models.net import DeviceDataset, StaticNet
from metisfl_amd.ops import bert as BO
from metisfl_amd.ops import nn as K
from metisfl_amd.ops import optim as opt_ops
from metisfl_amd.ops.optim import OptimizerSpec


# attention-output + QKV weight gradients grouped in one launch (MFL_BERT_WGRAD2=0:
# two launches, for A/B runs)
WGRAD2 = os.environ.get("MFL_BERT_WGRAD2", "1") == "1"
# the residual branch's gradient added in the FFN1 / QKV dgrad output stage
# (MFL_BERT_RESID_DGRAD=0: the LayerNorm backward writes a second copy of its
# dx that the dgrad accumulates into -- 25 MB more written per LayerNorm)
RESID_DGRAD = os.environ.get("MFL_BERT_RESID_DGRAD", "1") == "1"
# FFN1's forward stores gelu'(z) where it stored z, so the FFN2 dgrad's output
# stage multiplies by it instead of evaluating erf / exp per element
# (MFL_BERT_GELU_GRAD=0: store z, evaluate gelu'(z) in the backward)
GELU_GRAD = os.environ.get("MFL_BERT_GELU_GRAD", "1") == "1"
# the two FFN weight gradients in one grouped launch after the FFN2 dgrad
# (72 output tiles: 3 split-K slices instead of 7 each, fewer slab bytes)
FFN_WGRAD2 = os.environ.get("MFL_BERT_FFN_WGRAD2", "1") == "1"


@dataclass
class BertConfig:
    vocab: int = 30522
    hidden: int = 768
    layers: int = 12
    heads: int = 12
    ffn: int = 3072
    max_pos: int = 512
    type_vocab: int = 2
    seq: int = 128          # the fused attention kernel's sequence length
    max_pred: int = 20      # masked positions per sequence (BERT pre-training: 20 at seq 128)
    eps: float = 1e-12

    @property
    def vocab_padded(self) -> int:
        return (self.vocab + 63) // 64 * 64

    @property
    def rec_stride(self) -> int:
        r = 2 * self.seq + 2 * self.max_pred
        return (r + 3) // 4 * 4  # int32 record -> bf16 row of a multiple of 8

    def param_count(self) -> int:
        H, F, L = self.hidden, self.ffn, self.layers
        emb = self.vocab * H + self.max_pos * H + self.type_vocab * H + 2 * H
        layer = 3 * H * H + 3 * H + H * H + H + 2 * H + F * H + F + H * F + H + 2 * H
        head = H * H + H + 2 * H + self.vocab
        return emb + L * layer + head


BERT_BASE = BertConfig()
BERT_TINY = BertConfig(vocab=1000, hidden=256, layers=2, heads=4, ffn=512, max_pos=128, max_pred=8)


class BertMLM(StaticNet):
    """Masked-LM BERT learner.  ``make_dataset`` takes int32 records (see
    ``metisfl_amd.datasets.synthetic.synthetic_mlm``)."""

    graph_steps = 1  # a ~15 ms step: one graph per update already hides the launch

    def __init__(self, batch_size: int, device="cpu", optimizer: OptimizerSpec | None = None, seed: int = 0,
                 config: BertConfig | dict | None = None):
        if isinstance(config, dict):
            config = BertConfig(**config)
        self.cfg = c = config or BERT_BASE
        assert c.seq == BO.SEQ and c.hidden == c.heads * BO.HEAD_DIM, "attention kernel: seq 128, head dim 64"
        assert c.hidden % 256 == 0 and c.ffn % 8 == 0
        self.B = batch_size
        self.device = torch.device(device)
        self.input_shape = (2 * c.rec_stride,)
        self.state = FlatState(self._specs(), self.device,
                               optimizer or OptimizerSpec("adam_weight_decay", 1e-4, weight_decay=0.01,
                                                          epsilon=1e-6),
                               seed=seed)
        self._alloc()
        dev = self.device
        self.xb = torch.zeros((self.B,) + self.input_shape, dtype=torch.bfloat16, device=dev)
        self.rec = self.xb.view(torch.int32)
        self.yb = torch.zeros(self.B, dtype=torch.int32, device=dev)
        self.stats = torch.zeros(4, dtype=torch.float32, device=dev)
        self.eval_step_ctr = torch.zeros(1, dtype=torch.int32, device=dev)
        self._train_graph = None
        self._train_graph_k = None
        self._train_graph_ds = None
        self._eval_graph = None
        self._eval_graph_ds = None

    # ---- parameters --------------------------------------------------------------
    def _specs(self) -> list[VarSpec]:
        c = self.cfg
        H, F, Vp = c.hidden, c.ffn, c.vocab_padded
        s = [VarSpec("emb.word", (Vp, H), init="normal", live_rows=c.vocab),
             VarSpec("emb.pos", (c.max_pos, H), init="normal"),
             VarSpec("emb.type", (c.type_vocab, H), init="normal"),
             VarSpec("emb.ln.gamma", (H,), init="ones"), VarSpec("emb.ln.beta", (H,))]
        for i in range(c.layers):
            p = f"layer{i}."
            s += [VarSpec(p + "qkv.w", (3 * H, H), init="normal"), VarSpec(p + "qkv.b", (3 * H,)),
                  VarSpec(p + "out.w", (H, H), init="normal"), VarSpec(p + "out.b", (H,)),
                  VarSpec(p + "ln1.gamma", (H,), init="ones"), VarSpec(p + "ln1.beta", (H,)),
                  VarSpec(p + "ffn1.w", (F, H), init="normal"), VarSpec(p + "ffn1.b", (F,)),
                  VarSpec(p + "ffn2.w", (H, F), init="normal"), VarSpec(p + "ffn2.b", (H,)),
                  VarSpec(p + "ln2.gamma", (H,), init="ones"), VarSpec(p + "ln2.beta", (H,))]
        s += [VarSpec("head.w", (H, H), init="normal"), VarSpec("head.b", (H,)),
              VarSpec("head.ln.gamma", (H,), init="ones"), VarSpec("head.ln.beta", (H,)),
              VarSpec("head.dec.b", (Vp,))]
        return s

    def _alloc(self) -> None:
        c, dev = self.cfg, self.device
        B, T, H, F, P = self.B, c.seq, c.hidden, c.ffn, c.max_pred
        M, R = B * T, B * P
        e = lambda *shape: torch.zeros(shape, dtype=torch.bfloat16, device=dev)  # noqa: E731
        f = lambda n: torch.zeros(n, dtype=torch.float32, device=dev)  # noqa: E731
        self.emb_x = e(M, H)
        self.emb_mean, self.emb_rstd = f(M), f(M)
        # xs[0]: embedding LN output; xs[i + 1]: layer i output (= layer i+1 input)
        self.xs = [e(M, H) for _ in range(c.layers + 1)]
        self.acts = []
        for i in range(c.layers):
            self.acts.append(dict(
                x=self.xs[i], out=self.xs[i + 1], qkv=e(M, 3 * H), ctx=e(M, H), lse=f(B * c.heads * T),
                ao=e(M, H), a=e(M, H), m1=f(M), r1=f(M), z=e(M, F), h=e(M, F), fo=e(M, H), m2=f(M), r2=f(M)))
        self.out = self.xs[-1]
        # head
        self.hm, self.tz, self.th, self.u = e(R, H), e(R, H), e(R, H), e(R, H)
        self.hm_mean, self.hm_rstd = f(R), f(R)
        self.logits = e(R, c.vocab_padded)
        self.dlogits = e(R, c.vocab_padded)
        # gradient scratch (shared by all layers)
        self.g_out = [e(M, H), e(M, H)]
        self.g_fo, self.g_a, self.g_ao, self.g_ctx = e(M, H), e(M, H), e(M, H), e(M, H)
        self.g_h, self.g_z = e(M, F), e(M, F)
        self.g_qkv = e(M, 3 * H)
        self.g_u, self.g_th, self.g_tz, self.g_hm = e(R, H), e(R, H), e(R, H), e(R, H)
        # word-embedding gradient by token sort + segmented sum (no same-address
        # atomics for [MASK] / [CLS] rows); device only
        self.emb_scratch = BO.EmbGradScratch(M, H, c.vocab, dev) if torch.device(dev).type == "cuda" else None

    def all_layers(self):
        return []

    # shorthand views
    def _w(self, name):
        return self.state.bf16(name)

    def _p(self, name):
        return self.state.view(name)

    def _g(self, name):
        return self.state.grad(name)

    # ---- forward ---------------------------------------------------------------------
    def _forward(self) -> torch.Tensor:
        c = self.cfg
        B, T, H, F = self.B, c.seq, c.hidden, c.ffn
        M = B * T
        BO.emb_ln_fwd(self.rec, c.rec_stride, B, T, self._w("emb.word"), self._w("emb.pos"), self._w("emb.type"),
                      self.emb_x, self._p("emb.ln.gamma"), self._p("emb.ln.beta"), self.xs[0], self.emb_mean,
                      self.emb_rstd, H, c.eps)
        scale = 1.0 / np.sqrt(BO.HEAD_DIM)
        for i, A in enumerate(self.acts):
            p = f"layer{i}."
            BO.gemm_fwd(A["x"], self._w(p + "qkv.w"), A["qkv"], M, 3 * H, H, bias=self._p(p + "qkv.b"))
            BO.attn_fwd(A["qkv"], A["ctx"], A["lse"], B, c.heads, scale)
            BO.gemm_fwd(A["ctx"], self._w(p + "out.w"), A["ao"], M, H, H, bias=self._p(p + "out.b"), resid=A["x"])
            BO.ln_fwd(A["ao"], self._p(p + "ln1.gamma"), self._p(p + "ln1.beta"), A["a"], A["m1"], A["r1"], M, H,
                      c.eps)
            BO.gemm_fwd(A["a"], self._w(p + "ffn1.w"), A["z"], M, F, H, bias=self._p(p + "ffn1.b"), act_out=A["h"],
                        act_grad=GELU_GRAD)
            BO.gemm_fwd(A["h"], self._w(p + "ffn2.w"), A["fo"], M, H, F, bias=self._p(p + "ffn2.b"), resid=A["a"])
            BO.ln_fwd(A["fo"], self._p(p + "ln2.gamma"), self._p(p + "ln2.beta"), A["out"], A["m2"], A["r2"], M,
                      H, c.eps)
        return self.out

    def _head(self, train: bool) -> None:
        c = self.cfg
        B, T, H, P, Vp = self.B, c.seq, c.hidden, c.max_pred, c.vocab_padded
        R = B * P
        BO.mlm_gather(self.out, self.rec, c.rec_stride, B, T, P, self.hm, H)
        BO.gemm_fwd(self.hm, self._w("head.w"), self.tz, R, H, H, bias=self._p("head.b"), act_out=self.th)
        BO.ln_fwd(self.th, self._p("head.ln.gamma"), self._p("head.ln.beta"), self.u, self.hm_mean, self.hm_rstd,
                  R, H, c.eps)
        BO.gemm_fwd(self.u, self._w("emb.word"), self.logits, R, Vp, H, bias=self._p("head.dec.b"))
        BO.vocab_xent(self.logits, self.rec, c.rec_stride, B, T, P, c.vocab, Vp, self.stats,
                      dlogits=self.dlogits if train else None)

    # ---- backward ----------------------------------------------------------------
    def _backward(self) -> None:
        c = self.cfg
        B, T, H, F, P, Vp = self.B, c.seq, c.hidden, c.ffn, c.max_pred, c.vocab_padded
        M, R = B * T, B * P
        g = self._g
        # head
        BO.colsum(self.dlogits, g("head.dec.b"), R, Vp)
        BO.gemm_wgrad(self.u, self.dlogits, g("emb.word"), R, Vp, H, accumulate=True)  # tied decoder
        BO.gemm_dgrad(self.dlogits, self._w("emb.word"), self.g_u, R, Vp, H)
        BO.ln_bwd(self.g_u, self.th, self.hm_mean, self.hm_rstd, self._p("head.ln.gamma"), self.g_th,
                  g("head.ln.gamma"), g("head.ln.beta"), R, H)
        BO.gelu_bwd(self.g_th, self.tz, self.g_tz, R, H, dbias=g("head.b"))
        BO.gemm_wgrad(self.hm, self.g_tz, g("head.w"), R, H, H, zeroed=True)
        BO.gemm_dgrad(self.g_tz, self._w("head.w"), self.g_hm, R, H, H)
        dout = self.g_out[0]
        BO.mlm_scatter(self.g_hm, self.rec, c.rec_stride, B, T, P, dout, H)
        scale = 1.0 / np.sqrt(BO.HEAD_DIM)
        for i in reversed(range(c.layers)):
            A, p = self.acts[i], f"layer{i}."
            dx = self.g_out[1] if dout is self.g_out[0] else self.g_out[0]
            # the LN input's gradient g_fo feeds the FFN AND the residual
            # branch: the FFN1 dgrad below adds it in its output stage (no
            # second copy of it written here to accumulate into)
            BO.ln_bwd(dout, A["fo"], A["m2"], A["r2"], self._p(p + "ln2.gamma"), self.g_fo, g(p + "ln2.gamma"),
                      g(p + "ln2.beta"), M, H, dx2=None if RESID_DGRAD else self.g_a, dbias_prev=g(p + "ffn2.b"))
            if not FFN_WGRAD2:
                BO.gemm_wgrad(A["h"], self.g_fo, g(p + "ffn2.w"), M, H, F, zeroed=True)
            # GELU backward + FFN1 bias gradient in the dgrad epilogue: saves the
            # 300 MB round trip of a separate gelu_bwd (scripts/gelu_fuse_probe.py:
            # 128-134 us fused vs 137-150 unfused, with the A&S erf of common.h)
            BO.gemm_dgrad_gelu(self.g_fo, self._w(p + "ffn2.w"), self.g_z, A["z"], M, H, F,
                               dbias=g(p + "ffn1.b"), pre=GELU_GRAD)
            if FFN_WGRAD2:
                BO.gemm_wgrad2(A["h"], self.g_fo, g(p + "ffn2.w"), H, F, A["a"], self.g_z, g(p + "ffn1.w"), F, H, M)
            else:
                BO.gemm_wgrad(A["a"], self.g_z, g(p + "ffn1.w"), M, F, H, zeroed=True)
            if RESID_DGRAD:
                BO.gemm_dgrad(self.g_z, self._w(p + "ffn1.w"), self.g_a, M, F, H, resid=self.g_fo)
            else:
                BO.gemm_dgrad(self.g_z, self._w(p + "ffn1.w"), self.g_a, M, F, H, accumulate=True)
            BO.ln_bwd(self.g_a, A["ao"], A["m1"], A["r1"], self._p(p + "ln1.gamma"), self.g_ao, g(p + "ln1.gamma"),
                      g(p + "ln1.beta"), M, H, dx2=None if RESID_DGRAD else dx, dbias_prev=g(p + "out.b"))
            if not WGRAD2:
                BO.gemm_wgrad(A["ctx"], self.g_ao, g(p + "out.w"), M, H, H, zeroed=True)
            BO.gemm_dgrad(self.g_ao, self._w(p + "out.w"), self.g_ctx, M, H, H)
            BO.attn_bwd(A["qkv"], A["ctx"], A["lse"], self.g_ctx, self.g_qkv, B, c.heads, scale,
                        dbias=g(p + "qkv.b"))
            if WGRAD2:
                # the attention-output and QKV weight gradients in one grouped
                # launch: alone the 768 x 768 one needs ~28 short split-K
                # slices to fill the chip (gemm_big.hip gemm_pp_group_kernel)
                BO.gemm_wgrad2(A["ctx"], self.g_ao, g(p + "out.w"), H, H, A["x"], self.g_qkv, g(p + "qkv.w"),
                               3 * H, H, M)
            else:
                BO.gemm_wgrad(A["x"], self.g_qkv, g(p + "qkv.w"), M, 3 * H, H, zeroed=True)
            if RESID_DGRAD:
                BO.gemm_dgrad(self.g_qkv, self._w(p + "qkv.w"), dx, M, 3 * H, H, resid=self.g_ao)
            else:
                BO.gemm_dgrad(self.g_qkv, self._w(p + "qkv.w"), dx, M, 3 * H, H, accumulate=True)
            dout = dx
        BO.emb_ln_bwd(dout, self.emb_x, self.emb_mean, self.emb_rstd, self._p("emb.ln.gamma"), self.rec,
                      c.rec_stride, B, T, g("emb.word"), g("emb.pos"), g("emb.type"), g("emb.ln.gamma"),
                      g("emb.ln.beta"), H, scratch=self.emb_scratch)

    # ---- step bodies (captured into hipGraphs by StaticNet) ------------------------
    def _train_body(self, ds: DeviceDataset) -> None:
        st = self.state
        if not self.zero_grad_in_optimizer:
            st.grad32.zero_()
        K.gather_batch(ds.x, ds.y, ds.perm, st.step, ds.steps_per_epoch, self.B, self.xb, self.yb)
        self._forward()
        self._head(train=True)
        self._backward()
        if not st.optimizer_step(zero_grad=self.zero_grad_in_optimizer, tick=True):
            opt_ops.tick(st.step, 1)

    def _eval_body(self, ds: DeviceDataset) -> None:
        K.gather_batch(ds.x, ds.y, ds.perm, self.eval_step_ctr, ds.steps_per_epoch, self.B, self.xb, self.yb)
        self._forward()
        self._head(train=False)
        opt_ops.tick(self.eval_step_ctr, 1)

    # ---- data ----------------------------------------------------------------------
    def make_dataset(self, records, y=None, seed: int = 0, shuffle: bool = True,
                     batch_size: int | None = None) -> DeviceDataset:
        """``records``: int32 [N][rec_stride] (see ``synthetic_mlm``)."""
        r = torch.as_tensor(np.ascontiguousarray(records, dtype=np.int32))
        assert r.shape[1] == self.cfg.rec_stride, (r.shape, self.cfg.rec_stride)
        x = r.view(torch.bfloat16).to(self.device)
        yl = torch.zeros(r.shape[0], dtype=torch.int32, device=self.device)
        return DeviceDataset(x, yl, batch_size or self.B, seed=seed, shuffle=shuffle)

    def tokens_per_step(self) -> int:
        return self.B * self.cfg.seq

    def flops_per_step(self) -> float:
        """Model FLOPs of one training step (fwd + bwd = 3x fwd GEMM FLOPs)."""
        c = self.cfg
        M, R = self.B * c.seq, self.B * c.max_pred
        H, F = c.hidden, c.ffn
        layer = 2 * M * H * (3 * H + H + 2 * F) + 2 * 2 * self.B * c.heads * c.seq * c.seq * 64
        head = 2 * R * H * (H + c.vocab_padded)
        return 3.0 * (c.layers * layer + head)
