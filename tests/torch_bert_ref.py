"""Independent fp32 torch.nn BERT masked-LM (post-LN encoder, tied decoder)
used as an oracle for the HIP BERT learner (models/bert.py).  Written from
the architecture (Devlin et al.; HF BertForMaskedLM without dropout / NSP),
not from the framework's ops: nn.Linear / F.layer_norm / exact-erf GELU /
softmax attention / F.cross_entropy.  ``load_from_flat`` copies the learner's
fp32 master weights; ``grads_like_flat`` returns the oracle's gradients under
the learner's parameter names."""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F


class _Layer(nn.Module):
    def __init__(self, H, F_, heads, eps):
        super().__init__()
        self.qkv = nn.Linear(H, 3 * H)
        self.out = nn.Linear(H, H)
        self.ln1 = nn.LayerNorm(H, eps=eps)
        self.ffn1 = nn.Linear(H, F_)
        self.ffn2 = nn.Linear(F_, H)
        self.ln2 = nn.LayerNorm(H, eps=eps)
        self.heads = heads

    def forward(self, x):
        B, T, H = x.shape
        d = H // self.heads
        q, k, v = self.qkv(x).view(B, T, 3, self.heads, d).permute(2, 0, 3, 1, 4)
        att = torch.softmax(q @ k.transpose(-1, -2) / d ** 0.5, dim=-1)
        ctx = (att @ v).permute(0, 2, 1, 3).reshape(B, T, H)
        a = self.ln1(self.out(ctx) + x)
        return self.ln2(self.ffn2(F.gelu(self.ffn1(a))) + a)


class TorchBertMLM(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        H, Vp = cfg.hidden, cfg.vocab_padded
        self.cfg = cfg
        self.word = nn.Parameter(torch.zeros(Vp, H))
        self.pos = nn.Parameter(torch.zeros(cfg.max_pos, H))
        self.typ = nn.Parameter(torch.zeros(cfg.type_vocab, H))
        self.emb_ln = nn.LayerNorm(H, eps=cfg.eps)
        self.layers = nn.ModuleList(_Layer(H, cfg.ffn, cfg.heads, cfg.eps) for _ in range(cfg.layers))
        self.head = nn.Linear(H, H)
        self.head_ln = nn.LayerNorm(H, eps=cfg.eps)
        self.dec_b = nn.Parameter(torch.zeros(Vp))

    def forward(self, rec: torch.Tensor) -> torch.Tensor:
        """rec: int [B][rec_stride] records (datasets.synthetic_mlm); returns
        the mean masked-LM cross-entropy over the masked positions."""
        c = self.cfg
        T, P = c.seq, c.max_pred
        tok, pos, ids = rec[:, :T].long(), rec[:, T:T + P].long(), rec[:, T + P:T + 2 * P].long()
        x = self.emb_ln(self.word[tok] + self.pos[:T][None] + self.typ[0])
        for layer in self.layers:
            x = layer(x)
        sel = torch.gather(x, 1, pos[..., None].expand(-1, -1, x.shape[-1]))
        u = self.head_ln(F.gelu(self.head(sel)))
        logits = u @ self.word.t() + self.dec_b
        return F.cross_entropy(logits[..., :c.vocab].reshape(-1, c.vocab), ids.reshape(-1))

    def _names(self):
        m = {"emb.word": self.word, "emb.pos": self.pos, "emb.type": self.typ,
             "emb.ln.gamma": self.emb_ln.weight, "emb.ln.beta": self.emb_ln.bias,
             "head.w": self.head.weight, "head.b": self.head.bias, "head.ln.gamma": self.head_ln.weight,
             "head.ln.beta": self.head_ln.bias, "head.dec.b": self.dec_b}
        for i, L in enumerate(self.layers):
            p = f"layer{i}."
            m.update({p + "qkv.w": L.qkv.weight, p + "qkv.b": L.qkv.bias, p + "out.w": L.out.weight,
                      p + "out.b": L.out.bias, p + "ln1.gamma": L.ln1.weight, p + "ln1.beta": L.ln1.bias,
                      p + "ffn1.w": L.ffn1.weight, p + "ffn1.b": L.ffn1.bias, p + "ffn2.w": L.ffn2.weight,
                      p + "ffn2.b": L.ffn2.bias, p + "ln2.gamma": L.ln2.weight, p + "ln2.beta": L.ln2.bias})
        return m

    @torch.no_grad()
    def load_from_flat(self, state) -> None:
        for name, p in self._names().items():
            p.copy_(state.view(name).detach().float().cpu().reshape(p.shape))

    def grads_like_flat(self) -> dict:
        return {n: p.grad.detach().clone() for n, p in self._names().items()}
