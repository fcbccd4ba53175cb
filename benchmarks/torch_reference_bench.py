#!/usr/bin/env python3
"""Reference-style learner step on MI355X in plain PyTorch-ROCm (comparison point).

The reference publishes no round time (BASELINE.json ``"published": {}``).  Its
learners delegate local training to a framework training loop: Keras ``fit``
(metisfl/models/keras/keras_model_ops.py:156-164) or a user ``fit`` over a
PyTorch module (metisfl/models/pytorch/pytorch_model_ops.py:106-118, CPU-only
there).  This script measures what that style of learner costs on the SAME
MI355X for the SAME work as ``bench.py`` -- one local update of CIFAR-10
ResNet-18 at batch 32 with MomentumSGD (and, with ``--model bert``, one
BERT-base masked-LM update at batch 128 x 128 tokens with AdamW) -- in
several PyTorch configurations, all on MIOpen / hipBLASLt kernels:

  fp32            eager, NCHW, fp32            (what a naive port runs)
  bf16_cl         eager, channels_last, bf16 autocast
  bf16_cl_graph   bf16_cl captured into a CUDA(HIP) graph, replayed per step

and prints ms/step plus the implied federation round time for bench.py's
default config (50k samples / N learners x 4 local epochs, batch 32).  The
numbers are committed under profiles/ and quoted in BASELINE.md next to the
framework's own measurements.

  python benchmarks/torch_reference_bench.py --model resnet18 --steps 200
  python benchmarks/torch_reference_bench.py --model bert --steps 20
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import torch
import torch.nn as nn
import torch.nn.functional as F


class BasicBlock(nn.Module):
    def __init__(self, cin, cout, stride):
        super().__init__()
        self.c1 = nn.Conv2d(cin, cout, 3, stride, 1, bias=False)
        self.b1 = nn.BatchNorm2d(cout)
        self.c2 = nn.Conv2d(cout, cout, 3, 1, 1, bias=False)
        self.b2 = nn.BatchNorm2d(cout)
        self.sc = None
        if stride != 1 or cin != cout:
            self.sc = nn.Sequential(nn.Conv2d(cin, cout, 1, stride, bias=False), nn.BatchNorm2d(cout))

    def forward(self, x):
        o = F.relu(self.b1(self.c1(x)))
        o = self.b2(self.c2(o))
        return F.relu(o + (x if self.sc is None else self.sc(x)))


class TorchResNet18(nn.Module):
    """Same topology as metisfl_amd.models.resnet.ResNet18 (CIFAR stem, 11.17M params)."""

    def __init__(self, num_classes=10):
        super().__init__()
        self.stem = nn.Sequential(nn.Conv2d(3, 64, 3, 1, 1, bias=False), nn.BatchNorm2d(64), nn.ReLU())
        layers, cin = [], 64
        for c, s in zip((64, 128, 256, 512), (1, 2, 2, 2)):
            layers += [BasicBlock(cin, c, s), BasicBlock(c, c, 1)]
            cin = c
        self.layers = nn.Sequential(*layers)
        self.fc = nn.Linear(512, num_classes)

    def forward(self, x):
        h = self.layers(self.stem(x))
        return self.fc(torch.flatten(F.adaptive_avg_pool2d(h, 1), 1))


def _time(fn, steps, warmup):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e3 / steps


def resnet_variants(args, dev):
    out = {}
    B = args.batch
    n_train = 50000
    x_all = torch.randn(n_train if args.full_shard else 4096, 3, 32, 32, device=dev)
    y_all = torch.randint(0, 10, (x_all.shape[0],), device=dev)
    for name in args.variants:
        torch.manual_seed(0)
        model = TorchResNet18().to(dev)
        cl = name.startswith("bf16_cl")
        if cl:
            model = model.to(memory_format=torch.channels_last)
        opt = torch.optim.SGD(model.parameters(), lr=0.005, momentum=0.75,
                              foreach=True)
        xs = torch.empty(B, 3, 32, 32, device=dev)
        ys = torch.empty(B, dtype=torch.long, device=dev)
        if cl:
            xs = xs.to(memory_format=torch.channels_last)
        state = {"i": 0}

        def load():
            i = state["i"]
            state["i"] = (i + B) % (x_all.shape[0] - B)
            xs.copy_(x_all[i:i + B])
            ys.copy_(y_all[i:i + B])

        def step():
            opt.zero_grad(set_to_none=False)
            with torch.autocast("cuda", dtype=torch.bfloat16, enabled=name != "fp32"):
                loss = F.cross_entropy(model(xs), ys)
            loss.backward()
            opt.step()

        if name.endswith("_graph"):
            load()
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                for _ in range(3):
                    step()
            torch.cuda.current_stream().wait_stream(s)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                step()

            def run():
                load()
                g.replay()
        else:
            def run():
                load()
                step()

        ms = _time(run, args.steps, args.warmup)
        updates = math.ceil(n_train / B) * args.local_epochs  # 1 learner
        out[name] = {"ms_per_step": ms,
                     "implied_round_ms_1learner": ms * updates,
                     "implied_round_ms_8learners": ms * math.ceil(n_train / 8 / B) * args.local_epochs}
        print(f"[torch-ref] resnet18 {name}: {ms:.3f} ms/step", file=sys.stderr, flush=True)
        del model, opt
        torch.cuda.empty_cache()
    return out


def bert_variants(args, dev):
    from transformers import BertConfig, BertForMaskedLM

    out = {}
    B, T, P = args.bert_batch, 128, 20
    cfg = BertConfig()  # bert-base-uncased shape: 12 x 768, 30522 vocab
    for name in args.variants:
        if name == "fp32":
            continue  # AdamW fp32 BERT is not a fair bf16 comparison point
        torch.manual_seed(0)
        cfg._attn_implementation = "sdpa"
        model = BertForMaskedLM(cfg).to(dev)
        opt = torch.optim.AdamW(model.parameters(), lr=1e-4, weight_decay=0.01, foreach=True)
        ids = torch.randint(0, cfg.vocab_size, (B, T), device=dev)
        labels = torch.full((B, T), -100, dtype=torch.long, device=dev)
        pos = torch.rand(B, T, device=dev).argsort(1)[:, :P]
        labels.scatter_(1, pos, torch.randint(0, cfg.vocab_size, (B, P), device=dev))

        def step():
            opt.zero_grad(set_to_none=False)
            with torch.autocast("cuda", dtype=torch.bfloat16):
                loss = model(input_ids=ids, labels=labels).loss
            loss.backward()
            opt.step()

        run = step
        if name.endswith("_graph"):
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                for _ in range(3):
                    step()
            torch.cuda.current_stream().wait_stream(s)
            g = torch.cuda.CUDAGraph()
            try:
                with torch.cuda.graph(g):
                    step()
                run = g.replay
            except Exception as e:  # noqa: BLE001 -- report, keep the eager number
                print(f"[torch-ref] bert graph capture failed: {e}", file=sys.stderr)
                continue
        ms = _time(run, args.steps, args.warmup)
        out[name] = {"ms_per_step": ms, "tokens_per_s": B * T / (ms / 1e3)}
        print(f"[torch-ref] bert-base {name}: {ms:.2f} ms/step", file=sys.stderr, flush=True)
        del model, opt
        torch.cuda.empty_cache()
    return out


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", choices=("resnet18", "bert"), default="resnet18")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--bert-batch", type=int, default=128)
    ap.add_argument("--local-epochs", type=int, default=4)
    ap.add_argument("--full-shard", action="store_true")
    ap.add_argument("--variants", nargs="+", default=["fp32", "bf16_cl", "bf16_cl_graph"])
    ap.add_argument("--json-out", default="")
    args = ap.parse_args()
    if not torch.cuda.is_available():
        print("no GPU", file=sys.stderr)
        return 1
    dev = torch.device("cuda:0")
    torch.backends.cudnn.benchmark = True
    res = resnet_variants(args, dev) if args.model == "resnet18" else bert_variants(args, dev)
    line = json.dumps({"model": args.model, "device": torch.cuda.get_device_name(0),
                       "torch": torch.__version__, "results": res})
    print(line, flush=True)
    if args.json_out:
        with open(args.json_out, "w") as f:
            f.write(line + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
