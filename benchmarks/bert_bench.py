#!/usr/bin/env python3
"""BERT-base masked-LM federation benchmark (SURVEY §7.2 step 10 workload).

One step = ONE synchronous FedAvg round: every learner (one process per GPU)
runs ``--local-steps`` masked-LM updates (batch ``--batch`` x seq 128, 20
predictions per sequence, AdamW) on its synthetic shard, then the round
closes with a NUM_TRAINING_EXAMPLES-weighted FedAvg of the whole 110M-param
model (scale kernel + one RCCL all-reduce).  Weak scaling: per-learner work
is fixed.  Prints one JSON line (rank 0) with tokens/s over the whole job and
the model TFLOP/s per GPU.

  python benchmarks/bert_bench.py --steps 3 --warmup 1
  python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \
      --master-port 29511 benchmarks/bert_bench.py --gpus 8
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3, help="timed federation rounds")
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--local-steps", type=int, default=20)
    ap.add_argument("--lr", type=float, default=1e-4)
    ap.add_argument("--learners-per-gpu", type=int, default=1,
                    help="co-located learners per GPU (models/colocated.py), each on its own HIP stream")
    ap.add_argument("--json-out", type=str, default="")
    args = ap.parse_args()
    from metisfl_amd.utils.launch import ensure_world
    rc = ensure_world(args.gpus, __file__)
    if rc is not None:
        return rc

    import torch

    from metisfl_amd.datasets import synthetic_mlm
    from metisfl_amd.models.bert import BertMLM
    from metisfl_amd.ops.optim import OptimizerSpec
    from metisfl_amd.parallel.comm import Comm
    from metisfl_amd.parallel.federation import CollectiveFederation, FederationConfig

    comm = Comm()
    n = comm.world
    dev = comm.device
    opt = OptimizerSpec("adam_weight_decay", args.lr, weight_decay=0.01, epsilon=1e-6)
    L = max(1, args.learners_per_gpu)
    nets, dss = [], []
    for j in range(L):
        gi = comm.rank * L + j
        net = BertMLM(batch_size=args.batch, device=dev, optimizer=opt, seed=7)
        c = net.cfg
        rec = synthetic_mlm(args.batch * args.local_steps, c.seq, c.max_pred, c.vocab, seed=100 + gi,
                            rec_stride=c.rec_stride)
        nets.append(net)
        dss.append(net.make_dataset(rec, seed=gi))
    net = nets[0]
    cfg = FederationConfig(protocol="synchronous", batch_size=args.batch, local_epochs=1, evaluate_test=False)
    fed = CollectiveFederation(comm, nets, dss, cfg)

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)

    for _ in range(args.warmup):
        fed.run_round()
    comm.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        fed.run_round()
        if comm.rank == 0:
            r = fed.history[-1]
            print(f"[bert] round {r.global_iteration}: {r.round_ms:.1f} ms (train {r.train_ms:.1f}, "
                  f"agg {r.aggregation_ms:.2f}) loss {r.learner_meta[:, 4].mean():.3f}", file=sys.stderr,
                  flush=True)
    comm.barrier()
    sync()
    elapsed = comm.all_max(time.perf_counter() - t0)
    round_ms = elapsed * 1e3 / max(1, args.steps)
    timed = fed.history[-args.steps:]
    train_ms = sum(r.train_ms for r in timed) / max(1, len(timed))
    step_ms = train_ms / args.local_steps
    tokens = n * L * args.local_steps * net.tokens_per_step()
    out = {
        "metric": "BERT-base MLM federation throughput (tokens/s, whole job)",
        "value": tokens / (round_ms / 1e3),
        "unit": "tokens/s",
        "n_gpus": n,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round_ms,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "bf16",
        "data": "synthetic MLM records (bigram token chains, 20 masks/seq), random-init BERT-base",
        "config": {"model": "bert-base-mlm (110M, post-LN, tied decoder)", "global_batch": args.batch * n * L,
                   "learners": n * L, "learners_per_gpu": L,
                   "seq_len": c.seq, "local_steps": args.local_steps, "optimizer": "adamw",
                   "aggregation": "FedAvg(NUM_TRAINING_EXAMPLES), RCCL all-reduce",
                   "parallelism": f"fedavg-dp{n}"},
        "local_step_ms": step_ms,  # per update of each learner (co-located: the GPU runs L meanwhile)
        "model_tflops_per_gpu": L * net.flops_per_step() / (step_ms / 1e3) / 1e12,
        "aggregation_ms_mean": sum(r.aggregation_ms for r in timed) / max(1, len(timed)),
    }
    if comm.rank == 0:
        line = json.dumps(out)
        print(line, flush=True)
        if args.json_out:
            with open(args.json_out, "w") as f:
                f.write(line + "\n")
    comm.close()
    return 0


if __name__ == "__main__":
    from metisfl_amd.utils.launch import exit_process
    exit_process(main())  # no interpreter finalisation behind live c10d threads (utils/launch.py)
