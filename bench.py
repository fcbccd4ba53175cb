#!/usr/bin/env python3
"""Federation-round benchmark: 8-learner sync FedAvg, CIFAR-10, ResNet-18.

Metric (BASELINE.json): "federation-round time (ms) + rounds/sec, 8-learner
FedAvg CIFAR-10 ResNet-18".  One benchmark "step" is ONE federation round:

  every one of the ``--learners`` (default 8) learners trains its IID shard of
  the 50,000-image CIFAR-10 training set for ``--local-epochs`` epochs
  (batch 32, MomentumSGD lr 0.005 / momentum 0.75: the reference's CIFAR-10
  experiment config, examples/config/cifar10/
  test_localhost_synchronous_momentumsgd.yaml), evaluates its test shard
  (the reference learner evaluates at task end, keras_model_ops.py:174-176),
  then the round closes with NUM_TRAINING_EXAMPLES-weighted FedAvg (scale
  kernel + one RCCL all-reduce) leaving the community model resident on every
  GPU.

The federation is the same 8 learners at every GPU count: one process per
GPU hosts learners/N of them (models/colocated.py: each with its own model,
optimizer state, shard and step graphs, replayed on its own HIP stream, so
co-located learners share the GPU concurrently -- the reference likewise
runs several learners per GPU, e.g. 10 learners on 5 GPUs in
examples/config/cifar10/test_localhost_synchronous_momentumsgd.yaml).  At
N=8 that is one learner per MI355X (BASELINE config 2).  The dataset is
fixed (50k train / 10k test images) and split across the learners, so the
federation -- shards, step budgets, FedAvg weights -- and the total work per
round do not depend on N: scaling is "strong" and ``value`` (rounds/s of the
whole federation) is the whole-job aggregate.
Data are synthetic tensors of CIFAR-10's shape, weights random-init of the
ResNet-18 architecture (no network for datasets/checkpoints).

Precision: ``--dtype fp32`` (default) is the reference's precision -- the
reference trains fp32 Keras models (examples/keras/models/cifar_cnn.py:19-41,
keras_model_ops.py:117-197) -- on the fp32 convolution kernels (conv32.hip:
fp32 storage and accumulation, bf16x3 split products by default, exact fp32
MFMA products with ``--conv-products exact``); ``--dtype bf16`` is the
mixed-precision option, reported separately.

Launch: ``python bench.py`` (1 GPU), ``python bench.py --gpus N`` (spawns its
own N rank processes before touching any GPU), or under
``python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1
--master-port P bench.py --gpus N``.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

METRIC = "federation-round time (ms) + rounds/sec, 8-learner FedAvg CIFAR-10 ResNet-18"
BASELINE_VALUE = None  # BASELINE.json "published": {} -- no reference number exists


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--learners", type=int, default=8,
                    help="federation learners (BASELINE: 8), learners/N co-located on each GPU")
    ap.add_argument("--steps", type=int, default=3, help="timed federation rounds")
    ap.add_argument("--warmup", type=int, default=1, help="untimed federation rounds")
    ap.add_argument("--local-epochs", type=int, default=4)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--train-size", type=int, default=50000)
    ap.add_argument("--test-size", type=int, default=10000)
    ap.add_argument("--no-eval", action="store_true")
    ap.add_argument("--sync-community-eval", action="store_true",
                    help="evaluate the community model at the end of its round instead of in the background")
    ap.add_argument("--lr", type=float, default=0.005)
    ap.add_argument("--momentum", type=float, default=0.75)
    ap.add_argument("--secure-aggregation", action="store_true",
                    help="BASELINE config 4: CKKS secure aggregation (device encrypt / int64 "
                         "all-reduce of ciphertexts / device decrypt)")
    ap.add_argument("--dtype", choices=("fp32", "bf16"), default="fp32",
                    help="compute precision: fp32 = reference precision (default), bf16 = mixed")
    ap.add_argument("--conv-products", choices=("exact", "bf16x3"), default=None,
                    help="fp32 convolution products: exact fp32 MFMA, or bf16x3 split products "
                         "with fp32 storage/accumulation (default: ResNet18's default)")
    ap.add_argument("--exact-updates", type=int, default=300,
                    help="fp32 bf16x3 runs: also time this many local updates with exact fp32 products "
                         "(0: skip); reported as conv_products_exact")
    ap.add_argument("--width-mult", type=float, default=1.0, help=argparse.SUPPRESS)  # CPU plumbing tests only
    ap.add_argument("--checkpoint-every", type=int, default=0,
                    help="also checkpoint the federation every K rounds inside the timed rounds (device-staged, "
                         "written in the background: parallel/checkpoint.py); reports checkpoint_ms")
    ap.add_argument("--checkpoint-dir", type=str, default="")
    ap.add_argument("--json-out", type=str, default="")
    args = ap.parse_args()

    from metisfl_amd.utils.launch import ensure_world
    rc = ensure_world(args.gpus, __file__)
    if rc is not None:
        return rc

    import numpy as np
    import torch

    from metisfl_amd.models.resnet import ResNet18
    from metisfl_amd.ops.optim import OptimizerSpec
    from metisfl_amd.parallel.comm import Comm
    from metisfl_amd.parallel.federation import CollectiveFederation, FederationConfig

    comm = Comm()
    n = comm.world
    dev = comm.device
    torch.manual_seed(1234 + comm.rank)
    nl = max(args.learners, n)
    if nl % n:
        print(f"[bench] error: {nl} learners do not split evenly over {n} GPUs", file=sys.stderr)
        return 2
    L = nl // n  # learners co-located on this GPU

    def share(total: int, i: int) -> int:
        return total // nl + (1 if i < total % nl else 0)

    from metisfl_amd.models.colocated import configure_regime
    configure_regime(L)  # kernel choices for L learners per GPU, before the models are built
    opt = OptimizerSpec("momentum_sgd", args.lr, momentum=args.momentum)
    nets, train_dss, test_dss = [], [], []
    for j in range(L):
        gi = comm.rank * L + j  # global learner index
        # IID shard of the fixed-size dataset (strong scaling)
        g = torch.Generator(device=dev)
        g.manual_seed(1000 + gi)
        xtr = torch.randn((share(args.train_size, gi), 32, 32, 3), generator=g, device=dev)
        ytr = torch.randint(0, 10, (xtr.shape[0],), generator=g, device=dev)
        xte = torch.randn((share(args.test_size, gi), 32, 32, 3), generator=g, device=dev)
        yte = torch.randint(0, 10, (xte.shape[0],), generator=g, device=dev)
        net = ResNet18(batch_size=args.batch, device=dev, optimizer=opt, seed=7, dtype=args.dtype,
                       width_mult=args.width_mult, conv_products=args.conv_products)
        nets.append(net)
        train_dss.append(net.make_dataset(xtr, ytr, seed=gi))
        test_dss.append(net.make_dataset(xte, yte, seed=gi, shuffle=False))
        del xtr, xte
    net, train_ds = nets[0], train_dss[0]
    cfg = FederationConfig(protocol="synchronous", batch_size=args.batch,
                           local_epochs=args.local_epochs, evaluate_test=not args.no_eval,
                           evaluate_community=not args.no_eval,
                           # the community evaluation overlaps the next round's
                           # training (asynchronous, as the reference's); the last
                           # round's is waited for inside the timed region
                           defer_community_eval=not args.sync_community_eval,
                           secure_aggregation=args.secure_aggregation)
    engine = None
    if comm.rank == 0:  # the native controller keeps the round bookkeeping
        from metisfl_amd.parallel.engine_bridge import CollectiveController
        engine = CollectiveController(cfg, [share(args.train_size, i) for i in range(nl)])
    fed = CollectiveFederation(comm, nets, train_dss, cfg, test_ds=test_dss, engine=engine)

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)

    ckpt_dir = None
    if args.checkpoint_every > 0:
        import tempfile
        ckpt_dir = args.checkpoint_dir or tempfile.mkdtemp(prefix="metisfl_bench_ckpt_")

    def maybe_checkpoint():
        r = fed.history[-1]
        if ckpt_dir and r.global_iteration % args.checkpoint_every == 0:
            r.checkpoint_ms = fed.save_checkpoint(ckpt_dir, block=False)

    for _ in range(args.warmup):
        fed.run_round()
        maybe_checkpoint()
        if comm.rank == 0:
            r = fed.history[-1]
            print(f"[bench] warmup round {r.global_iteration}: {r.round_ms:.1f} ms "
                  f"(train {r.train_ms:.1f}, agg {r.aggregation_ms:.2f})", file=sys.stderr, flush=True)
    fed.finish_evaluations()  # the timed rounds start with no evaluation in flight
    comm.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        fed.run_round()
        maybe_checkpoint()
        if comm.rank == 0:
            r = fed.history[-1]
            print(f"[bench] round {r.global_iteration}: {r.round_ms:.1f} ms "
                  f"(train {r.train_ms:.1f}, agg {r.aggregation_ms:.2f}) loss "
                  f"{r.learner_meta[:, 4].mean():.3f}", file=sys.stderr, flush=True)
    fed.finish_evaluations()  # the last round's community evaluation, inside the timed region
    comm.barrier()
    sync()
    elapsed = time.perf_counter() - t0
    fed.flush_checkpoints()  # background writes finish outside the timed region
    elapsed = comm.all_max(elapsed)
    timed = fed.history[-args.steps:] if args.steps else []
    round_ms = elapsed * 1e3 / max(1, args.steps)
    rounds_per_s = args.steps / elapsed if elapsed > 0 else 0.0
    updates = fed.num_local_updates[0]
    agg_ms = sum(r.aggregation_ms for r in timed) / max(1, len(timed))
    model_bytes = net.state.model32.numel() * 4
    if nl == 1:
        aggregation = "none (single learner: the round ends with the local model)"
    elif args.secure_aggregation:
        aggregation = ("PWA(NUM_TRAINING_EXAMPLES) over RNS-CKKS (N=8192, 52-bit scale): "
                       "device encrypt, int64 RCCL all-reduce of ciphertexts, device decrypt")
    elif n == 1:
        aggregation = f"FedAvg(NUM_TRAINING_EXAMPLES) of {nl} co-located learners: one weighted-sum kernel"
    elif L > 1:
        aggregation = (f"FedAvg(NUM_TRAINING_EXAMPLES): weighted-sum kernel over the {L} learners of each GPU "
                       "+ one RCCL all-reduce")
    else:
        aggregation = "FedAvg(NUM_TRAINING_EXAMPLES): scale kernel + one RCCL all-reduce"
    out = {
        "metric": METRIC,
        "value": rounds_per_s,
        "unit": "rounds/s",
        "n_gpus": n,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round_ms,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": (rounds_per_s / BASELINE_VALUE) if BASELINE_VALUE else None,
        "dtype": args.dtype,
        "data": "synthetic (CIFAR-10 shapes, IID shards), random-init ResNet-18",
        "config": {
            "model": "resnet18-cifar",
            "dataset": "cifar10 (50k train / 10k test, synthetic)",
            "learners": nl,
            "learners_per_gpu": L,
            "global_batch": args.batch * nl,
            "per_learner_batch": args.batch,
            "seq_len": None,
            "local_epochs": args.local_epochs,
            "local_updates_per_round": updates,
            "optimizer": f"momentum_sgd(lr={args.lr}, momentum={args.momentum})",
            "aggregation": aggregation,
            "protocol": "synchronous",
            "parallelism": f"fedavg-dp{n}",
            "test_eval": not args.no_eval,
            **({"conv_products": net.conv_products} if args.dtype == "fp32" else {}),
            **({"width_mult": args.width_mult} if args.width_mult != 1.0 else {}),
        },
        "round_ms": round_ms,
        "rounds_per_s": rounds_per_s,
        "train_ms_mean": sum(r.train_ms for r in timed) / max(1, len(timed)),
        "aggregation_ms_mean": agg_ms,
        "collective": {"backend": comm.backend, "world_size": n, "model_bytes": model_bytes,
                       "allreduce_gbps": (model_bytes / (agg_ms * 1e-3) / 1e9) if n > 1 and agg_ms > 0 else None},
        "he_ms_mean": ({k: sum(r.he_stats[k] for r in timed) / max(1, len(timed))
                        for k in ("encrypt_ms", "allreduce_ms", "decrypt_ms")}
                       if args.secure_aggregation and timed else None),
        "samples_per_s": (args.train_size * args.local_epochs) / (round_ms / 1e3) if round_ms else 0.0,
    }
    out["community_eval_ms_mean"] = sum(r.community_eval_ms for r in timed) / max(1, len(timed))
    if fed.group is not None and fed.group.last_eval_ms:
        out["last_round_device_ms"] = {"train_max": float(timed[-1].train_ms),
                                       "test_eval_per_learner": [round(x, 2) for x in fed.group.last_eval_ms],
                                       "first_start_to_last_eval_end": fed.group.last_span_ms,
                                       "host_phases": fed.group.last_host_ms,
                                       "train_per_learner": fed.group.last_ms}
    out["phase_ms_mean"] = ({k: sum(r.phase_ms[k] for r in timed) / len(timed) for k in timed[0].phase_ms}
                            if timed and timed[0].phase_ms else None)
    out["community_eval"] = ("deferred: on a frozen copy of each community model, overlapping the next round's "
                             "training; the last round's completes inside the timed region"
                             if cfg.defer_community_eval and fed._ce else "synchronous, at the end of its round")
    ev = [r.community_eval for r in timed if r.community_eval]
    out["community_accuracy_last"] = (float(np.mean([e["accuracy"] for e in ev[-1] if e["num_examples"]]))
                                      if ev else None)
    out["lineage_snapshot_ms_mean"] = sum(r.snapshot_ms for r in timed) / max(1, len(timed))
    if ckpt_dir:
        ck = [r.checkpoint_ms for r in timed if r.global_iteration % args.checkpoint_every == 0]
        out["checkpoint"] = {"every": args.checkpoint_every, "count": len(ck),
                             "critical_path_ms_mean": sum(ck) / max(1, len(ck)),
                             "background_write_ms_last": fed._ckpt.last_write_ms if fed._ckpt else None,
                             "wait_for_previous_ms_last": fed._ckpt.last_wait_ms if fed._ckpt else None,
                             "d2d_issue_ms_last": fed._ckpt.last_d2d_issue_ms if fed._ckpt else None,
                             "prep_ms_last": getattr(fed, "last_checkpoint_prep_ms", None),
                             "dir": ckpt_dir}
    out["aggregation_weights"] = [float(w) for w in timed[-1].weights] if timed and timed[-1].weights is not None else None
    out["community_model"] = _community_digests(comm, net)
    if args.dtype == "fp32" and net.conv_products == "bf16x3" and args.exact_updates > 0:
        out["conv_products_exact"] = _exact_pass(args, comm, train_dss, opt, sync, out, updates)
    if comm.rank == 0:
        line = json.dumps(out)
        print(line, flush=True)
        if args.json_out:
            with open(args.json_out, "w") as f:
                f.write(line + "\n")
    comm.close()
    return 0


def _community_digests(comm, net) -> dict:
    """SHA-256 of every rank's resident community model (after the last
    all-reduce the replicas must be bitwise identical)."""
    import hashlib

    import torch
    h = hashlib.sha256(net.state.model32.detach().cpu().numpy().tobytes()).digest()
    words = [int.from_bytes(h[4 * i:4 * i + 4], "little") for i in range(4)]  # 128 bits, exact in fp64
    rows = comm.all_gather_rows(torch.tensor(words, dtype=torch.float64, device=comm.device)).cpu().numpy()
    digests = ["".join(f"{int(w):08x}" for w in r) for r in rows]
    return {"sha256_128": digests, "identical": len(set(digests)) == 1}


def _exact_pass(args, comm, train_dss, opt, sync, out, updates) -> dict:
    """The strict-IEEE alternative, timed after the headline rounds: fresh
    ResNet-18 learners (as many as this GPU hosts, co-located the same way)
    whose convolutions multiply on the exact fp32 MFMA
    (v_mfma_f32_32x32x2_f32) run ``--exact-updates`` local updates each
    (after 16 untimed ones that capture their step graphs); the round-time
    estimate swaps the measured bf16x3 training time for the exact one and
    keeps the round's measured evaluation / aggregation time."""
    import torch
    from metisfl_amd.models.colocated import CoLocatedLearners
    from metisfl_amd.models.resnet import ResNet18
    nets = [ResNet18(batch_size=args.batch, device=comm.device, optimizer=opt, seed=7, dtype="fp32",
                     width_mult=args.width_mult, conv_products="exact") for _ in train_dss]
    group = CoLocatedLearners(nets, train_dss)
    k = args.exact_updates
    warm = 16
    group.train([warm] * len(nets), [0] * len(nets))
    comm.barrier()
    sync()
    t0 = time.perf_counter()
    group.train([k] * len(nets), [warm] * len(nets))
    sync()
    el = comm.all_max(time.perf_counter() - t0)
    exact_upd = el * 1e3 / k  # per local update of every co-located learner
    fast_upd = out["train_ms_mean"] / max(1, updates)
    from metisfl_amd.ops.nn import set_conv_products
    set_conv_products("bf16x3")
    del nets, group
    if comm.device.type == "cuda":
        torch.cuda.empty_cache()
    return {"updates_timed": k, "learners": len(train_dss), "ms_per_update": exact_upd,
            "bf16x3_ms_per_update": fast_upd,
            "round_ms_est": out["round_ms"] + (exact_upd - fast_upd) * updates,
            "method": "measured time per local update of the co-located learners x local updates per "
                      "round + the measured non-training part of the bf16x3 round"}


if __name__ == "__main__":
    from metisfl_amd.utils.launch import exit_process
    exit_process(main())  # no interpreter finalisation behind live c10d threads (utils/launch.py)
