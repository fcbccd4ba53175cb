#!/usr/bin/env python3
"""Asynchronous-protocol benchmark (BASELINE config 3): CIFAR-10 ResNet-18,
``--learners`` asynchronous learners over ``--gpus`` GPUs (learners/GPU
co-located on their own HIP streams), FedRec with staleness-aware weights.

Every learner trains ``--tasks`` consecutive tasks of ``--local-epochs`` over
its IID shard of the fixed 50k-image training set (batch 32, MomentumSGD lr
0.005 / 0.75: the reference's CIFAR-10 config).  At each task end a learner
is folded into the community model (rank 0's learners on the device, the
other ranks' with one point-to-point RCCL send each way) with the polynomial
staleness discount and continues from the new community model -- one FedRec
core for every placement (parallel/async_federation.py).
The reference dispatches the same protocol through its controller
(AsynchronousScheduler, FedRec; scheduling/asynchronous_scheduler.h:12-18,
aggregation/federated_recency.cc:8-100) over gRPC.

Reports (rank 0, one JSON line): community-model updates per second over the
timed tasks (whole job), mean task time, mean FedRec update latency on the
aggregator, mean staleness.  Synthetic data, random init.

  python benchmarks/async_bench.py                       # 8 learners on 1 GPU
  python benchmarks/async_bench.py --gpus 2 --learners 8  # 4 per GPU (spawns its ranks)
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
    ap.add_argument("--learners", type=int, default=8,
                    help="asynchronous learners over all GPUs; a GPU's learners are co-located (own streams)")
    ap.add_argument("--tasks", type=int, default=3, help="timed tasks per learner")
    ap.add_argument("--warmup", type=int, default=1, help="untimed tasks per learner")
    ap.add_argument("--local-epochs", type=int, default=1)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--train-size", type=int, default=50000)
    ap.add_argument("--staleness", default="polynomial")
    ap.add_argument("--poll-every", type=int, default=32)
    ap.add_argument("--json-out", default="")
    ap.add_argument("--width-mult", type=float, default=1.0, help=argparse.SUPPRESS)  # CPU plumbing tests only
    ap.add_argument("--secure-aggregation", action="store_true",
                    help="CKKS: learners submit ciphertexts, PWA over the latest ones (AsyncPWA)")
    ap.add_argument("--delays-ms", default="",
                    help="comma list: per-rank sleep after each task (uneven learner speeds; contention tests)")
    args = ap.parse_args()
    from metisfl_amd.utils.launch import ensure_world
    rc = ensure_world(args.gpus, __file__)
    if rc is not None:
        return rc

    import numpy as np
    import torch

    from metisfl_amd.models.colocated import CoLocatedLearners
    from metisfl_amd.models.resnet import ResNet18
    from metisfl_amd.ops.optim import OptimizerSpec
    from metisfl_amd.parallel.async_federation import AsyncCollectiveFederation
    from metisfl_amd.parallel.comm import Comm
    from metisfl_amd.parallel.federation import FederationConfig

    comm = Comm()
    n, dev = comm.world, comm.device
    L = max(args.learners, n)
    owners = [min(n - 1, g * n // L) for g in range(L)]  # contiguous blocks of learners per rank
    gids = [g for g in range(L) if owners[g] == comm.rank]
    from metisfl_amd.models.colocated import configure_regime
    configure_regime(len(gids))  # kernel choices for this GPU's co-located learners
    nets, dss = [], []
    for g in gids:
        ng = args.train_size // L + (1 if g < args.train_size % L else 0)
        gen = torch.Generator(device=dev)
        gen.manual_seed(2000 + g)
        x = torch.randn((ng, 32, 32, 3), generator=gen, device=dev)
        y = torch.randint(0, 10, (ng,), generator=gen, device=dev)
        net = ResNet18(batch_size=args.batch, device=dev, seed=7, width_mult=args.width_mult,
                       optimizer=OptimizerSpec("momentum_sgd", 0.005, momentum=0.75))
        nets.append(net)
        dss.append(net.make_dataset(x, y, seed=g))
        del x
    # co-location settings (pair ring, streams) of a GPU hosting several learners
    group = CoLocatedLearners(nets, dss) if len(nets) > 1 else None
    cfg = FederationConfig(protocol="asynchronous", batch_size=args.batch, local_epochs=args.local_epochs,
                           evaluate_test=False, staleness=args.staleness,
                           secure_aggregation=args.secure_aggregation)
    delays = [float(v) for v in args.delays_ms.split(",") if v.strip()]
    delay = delays[comm.rank % len(delays)] / 1e3 if delays else 0.0
    fed = AsyncCollectiveFederation(comm, nets, dss, cfg, tasks_per_learner=max(1, args.warmup),
                                    poll_every=args.poll_every, broadcast_initial=n > 1, gids=gids, owners=owners,
                                    streams=group.streams if group is not None else None)
    if args.warmup:
        fed.run(debug_delay_s=delay)
    comm.barrier()
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    n0 = len(fed.updates)
    fed.tasks = args.tasks
    t0 = time.perf_counter()
    ups = fed.run(debug_delay_s=delay)[n0:]
    comm.barrier()
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    elapsed = comm.all_max(time.perf_counter() - t0)
    if comm.rank == 0:
        nup = len(ups)
        out = {
            "metric": "async FedRec community updates/s (whole job), CIFAR-10 ResNet-18",
            "value": nup / elapsed, "unit": "updates/s", "n_gpus": n, "steps": args.tasks,
            "warmup": args.warmup, "ms_per_step": elapsed * 1e3 / max(1, args.tasks),
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
            "dtype": "fp32" if nets[0].compute_dtype == torch.float32 else "bf16",
            "data": "synthetic (CIFAR-10 shapes, IID shards), random-init ResNet-18",
            "config": {"model": "resnet18-cifar", "learners": L, "learners_per_gpu": len(gids),
                       "per_learner_batch": args.batch, "local_epochs_per_task": args.local_epochs,
                       "local_updates_per_task": fed.num_local_updates, "protocol": "asynchronous",
                       "aggregation": (f"CKKS PWA over the latest ciphertexts, staleness={args.staleness}"
                                       if fed.secure else f"FedRec, staleness={args.staleness}"),
                       "parallelism": f"fedasync-{L}-learners-on-{n}-gpus"},
            "updates": nup,
            "local_updates_per_s": sum(u.completed_batches for u in ups) / elapsed,
            "fedrec_update_ms_mean": sum(u.aggregation_ms for u in ups) / max(1, nup),
            "staleness_mean": sum(u.staleness for u in ups) / max(1, nup),
            "staleness_max": max((u.staleness for u in ups), default=0),
            "updates_per_learner": [sum(1 for u in ups if u.learner == g) for g in range(L)],
            "community_model_matches_host": bool(np.allclose(fed.community_reference(),
                                                             fed.community().double().cpu().numpy(),
                                                             rtol=1e-5, atol=1e-5 if fed.secure else 1e-6)),
        }
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
