#!/usr/bin/env python3
"""Asynchronous-protocol benchmark (BASELINE config 3): CIFAR-10 ResNet-18,
one learner per GPU, FedRec with staleness-aware weights.

Every learner trains ``--tasks`` consecutive tasks of ``--local-epochs`` over
its IID shard of the fixed 50k-image training set (batch 32, MomentumSGD lr
0.005 / 0.75: the reference's CIFAR-10 config).  At each task end a learner
submits its model to the aggregator (rank 0) with one point-to-point RCCL
send, rank 0 applies the FedRec update with the polynomial staleness
discount and answers with the new community model (async_federation.py).
The reference dispatches the same protocol through its controller
(AsynchronousScheduler, FedRec; scheduling/asynchronous_scheduler.h:12-18,
aggregation/federated_recency.cc:8-100) over gRPC.

Reports (rank 0, one JSON line): community-model updates per second over the
timed tasks (whole job), mean task time, mean FedRec update latency on the
aggregator, mean staleness.  Synthetic data, random init.

  python benchmarks/async_bench.py
  python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \\
      --master-port 29512 benchmarks/async_bench.py --gpus 8
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
                    help="asynchronous learners; on one GPU they are co-located (parallel/async_colocated.py), on "
                         "N GPUs there is one per GPU")
    ap.add_argument("--tasks", type=int, default=3, help="timed tasks per learner")
    ap.add_argument("--warmup", type=int, default=1, help="untimed tasks per learner")
    ap.add_argument("--local-epochs", type=int, default=1)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--train-size", type=int, default=50000)
    ap.add_argument("--staleness", default="polynomial")
    ap.add_argument("--poll-every", type=int, default=32)
    ap.add_argument("--json-out", default="")
    ap.add_argument("--width-mult", type=float, default=1.0, help=argparse.SUPPRESS)  # CPU plumbing tests only
    ap.add_argument("--delays-ms", default="",
                    help="comma list: per-rank sleep after each task (uneven learner speeds; contention tests)")
    args = ap.parse_args()
    from metisfl_amd.utils.launch import ensure_world
    rc = ensure_world(args.gpus, __file__)
    if rc is not None:
        return rc

    import numpy as np
    import torch

    from metisfl_amd.models.resnet import ResNet18
    from metisfl_amd.ops.optim import OptimizerSpec
    from metisfl_amd.parallel.async_federation import AsyncCollectiveFederation
    from metisfl_amd.parallel.comm import Comm
    from metisfl_amd.parallel.federation import FederationConfig

    comm = Comm()
    n = comm.world
    dev = comm.device
    if n == 1 and args.learners > 1:
        return _colocated(args, comm)
    n_train = args.train_size // n + (1 if comm.rank < args.train_size % n else 0)
    g = torch.Generator(device=dev)
    g.manual_seed(2000 + comm.rank)
    x = torch.randn((n_train, 32, 32, 3), generator=g, device=dev)
    y = torch.randint(0, 10, (n_train,), generator=g, device=dev)
    net = ResNet18(batch_size=args.batch, device=dev, seed=7, width_mult=args.width_mult,
                   optimizer=OptimizerSpec("momentum_sgd", 0.005, momentum=0.75))
    ds = net.make_dataset(x, y, seed=comm.rank)
    del x
    cfg = FederationConfig(protocol="asynchronous", batch_size=args.batch, local_epochs=args.local_epochs,
                           evaluate_test=False, staleness=args.staleness)

    delays = [float(v) for v in args.delays_ms.split(",") if v.strip()]
    delay = delays[comm.rank % len(delays)] / 1e3 if delays else 0.0

    fed_last = []

    def run(tasks):
        fed = AsyncCollectiveFederation(comm, net, ds, cfg, tasks_per_learner=tasks,
                                        poll_every=args.poll_every, broadcast_initial=False)
        fed_last[:] = [fed]
        return fed.run(debug_delay_s=delay)

    if args.warmup:
        run(args.warmup)
    comm.barrier()
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    ups = run(args.tasks)
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
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "fp32" if net.compute_dtype == torch.float32 else "bf16",
            "data": "synthetic (CIFAR-10 shapes, IID shards), random-init ResNet-18",
            "config": {"model": "resnet18-cifar", "learners": n, "per_learner_batch": args.batch,
                       "local_epochs_per_task": args.local_epochs, "protocol": "asynchronous",
                       "aggregation": f"FedRec, staleness={args.staleness}", "parallelism": f"fedasync-{n}"},
            "updates": nup,
            "fedrec_update_ms_mean": sum(u.aggregation_ms for u in ups) / max(1, nup),
            "staleness_mean": sum(u.staleness for u in ups) / max(1, nup),
            "staleness_max": max((u.staleness for u in ups), default=0),
            "updates_per_learner": [sum(1 for u in ups if u.learner == r) for r in range(n)],
            "community_model_matches_host": bool(np.allclose(fed_last[0].community_reference(),
                                                             fed_last[0]._community().double().cpu().numpy(),
                                                             rtol=1e-5, atol=1e-6)) if n > 1 else None,
        }
        line = json.dumps(out)
        print(line, flush=True)
        if args.json_out:
            with open(args.json_out, "w") as f:
                f.write(line + "\n")
    comm.close()
    return 0


def _colocated(args, comm) -> int:
    """BASELINE config 3 on one GPU: ``--learners`` co-located learners, each
    on its own HIP stream, FedRec on the device after every finished task."""
    import numpy as np
    import torch

    from metisfl_amd.models.colocated import CoLocatedLearners
    from metisfl_amd.models.resnet import ResNet18
    from metisfl_amd.ops.optim import OptimizerSpec
    from metisfl_amd.parallel.async_colocated import CoLocatedAsyncFederation
    from metisfl_amd.parallel.federation import FederationConfig

    dev = comm.device
    L = args.learners
    nets, dss = [], []
    for j in range(L):
        nj = args.train_size // L + (1 if j < args.train_size % L else 0)
        g = torch.Generator(device=dev)
        g.manual_seed(2000 + j)
        x = torch.randn((nj, 32, 32, 3), generator=g, device=dev)
        y = torch.randint(0, 10, (nj,), generator=g, device=dev)
        net = ResNet18(batch_size=args.batch, device=dev, seed=7, width_mult=args.width_mult,
                       optimizer=OptimizerSpec("momentum_sgd", 0.005, momentum=0.75))
        nets.append(net)
        dss.append(net.make_dataset(x, y, seed=j))
        del x
    cfg = FederationConfig(protocol="asynchronous", batch_size=args.batch, local_epochs=args.local_epochs,
                           evaluate_test=False, staleness=args.staleness)
    fed = CoLocatedAsyncFederation(CoLocatedLearners(nets, dss), cfg)
    if args.warmup:
        fed.run(args.warmup)
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    n0 = len(fed.updates)
    t0 = time.perf_counter()
    ups = fed.run(args.tasks)[n0:]
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    nup = len(ups)
    out = {
        "metric": "async FedRec community updates/s (whole job), CIFAR-10 ResNet-18",
        "value": nup / elapsed, "unit": "updates/s", "n_gpus": 1, "steps": args.tasks,
        "warmup": args.warmup, "ms_per_step": elapsed * 1e3 / max(1, args.tasks),
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
        "dtype": "fp32" if nets[0].compute_dtype == torch.float32 else "bf16",
        "data": "synthetic (CIFAR-10 shapes, IID shards), random-init ResNet-18",
        "config": {"model": "resnet18-cifar", "learners": L, "learners_per_gpu": L, "per_learner_batch": args.batch,
                   "local_epochs_per_task": args.local_epochs, "local_updates_per_task": fed.nums[0],
                   "protocol": "asynchronous", "aggregation": f"FedRec, staleness={args.staleness}",
                   "parallelism": f"fedasync-colocated-{L}"},
        "updates": nup,
        "local_updates_per_s": sum(u.completed_batches for u in ups) / elapsed,
        "fedrec_update_host_ms_mean": sum(u.aggregation_ms for u in ups) / max(1, nup),
        "staleness_mean": sum(u.staleness for u in ups) / max(1, nup),
        "staleness_max": max((u.staleness for u in ups), default=0),
        "updates_per_learner": [sum(1 for u in ups if u.learner == r) for r in range(L)],
        "train_loss_last": [u.train_loss for u in ups[-L:]],
        "community_model_matches_host": bool(np.allclose(fed.community_reference(),
                                                         fed.community().double().cpu().numpy(),
                                                         rtol=1e-5, atol=1e-6)),
    }
    line = json.dumps(out)
    print(line, flush=True)
    if args.json_out:
        with open(args.json_out, "w") as f:
            f.write(line + "\n")
    comm.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
