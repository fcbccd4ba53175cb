#!/usr/bin/env python3
"""User-model federation on the collective data plane:
a TorchModelDef -- the BrainAge 3D CNN of examples/neuroimaging.py (the
reference's examples/keras/models/brainage_cnns.py), or the Ionosphere MLP
of examples/pytorch/dummy.py -- trained by ``--learners`` learners over
``--gpus`` ranks (a rank's learners co-located on their own streams),
synchronous FedAvg every round: K1 over a rank's learners + one all-reduce
(models/torch_net.py: the module's parameters / buffers are views of one
flat buffer the fused HIP optimizer updates).

Reports (rank 0, one JSON line): ms per round, local updates per second
(whole job), and the SHA-256 of every rank's community model (after the
all-reduce the replicas must be bitwise identical).  Synthetic MRI-shaped
volumes / Ionosphere-shaped rows, random init.

  python benchmarks/torch_model_bench.py [--model brainage3d|ionosphere] [--gpus N] [--learners L]
"""
from __future__ import annotations

import argparse
import hashlib
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
    ap.add_argument("--learners", type=int, default=2)
    ap.add_argument("--model", default="brainage3d", choices=["brainage3d", "ionosphere"])
    ap.add_argument("--shape", type=int, nargs=3, default=[32, 32, 32])
    ap.add_argument("--samples", type=int, default=64, help="training volumes / rows per learner")
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--local-epochs", type=int, default=1)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    args = ap.parse_args()
    from metisfl_amd.utils.launch import ensure_world
    rc = ensure_world(args.gpus, __file__)
    if rc is not None:
        return rc

    import numpy as np
    import torch

    from examples.models.torch_models import BrainAge3DCNN, IonosphereMLP, synthetic_volumes
    from metisfl_amd.models.torch_net import TorchNet
    from metisfl_amd.ops.optim import OptimizerSpec
    from metisfl_amd.parallel.comm import Comm
    from metisfl_amd.parallel.federation import CollectiveFederation, FederationConfig

    comm = Comm()
    n, dev = comm.world, comm.device
    if args.learners % n:
        print(f"[torch_model_bench] {args.learners} learners do not split over {n} ranks", file=sys.stderr)
        return 2
    L = args.learners // n
    if args.model == "brainage3d":
        mdef, opt = BrainAge3DCNN(filters=(16, 32, 64, 128)), OptimizerSpec("vanilla_sgd", 5e-5)
    else:
        mdef, opt = IonosphereMLP(), OptimizerSpec("momentum_sgd", 0.05, momentum=0.5)
    nets, dss, tds = [], [], []
    for j in range(L):
        g = comm.rank * L + j
        net = TorchNet(mdef, args.batch, device=dev, optimizer=opt, seed=7)
        if args.model == "brainage3d":
            x, y = synthetic_volumes(args.samples, tuple(args.shape), seed=g)
            xt, yt = synthetic_volumes(8, tuple(args.shape), seed=1000 + g)
        else:
            rng = np.random.default_rng(g)
            x = rng.uniform(-1, 1, (args.samples, 34)).astype(np.float32)
            y = (x @ np.random.default_rng(7).standard_normal(34) > 0).astype(np.int64)
            xt, yt = x[:16], y[:16]
        nets.append(net)
        dss.append(net.make_dataset(x, y, seed=g))
        tds.append(net.make_dataset(xt, yt, seed=g, shuffle=False))
    cfg = FederationConfig(batch_size=args.batch, local_epochs=args.local_epochs)
    fed = CollectiveFederation(comm, nets, dss, cfg, test_ds=tds)

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)

    for _ in range(args.warmup):
        fed.run_round()
    comm.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(args.rounds):
        rec = fed.run_round()
    comm.barrier()
    sync()
    el = comm.all_max(time.perf_counter() - t0)
    h = hashlib.sha256(nets[0].state.model32.detach().cpu().numpy().tobytes()).digest()
    words = [int.from_bytes(h[4 * i:4 * i + 4], "little") for i in range(4)]
    rows = comm.all_gather_rows(torch.tensor(words, dtype=torch.float64, device=dev)).cpu().numpy()
    digests = ["".join(f"{int(w):08x}" for w in r) for r in rows]
    updates = sum(fed.num_local_updates) * args.rounds
    out = {"benchmark": "user-model federation (TorchModelDef) on the collective data plane",
           "model": args.model, "n_gpus": n, "learners": args.learners, "learners_per_gpu": L,
           "ms_per_round": el * 1e3 / max(1, args.rounds), "local_updates_per_s": updates / el if el else 0.0,
           "params": int(nets[0].state.n_params), "variables": len(nets[0].state.specs),
           "last_round_weights": [float(w) for w in rec.weights],
           "community_eval": rec.community_eval,
           "community_model": {"sha256_128": digests, "identical": len(set(digests)) == 1},
           "data": "synthetic", "config": {"batch": args.batch, "local_epochs": args.local_epochs,
                                           "shape": args.shape if args.model == "brainage3d" else [34]}}
    if comm.rank == 0:
        print(json.dumps(out), flush=True)
    comm.close()
    return 0


if __name__ == "__main__":
    from metisfl_amd.utils.launch import exit_process
    exit_process(main())  # no interpreter finalisation behind live c10d threads (utils/launch.py)
