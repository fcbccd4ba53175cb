"""Round time with and without per-round background checkpoints, 8 ranks on
the gloo backend (CPU), full-width ResNet-18 (11.2M parameters: every rank
writes its learner's momentum buffer, rank 0 the 45 MB community model too).

The driver's collective learners checkpoint with ``save_checkpoint(block=
False)`` (learner/collective.py): a snapshot on the caller's path, the
serialization and file writes on a background thread with the GIL released
(parallel/checkpoint.py).  This measures what that costs a round.

python scripts/ckpt_overhead_gloo.py [--world 8] [--rounds 4] [--updates 6]
"""
import argparse
import json
import os
import socket
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, a, out):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(1)
    from metisfl_amd.models.resnet import ResNet18
    from metisfl_amd.ops.optim import OptimizerSpec
    from metisfl_amd.parallel.comm import Comm
    from metisfl_amd.parallel.federation import CollectiveFederation, FederationConfig
    comm = Comm(backend="gloo")
    net = ResNet18(batch_size=a.batch, device="cpu", seed=rank + 1,
                   optimizer=OptimizerSpec("momentum_sgd", learning_rate=0.01, momentum=0.9))
    rng = np.random.default_rng(rank)
    n = a.batch * a.updates
    ds = net.make_dataset(rng.standard_normal((n, 32, 32, 3)).astype(np.float32), rng.integers(0, 10, n), seed=rank)
    cfg = FederationConfig(batch_size=a.batch, local_epochs=1, evaluate_test=False, evaluate_community=False)
    fed = CollectiveFederation(comm, net, ds, cfg)
    res = {}
    for mode in ("none", "every_round", "none", "every_round"):
        ck = os.path.join(a.dir, f"ckpt_{mode}")
        times, held = [], []
        fed.run_round()  # warm-up
        for _ in range(a.rounds):
            comm.barrier()
            t0 = time.perf_counter()
            fed.run_round()
            h = fed.save_checkpoint(ck, block=False) if mode == "every_round" else 0.0
            comm.barrier()
            times.append((time.perf_counter() - t0) * 1e3)
            held.append(h)
        fed.flush_checkpoints()
        comm.barrier()
        res.setdefault(mode, []).append({"round_ms": times, "held_ms": held,
                                         "write_ms_last": getattr(fed._ckpt, "last_write_ms", None)
                                         if fed._ckpt is not None else None})
    if rank == 0:
        with open(out, "w") as f:
            json.dump(res, f)
    comm.close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--updates", type=int, default=6, help="local updates per round")
    ap.add_argument("--batch", type=int, default=8)
    a = ap.parse_args()
    with tempfile.TemporaryDirectory() as d:
        a.dir = d
        out = os.path.join(d, "res.json")
        mp.spawn(_worker, args=(a.world, _free_port(), a, out), nprocs=a.world, join=True)
        res = json.load(open(out))
    summary = {}
    for mode, runs in res.items():
        rt = [t for r in runs for t in r["round_ms"]]
        summary[mode] = {"round_ms_mean": float(np.mean(rt)), "round_ms_median": float(np.median(rt)),
                         "held_ms_mean": float(np.mean([h for r in runs for h in r["held_ms"]])),
                         "write_ms_last": runs[-1]["write_ms_last"]}
    base, ck = summary["none"]["round_ms_median"], summary["every_round"]["round_ms_median"]
    print(json.dumps({"world": a.world, "model": "resnet18 (11.2M params)", "updates_per_round": a.updates,
                      "batch": a.batch, "rounds_per_mode": 2 * a.rounds, "summary": summary,
                      "overhead_pct_median": 100.0 * (ck - base) / base, "raw": res}, indent=1))


if __name__ == "__main__":
    main()
