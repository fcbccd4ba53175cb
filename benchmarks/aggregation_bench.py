#!/usr/bin/env python3
"""Aggregation scenario benchmark (reference: the stale, non-building
scenarios/sync_model_aggregation_performance_main.cc:14-87 -- N learners x
T tensors x V values, FedStride, in-memory store).

Measures, for N learner models of T tensors x V fp32 values:
  * host   -- the native engine's FedAvg / FedStride over serialized Model
              protos (the reference controller's CPU path, OpenMP),
  * engine_device -- the same engine call with the controller's device
              backend (engine/device_agg.*): models staged into HBM on arrival
              (as Controller::learner_completed_task does), one multi-tensor
              launch, result copied back into the engine's model; plus the
              cold variant that uploads inside the call,
  * device -- the HIP multi-tensor weighted sum K1 over device-resident flat
              models (one launch for all tensors),
  * rccl   -- scale + all-reduce of the flat model when launched with
              torchrun over several GPUs (the collective path's aggregation).
Prints one JSON line.

  python benchmarks/aggregation_bench.py --learners 8 --tensors 100 --values 100000
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def _timeit(fn, reps):
    fn()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    return (time.perf_counter() - t0) * 1e3 / reps


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--learners", type=int, default=8)
    ap.add_argument("--tensors", type=int, default=100)
    ap.add_argument("--values", type=int, default=100000)
    ap.add_argument("--stride", type=int, default=2)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--no-host", action="store_true")
    a = ap.parse_args()

    import torch

    from metisfl_amd import _engine as E
    from metisfl_amd.ops import aggregate as agg
    from metisfl_amd.utils.tensor_codec import model_from_arrays

    N, T, V = a.learners, a.tensors, a.values
    rng = np.random.default_rng(0)
    weights = list(rng.random(N) + 0.5)
    weights = [w / sum(weights) for w in weights]
    out = {"learners": N, "tensors": T, "values_per_tensor": V, "model_mb": T * V * 4 / 2 ** 20}

    names = [f"t{i}" for i in range(T)]
    models = [model_from_arrays(names, [rng.standard_normal(V).astype(np.float32) for _ in range(T)])
              .SerializeToString() for _ in range(N)]
    dev_ok = E.device_aggregation_available()
    E.set_device_aggregation(False)
    # the engine's aggregation as the controller runs it, over parsed models:
    # *_ms include serializing the result to Python bytes, *_engine_ms is the
    # engine call alone (what the controller's aggregation metric records)
    staged_host = E.StagedModels([f"L{i}" for i in range(N)], models)
    if not a.no_host:
        out["host_fedavg_ms"] = _timeit(lambda: staged_host.aggregate("fed_avg", weights), a.reps)
        out["host_fedavg_engine_ms"] = staged_host.last_aggregate_ms
        out["host_fedstride_ms"] = _timeit(lambda: staged_host.aggregate("fed_stride", weights, a.stride),
                                           a.reps)
        out["host_fedstride_engine_ms"] = staged_host.last_aggregate_ms
    del staged_host
    if dev_ok:
        E.set_device_aggregation(True, 0)
        host_bytes = E.aggregate_models("fed_avg", models, weights) if a.no_host else None
        # controller path with residency: models staged on arrival, aggregated from HBM
        staged = E.StagedModels([f"L{i}" for i in range(N)], models)
        out["engine_device_fedavg_ms"] = _timeit(lambda: staged.aggregate("fed_avg", weights), a.reps)
        out["engine_device_fedavg_engine_ms"] = staged.last_aggregate_ms
        st = E.device_aggregation_stats()
        out["engine_device_fedavg_kernel_ms"] = st["last_kernel_ms"]
        out["engine_device_fedavg_download_ms"] = st["last_download_ms"]
        out["engine_device_stage_ms_per_model"] = st["last_upload_ms"]
        out["engine_device_fedstride_ms"] = _timeit(lambda: staged.aggregate("fed_stride", weights, a.stride),
                                                    a.reps)
        out["engine_device_fedstride_engine_ms"] = staged.last_aggregate_ms
        E.set_device_aggregation(False)
        ref = staged.aggregate("fed_avg", weights)
        E.set_device_aggregation(True, 0)
        out["engine_device_byte_identical"] = staged.aggregate("fed_avg", weights) == ref
        # cold: the inputs are uploaded inside the call (no residency)
        out["engine_device_cold_fedavg_ms"] = _timeit(lambda: E.aggregate_models("fed_avg", models, weights),
                                                      max(1, a.reps // 2))
        out["device"] = E.device_aggregation_stats().get("device_name")
        del staged, host_bytes
    del models

    if torch.cuda.is_available():
        dev = torch.device("cuda")
        flats = [torch.randn(T * V, device=dev) for _ in range(N)]
        res = torch.empty(T * V, device=dev)

        def k1():
            agg.weighted_sum(res, flats, weights)
            torch.cuda.synchronize()
        ms = _timeit(k1, a.reps * 4)
        out["device_k1_ms"] = ms
        out["device_k1_gbps"] = (N + 1) * T * V * 4 / (ms * 1e6)
        ref = sum(w * f.double() for w, f in zip(weights, flats))
        out["device_k1_max_rel_err"] = float(((res.double() - ref).abs().max() / ref.abs().max()).item())

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1 and torch.cuda.is_available():
        from metisfl_amd.ops import optim as opt_ops
        from metisfl_amd.parallel.comm import Comm
        comm = Comm()
        x = torch.randn(T * V, device=comm.device)

        def ar():
            opt_ops.scale_(x, 1.0 / world)
            comm.all_reduce_(x)
            torch.cuda.synchronize()
        ms = _timeit(ar, a.reps * 4)
        out["rccl_allreduce_ms"] = ms
        out["rccl_busbw_gbps"] = 2 * (world - 1) / world * T * V * 4 / (ms * 1e6)
        out["ranks"] = world
        if comm.rank != 0:
            comm.close()
            return 0
        comm.close()
    print(json.dumps(out))
    return 0


if __name__ == "__main__":
    sys.exit(main())
