#!/usr/bin/env python3
"""Controller orchestration at scale: N echo learners against the gRPC
controller (reference: examples/keras/scalability_testing.py:21-115 driven
with the no-train/no-eval learner of test/learner_notrain_noeval.py:16-198;
the reference's only timing datum is "10-20 s to dispatch ~100 MB models to
all learners", controller.cc:594-604).

The controller (servicer + native engine, FedAvg, in-memory store) runs in
this process; the learners run in ``--workers`` worker processes, each
hosting its share of echo learners with their own gRPC servers.  An echo
learner records when its RunTask arrived and sends the model straight back,
so a round is pure orchestration: dispatch N run tasks, receive N model
uploads, store + aggregate, dispatch N evaluations.

Per round (rounds 2.., the first one includes joins):
  * dispatch_ms       -- controller round start -> the LAST learner received
                         its run task (community model fan-out to all learners)
  * collect_ms        -- round start -> the controller has inserted the last model
  * aggregation_ms    -- the engine's model_aggregation_total_duration_ms
  * round_ms          -- start of round r -> start of round r+1

  python benchmarks/scalability.py --learners 16,64,256 --model-mb 6.4
  python benchmarks/scalability.py --learners 16 --model-mb 100
Prints one JSON line per (learners, model size).
"""
from __future__ import annotations

import argparse
import json
import multiprocessing as mp
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def _ts(t) -> float:
    return t.seconds + t.nanos * 1e-9


def _worker(port: int, first: int, count: int, q, stop, ready, tmpdir: str) -> None:
    os.environ.setdefault("HIP_VISIBLE_DEVICES", "")  # learners here never touch a GPU
    from metisfl_amd.learner.fake import EchoModelOps
    from metisfl_amd.learner.learner import Learner
    from metisfl_amd.learner.learner_servicer import LearnerServicer
    from metisfl_amd.models.model_dataset import ModelDatasetClassification
    from metisfl_amd.utils.proto_messages_factory import MetisProtoMessages as M

    class TimedEcho(EchoModelOps):
        def __init__(self, idx):
            super().__init__(0.0)
            self.idx = idx

        def train_model(self, train_dataset, learning_task_pb, *a, **kw):
            q.put((self.idx, int(learning_task_pb.global_iteration), time.time()))
            return super().train_model(train_dataset, learning_task_pb, *a, **kw)

    ctrl = M.construct_server_entity_pb("127.0.0.1", port)
    x = np.zeros((4, 2), np.float32)
    y = np.zeros(4, np.int64)
    servers = []
    for i in range(first, first + count):
        ds = ModelDatasetClassification(x, y)
        ln = Learner(M.construct_server_entity_pb("127.0.0.1", 0), ctrl, TimedEcho(i), ds,
                     learner_credentials_fp=os.path.join(tmpdir, f"cred{i}"))
        srv = LearnerServicer(ln, servicer_workers=2)
        srv.init_servicer()
        servers.append(srv)
    ready.put(count)
    stop.wait()
    for s in servers:
        s.stop()


def run_case(n: int, model_mb: float, rounds: int, workers: int, tmpdir: str) -> dict:
    from metisfl_amd import _engine as E
    from metisfl_amd.controller.servicer import ControllerServicer
    from metisfl_amd.utils.grpc_controller_client import GRPCControllerClient
    from metisfl_amd.utils.proto_messages_factory import MetisProtoMessages as M
    from metisfl_amd.utils.proto_messages_factory import ModelProtoMessages as MM
    from metisfl_amd.utils.tensor_codec import model_from_arrays

    opt = MM.construct_optimizer_config_pb(MM.construct_vanilla_sgd_optimizer_pb(0.01))
    params = M.construct_controller_params_pb(
        M.construct_server_entity_pb("127.0.0.1", 0),
        M.construct_global_model_specs(M.construct_aggregation_rule_pb("FedAvg", "NumTrainingExamples", 0), 1.0),
        M.construct_communication_specs_pb("SYNCHRONOUS", None, None),
        M.construct_model_store_config_pb("InMemory", "LineageLengthEviction", 1),
        M.construct_controller_modelhyperparams_pb(4, 1, opt, 0.0))
    srv = ControllerServicer(params, dispatch_workers=min(64, max(16, n)))
    port = srv.start()
    client = GRPCControllerClient(M.construct_server_entity_pb("127.0.0.1", port))
    n_vals = int(model_mb * 1e6 / 4)
    per = 1 << 20
    arrays = [np.full(min(per, n_vals - o), 0.5, np.float32) for o in range(0, n_vals, per)]
    model = model_from_arrays([f"v{i}" for i in range(len(arrays))], arrays)
    client.replace_community_model(1, model)

    ctx = mp.get_context("spawn")
    q, stop, ready = ctx.Queue(), ctx.Event(), ctx.Queue()
    procs, first = [], 0
    for w in range(workers):
        cnt = n // workers + (w < n % workers)
        if cnt == 0:
            continue
        p = ctx.Process(target=_worker, args=(port, first, cnt, q, stop, ready, tmpdir), daemon=True)
        p.start()
        procs.append(p)
        first += cnt
    t_join0 = time.time()
    for _ in procs:
        ready.get(timeout=600)
    join_s = time.time() - t_join0
    # rounds that ran while learners were still joining had fewer members:
    # measure from the first round started after the last join
    base = srv.engine.global_iteration()
    target = base + rounds + 2  # the last round only closes its predecessor
    deadline = time.time() + 60 + rounds * (10 + n * model_mb * 0.02)
    while srv.engine.global_iteration() < target and time.time() < deadline:
        time.sleep(0.05)
    recv: dict[tuple[int, int], float] = {}
    time.sleep(1.0)  # let the workers' queue feeders flush
    while not q.empty():
        i, gi, t = q.get()
        recv[(i, gi)] = t
    md = client.get_runtime_metadata(0).metadata
    out_rounds = []
    by_gi = {m.global_iteration: m for m in md}
    for gi in range(base + 1, target):
        m, nxt = by_gi.get(gi), by_gi.get(gi + 1)
        if m is None or nxt is None or len(m.completed_by_learner_id) < n:
            continue
        start = _ts(m.started_at)
        arr = [recv[(i, gi)] for i in range(n) if (i, gi) in recv]
        ins = [_ts(t) for t in m.train_task_received_at.values()]
        out_rounds.append({
            "global_iteration": gi,
            "dispatch_ms": (max(arr) - start) * 1e3 if len(arr) == n else None,
            "collect_ms": (max(ins) - start) * 1e3 + max(m.model_insertion_duration_ms.values()),
            "aggregation_ms": m.model_aggregation_total_duration_ms,
            "round_ms": (_ts(nxt.started_at) - start) * 1e3,
        })
    if not out_rounds:
        print("[scalability] no complete round: " + "; ".join(
            f"gi {m.global_iteration}: {len(m.completed_by_learner_id)} done" for m in md), file=sys.stderr)
    stop.set()
    for p in procs:
        p.join(timeout=30)
        if p.is_alive():
            p.kill()
    client.shutdown()
    srv.stop()

    def med(k):
        v = [r[k] for r in out_rounds if r[k] is not None]
        return float(np.median(v)) if v else None
    return {"learners": n, "model_mb": model_mb, "model_vars": len(arrays), "workers": len(procs),
            "join_s": join_s, "rounds_measured": len(out_rounds), "dispatch_ms": med("dispatch_ms"),
            "collect_ms": med("collect_ms"), "aggregation_ms": med("aggregation_ms"),
            "round_ms": med("round_ms"), "device_aggregation": E.device_aggregation_stats(),
            "per_round": out_rounds}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--learners", default="16,64,256")
    ap.add_argument("--model-mb", default="6.4")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--workers", type=int, default=min(8, os.cpu_count() or 4))
    ap.add_argument("--json-out", default="")
    a = ap.parse_args()
    import tempfile
    results = []
    for mb in [float(x) for x in a.model_mb.split(",")]:
        for n in [int(x) for x in a.learners.split(",")]:
            with tempfile.TemporaryDirectory() as td:
                r = run_case(n, mb, a.rounds, min(a.workers, n), td)
            print(json.dumps({k: v for k, v in r.items() if k != "per_round"}), flush=True)
            results.append(r)
    if a.json_out:
        with open(a.json_out, "w") as f:
            json.dump(results, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
