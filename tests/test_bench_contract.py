"""The benchmark-script contract the round driver depends on (bench.py and
benchmarks/*): one JSON line from rank 0 with the BASELINE metric and the
required keys, on 1 process and on 2 processes (torch.distributed.run, gloo
on the CPU -- the same code path the RCCL run takes on GPUs), with tiny
synthetic shards so it finishes in seconds."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REQUIRED = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
            "scaling", "vs_baseline", "dtype", "data", "config"}
TINY = ["--train-size", "64", "--test-size", "32", "--batch", "8", "--local-epochs", "1", "--steps", "1",
        "--warmup", "0", "--exact-updates", "2"]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _env():
    env = dict(os.environ)
    env["CUDA_VISIBLE_DEVICES"] = ""  # CPU path even on a GPU box
    env["HIP_VISIBLE_DEVICES"] = ""
    env["OMP_NUM_THREADS"] = "2"
    env["PYTHONPATH"] = ROOT
    return env


def _json_line(out: str) -> dict:
    lines = [l for l in out.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out[-2000:]
    return json.loads(lines[0])


def test_bench_single_process_json_contract():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *TINY], cwd=ROOT, env=_env(),
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _json_line(r.stdout)
    assert REQUIRED <= set(d)
    assert d["metric"] == json.load(open(os.path.join(ROOT, "BASELINE.json")))["metric"]
    assert d["n_gpus"] == 1 and d["steps"] == 1 and d["value"] > 0 and d["higher_is_better"] is True
    assert d["config"]["model"] == "resnet18-cifar"
    assert d["config"]["learners"] == 8 and d["config"]["learners_per_gpu"] == 8
    assert d["community_eval_ms_mean"] > 0
    ex = d["conv_products_exact"]  # the strict-IEEE alternative is timed in the same run
    assert ex["updates_timed"] == 2 and ex["ms_per_update"] > 0 and ex["round_ms_est"] > 0


def test_bench_two_ranks_one_json_line():
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", "2", *TINY]
    r = subprocess.run(cmd, cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _json_line(r.stdout)  # rank 0 only
    # the federation is always the BASELINE's 8 learners: 4 co-located per GPU here
    assert d["n_gpus"] == 2 and d["config"]["learners"] == 8 and d["config"]["learners_per_gpu"] == 4
    assert d["config"]["parallelism"] == "fedavg-dp2"
    w = d["aggregation_weights"]
    assert len(w) == 8 and abs(sum(w) - 1.0) < 1e-9
    assert d["community_model"]["identical"]


def test_async_bench_json_contract():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "benchmarks", "async_bench.py"), "--train-size", "32",
                        "--batch", "8", "--tasks", "1", "--warmup", "0", "--poll-every", "2", "--learners", "1"],
                       cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _json_line(r.stdout)
    assert REQUIRED <= set(d) and d["updates"] == 1


def test_async_bench_colocated_learners():
    """BASELINE config 3 on one GPU: 4 co-located asynchronous learners, FedRec
    on the device after every task; later finishers see staleness > 0 and the
    community model equals the host recomputation."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "benchmarks", "async_bench.py"), "--train-size", "64",
                        "--batch", "4", "--tasks", "2", "--warmup", "1", "--learners", "4", "--width-mult", "0.125"],
                       cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _json_line(r.stdout)
    assert REQUIRED <= set(d) and d["updates"] == 8 and d["updates_per_learner"] == [2, 2, 2, 2]
    assert d["config"]["learners_per_gpu"] == 4 and d["staleness_max"] > 0
    assert d["community_model_matches_host"] is True


def test_async_bench_colocated_learners_on_two_ranks():
    """BASELINE config 3 at N = 2: 8 asynchronous learners, 4 co-located per
    rank -- every learner a FedRec participant (rank 0's on the device, rank
    1's over point-to-point transfers)."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "benchmarks", "async_bench.py"), "--gpus", "2",
                        "--learners", "8", "--train-size", "128", "--batch", "4", "--tasks", "2", "--warmup", "0",
                        "--width-mult", "0.125", "--delays-ms", "0,30"], cwd=ROOT, env=_env(), capture_output=True,
                       text=True, timeout=900)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _json_line(r.stdout)
    assert d["n_gpus"] == 2 and d["config"]["learners"] == 8 and d["config"]["learners_per_gpu"] == 4
    assert d["updates"] == 16 and d["updates_per_learner"] == [2] * 8
    assert d["staleness_max"] > 0
    assert d["community_model_matches_host"] is True


def test_async_bench_eight_ranks_uneven_delays():
    """8 asynchronous learners (gloo) with uneven per-task delays: the
    threaded aggregator serves every submission under contention, staleness
    shows up, and the community model equals the host recomputation."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "benchmarks", "async_bench.py"), "--gpus", "8",
                        "--train-size", "256", "--batch", "8", "--tasks", "3", "--warmup", "0",
                        "--width-mult", "0.125", "--delays-ms", "0,40,5,80,0,120,10,60"], cwd=ROOT, env=_env(),
                       capture_output=True, text=True, timeout=1200)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _json_line(r.stdout)
    assert d["n_gpus"] == 8 and d["updates"] == 24
    assert d["updates_per_learner"] == [3] * 8
    assert d["staleness_max"] > 0
    assert d["community_model_matches_host"] is True


def test_bert_bench_spawn_world_mismatch():
    env = _env()
    env.update({"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    r = subprocess.run([sys.executable, os.path.join(ROOT, "benchmarks", "bert_bench.py"), "--gpus", "2"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 2 and "WORLD_SIZE" in r.stderr


def test_bench_spawns_its_own_ranks():
    """``bench.py --gpus 2`` with no launcher runs 2 learners by itself."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", *TINY,
                        "--width-mult", "0.125"], cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _json_line(r.stdout)
    assert d["n_gpus"] == 2 and d["config"]["learners"] == 8
    assert d["collective"]["world_size"] == 2 and d["collective"]["backend"] == "gloo"
    assert d["dtype"] == "fp32"


def test_bench_eight_ranks_gloo():
    """The driver's 8-GPU scaling run, rehearsed on 8 gloo ranks: one JSON
    line, world size 8, the FedAvg weights sum to 1, the community model is
    bitwise identical on every rank and the all-reduce bandwidth is reported."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8", *TINY,
                        "--width-mult", "0.125", "--train-size", "128", "--test-size", "64"], cwd=ROOT, env=_env(),
                       capture_output=True, text=True, timeout=1200)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _json_line(r.stdout)
    assert d["n_gpus"] == 8 and d["collective"]["world_size"] == 8 and d["config"]["parallelism"] == "fedavg-dp8"
    w = d["aggregation_weights"]
    assert len(w) == 8 and abs(sum(w) - 1.0) < 1e-9
    assert d["community_model"]["identical"] and len(d["community_model"]["sha256_128"]) == 8
    assert d["collective"]["allreduce_gbps"] and d["collective"]["allreduce_gbps"] > 0


def test_bench_world_size_mismatch_fails():
    env = _env()
    env.update({"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", *TINY], cwd=ROOT,
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
