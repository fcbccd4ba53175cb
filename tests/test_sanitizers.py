"""Race detection / memory-error presets for the native controller engine
(SURVEY §5.2): the engine sources plus a multi-threaded stress driver
(csrc/tests/engine_stress.cc) are built with ThreadSanitizer and with
AddressSanitizer + UndefinedBehaviorSanitizer (host code only -- GPU ASan is
not available on this pool) and must run clean: concurrent joins / task
completions / leaves / evictions against lineage readers, on the synchronous
and asynchronous schedulers.

The TSan build omits -fopenmp (libgomp's barriers are invisible to TSan and
report false positives); the aggregation loops then run serially, which
does not change what the engine's own locking has to protect."""
import glob
import os
import subprocess

import numpy as np
import pytest

from metisfl_amd.utils.proto_messages_factory import MetisProtoMessages as M
from metisfl_amd.utils.proto_messages_factory import ModelProtoMessages as MM
from metisfl_amd.utils.tensor_codec import model_from_arrays

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "metisfl_amd", "csrc")
OUT = os.path.join(ROOT, "build", "sanitize")
THREADS, ITERS = 6, 60


def _sources():
    return sorted(glob.glob(os.path.join(CSRC, "common", "*.cc")) + glob.glob(os.path.join(CSRC, "engine", "*.cc"))
                  + glob.glob(os.path.join(CSRC, "he", "*.cc")) + [os.path.join(CSRC, "tests", "engine_stress.cc")])


def _build(kind):
    exe = os.path.join(OUT, kind, "engine_stress")
    srcs = _sources()
    hdrs = glob.glob(os.path.join(CSRC, "*", "*.h"))
    if os.path.exists(exe) and os.path.getmtime(exe) > max(os.path.getmtime(p) for p in srcs + hdrs):
        return exe
    os.makedirs(os.path.dirname(exe), exist_ok=True)
    flags = {"tsan": ["-fsanitize=thread"],
             "asan": ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined", "-fopenmp"]}[kind]
    # the controller's device-aggregation kernels come from the in-tree native
    # build (hipcc object); with no GPU visible the engine stays on its host rules
    from metisfl_amd.csrc import build as native_build
    native_build.build(["_engine"])
    kobj = glob.glob(os.path.join(ROOT, "build", "native", "engine", "*.hip.o"))
    rocm = os.environ.get("ROCM_PATH", "/opt/rocm")
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-pthread", f"-I{CSRC}",
           "-D__HIP_PLATFORM_AMD__", f"-I{rocm}/include", *flags, *srcs, *kobj, "-o", exe,
           f"-L{rocm}/lib", f"-Wl,-rpath,{rocm}/lib", "-lamdhip64"]
    subprocess.run(cmd, check=True, capture_output=True, text=True, timeout=900)
    return exe


def _params(protocol):
    opt = MM.construct_optimizer_config_pb(MM.construct_vanilla_sgd_optimizer_pb(0.01))
    p = M.construct_controller_params_pb(
        M.construct_server_entity_pb("localhost", 50051),
        M.construct_global_model_specs(M.construct_aggregation_rule_pb(
            "FedAvg" if protocol == "SYNCHRONOUS" else "FedRec", "NumTrainingExamples", 0, None), 1.0),
        M.construct_communication_specs_pb(protocol, 2, False),
        M.construct_model_store_config_pb("InMemory", "LineageLengthEviction", 2, "127.0.0.1", None),
        M.construct_controller_modelhyperparams_pb(10, 1, opt, 0.0))
    return p.SerializeToString()


def _inputs(d):
    def w(name, b):
        with open(os.path.join(d, name), "wb") as f:
            f.write(b)
    w("params_sync.bin", _params("SYNCHRONOUS"))
    w("params_async.bin", _params("ASYNCHRONOUS"))
    vals = [np.arange(64, dtype=np.float32), np.ones((4, 8), np.float32)]
    w("model.bin", MM.construct_federated_model_pb(1, model_from_arrays(["a", "b"], vals), 0).SerializeToString())
    for i in range(THREADS):
        w(f"entity_{i}.bin", M.construct_server_entity_pb("stress-host", 6000 + i).SerializeToString())
        w(f"dataset_{i}.bin", M.construct_dataset_spec_pb(10 + i, 0, 0).SerializeToString())
        meta = M.construct_task_execution_metadata_pb(1, None, 1.0, 4, 10, 5.0, 1.0)
        task = M.construct_completed_learning_task_pb(
            model_from_arrays(["a", "b"], [v * (i + 1) for v in vals]), meta, "")
        w(f"completed_{i}.bin", task.SerializeToString())


@pytest.mark.parametrize("kind", ["tsan", "asan"])
def test_engine_under_sanitizer(kind, tmp_path):
    try:
        exe = _build(kind)
    except subprocess.CalledProcessError as e:  # pragma: no cover - toolchain without the runtime
        if "cannot find" in e.stderr and "libtsan" in e.stderr + "libasan":
            pytest.skip(f"{kind} runtime not installed")
        raise
    _inputs(str(tmp_path))
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1 exitcode=66 second_deadlock_stack=1",
               ASAN_OPTIONS="detect_leaks=1:halt_on_error=1", UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([exe, str(tmp_path), str(THREADS), str(ITERS)], capture_output=True, text=True,
                       timeout=600, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-6000:]
    assert "WARNING: ThreadSanitizer" not in r.stderr and "ERROR: AddressSanitizer" not in r.stderr
    assert "runtime error" not in r.stderr
    assert r.stdout.count("global_iteration=") == 2
