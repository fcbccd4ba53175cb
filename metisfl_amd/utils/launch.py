"""Launcher-less multi-rank entry for the benchmark scripts.

``script.py --gpus N`` with no torch.distributed environment re-launches the
script as N ranks through ``torch.distributed.run`` (one process per GPU,
rendezvous on 127.0.0.1) BEFORE anything touches a GPU, relays their output
and returns the launcher's exit code; under a launcher it checks that
``WORLD_SIZE`` agrees with ``--gpus``.  Children are started as subprocesses,
never by exec.
"""
from __future__ import annotations

import os
import socket
import subprocess
import sys


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n: int, script: str, argv: list[str]) -> int:
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.abspath(script), *argv]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC (RCCL peer buffers)
    return subprocess.run(cmd, env=env).returncode


def ensure_world(gpus: int, script: str, argv: list[str] | None = None, tag: str = "bench") -> int | None:
    """None: this process is a rank of the right world -- run.  An int: the
    exit code to return (the spawned job's, or 2 on a world-size mismatch)."""
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and gpus > 1:
        return spawn_ranks(gpus, script, sys.argv[1:] if argv is None else argv)
    if env_world is not None and int(env_world) != gpus:
        print(f"[{tag}] error: --gpus {gpus} but WORLD_SIZE={env_world}", file=sys.stderr)
        return 2
    return None


def exit_process(code: int | None = 0) -> None:
    """End a rank process WITHOUT interpreter finalisation, once its work is
    done: non-daemon threads are joined, logs and stdio flushed, then
    ``os._exit``.

    Why: a torch.distributed worker thread (gloo's ``runLoop``, after the
    last barrier has already released the main thread) can still be dropping
    the last C++ reference to a tensor whose Python object it must decref.
    If that lands while the interpreter is finalising, Python force-exits the
    thread through noexcept C++ frames -> ``std::terminate`` -> SIGABRT, after
    a run that succeeded (~1 in 60 two-rank CPU runs under load; traced with
    a terminate-handler backtrace to ``ProcessGroupGloo::runLoop`` ->
    ``TensorImpl::decref_pyobject`` -> ``PyEval_AcquireThread`` ->
    ``pthread_exit``).  A launcher (torchrun, the driver, the test harness)
    would count that rank as failed."""
    import logging
    import threading
    if os.environ.get("MFL_EXIT_FINALIZE") == "1" or any(k.startswith("ROCPROF") for k in os.environ):
        # under rocprofv3 (or on request) the interpreter must finalise: the
        # profiler writes its traces from the tool library's exit handlers,
        # which os._exit skips (a profiled bench left no output at all)
        for s in (sys.stdout, sys.stderr):
            try:
                s.flush()
            except Exception:  # noqa: BLE001 - closed stream: nothing to flush
                pass
        sys.exit(int(code or 0))
    me = threading.current_thread()
    for t in threading.enumerate():
        if t is not me and not t.daemon:
            t.join()
    logging.shutdown()
    for s in (sys.stdout, sys.stderr):
        try:
            s.flush()
        except Exception:  # noqa: BLE001 - closed stream: nothing to flush
            pass
    os._exit(int(code or 0))


def exits_hard(fn):
    """Decorator for ``torch.multiprocessing`` rank functions: a rank that
    returns normally leaves through ``exit_process(0)``; an exception still
    propagates to the spawn wrapper (which records it and exits 1)."""
    import functools

    @functools.wraps(fn)
    def rank_main(*args, **kwargs):
        fn(*args, **kwargs)
        exit_process(0)
    return rank_main
