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
