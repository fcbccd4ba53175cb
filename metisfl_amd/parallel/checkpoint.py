"""Checkpoints and community-model snapshots off the round's critical path.

The reference has no checkpointing and replaces its in-memory
community model every global iteration (controller.cc:466).  Here a round
ends with the community model resident in HBM; persisting it (or handing it
to the controller's lineage) used to mean a synchronous D2H copy, a Python
proto build and file writes on every rank before the next round could start.

``AsyncSnapshot`` splits that into
  1. a device-to-device copy on the caller's stream (HBM rate, ~30 us for
     ResNet-18's model + momentum), then a device -> pinned-host copy of that
     private copy on a side HIP stream (the compute stream does not wait for
     it, and may overwrite the originals right away), and
  2. everything else -- waiting for the copy, serialization, file writes,
     gRPC -- on one background thread, while the next round trains.
The pinned buffers are reused; a new snapshot waits for the previous one only
if that is still being written (back-pressure instead of unbounded memory).

Checkpoint directories are versioned: ``<root>/round_<gi>/`` holds the files
of one checkpoint and ``<root>/LATEST`` names the newest COMPLETE one; it is
replaced atomically after every rank's files are on disk (ranks report
through the process group's key-value store), so a crash mid-write leaves
the previous checkpoint valid.  ``resolve`` maps a root (or a legacy flat
directory) to the checkpoint to load.
"""
from __future__ import annotations

import os
import shutil
import threading
import time

import torch

LATEST = "LATEST"
PUBLISH_POLL_S = 0.05  # rank 0's poll interval for the other ranks' checkpoint keys


def resolve(path: str | None) -> str | None:
    """The checkpoint directory to load from ``path``: the one LATEST names,
    or ``path`` itself when it holds a (legacy, flat) checkpoint; None when
    there is none."""
    if not path:
        return None
    latest = os.path.join(path, LATEST)
    if os.path.exists(latest):
        with open(latest) as f:
            name = f.read().strip()
        d = os.path.join(path, name)
        if os.path.exists(os.path.join(d, "federation.json")):
            return d
    if os.path.exists(os.path.join(path, "federation.json")):
        return path
    return None


def atomic_write(path: str, data: bytes) -> None:
    tmp = f"{path}.tmp{os.getpid()}"
    with open(tmp, "wb") as f:
        f.write(data)
    os.replace(tmp, path)


def atomic_torch_save(obj, path: str) -> None:
    tmp = f"{path}.tmp{os.getpid()}"
    torch.save(obj, tmp)
    os.replace(tmp, path)


_ST_DTYPES = {torch.float32: "F32", torch.float64: "F64", torch.float16: "F16", torch.bfloat16: "BF16",
              torch.int64: "I64", torch.int32: "I32", torch.int16: "I16", torch.int8: "I8", torch.uint8: "U8",
              torch.bool: "BOOL"}


def save_tensors(tensors: dict, path: str) -> None:
    """Write host tensors in the safetensors layout, atomically.  The native
    writer (_engine.write_safetensors) holds no GIL while it writes, so a
    background checkpoint never competes with the training thread's launch
    loop for the interpreter; ``load_tensors`` (safetensors' own reader)
    reads it back without executing anything from the file."""
    from metisfl_amd import _engine as E
    names, bufs, dts, shapes = [], [], [], []
    for k in sorted(tensors):
        t = tensors[k].detach().cpu().contiguous()
        names.append(k)
        # bf16 has no buffer protocol: ship its bits as int16
        bufs.append((t.view(torch.int16) if t.dtype == torch.bfloat16 else t).reshape(-1).numpy())
        dts.append(_ST_DTYPES[t.dtype])
        shapes.append(list(t.shape))
    E.write_safetensors(path, names, bufs, dts, shapes)


def load_tensors(path: str) -> dict:
    from safetensors.torch import load_file
    return load_file(path)


def write_federated_model(path: str, flat, specs, num_contributors: int, global_iteration: int) -> None:
    """Serialize the flat fp32 community model as the reference's
    ``FederatedModel`` message (model.proto:48-52) natively, GIL released."""
    from metisfl_amd import _engine as E
    E.write_federated_model(path, flat, [s.name for s in specs], [list(s.shape) for s in specs],
                            [int(s.offset) for s in specs], [bool(s.trainable) for s in specs],
                            int(num_contributors), int(global_iteration))


class AsyncSnapshot:
    """One background writer with reusable pinned staging buffers."""

    def __init__(self, device: torch.device, name: str = "metisfl-snapshot"):
        self.device = torch.device(device)
        self.cuda = self.device.type == "cuda"
        self.stream = torch.cuda.Stream(device=self.device) if self.cuda else None
        self._host: dict[str, torch.Tensor] = {}   # pinned host staging
        self._dev: dict[str, torch.Tensor] = {}    # device-side snapshot copies
        self._thread: threading.Thread | None = None
        self._error: BaseException | None = None
        self.name = name
        self.last_stage_ms = 0.0
        self.last_wait_ms = 0.0    # of last_stage_ms: waiting for the previous snapshot's writer
        self.last_d2d_issue_ms = 0.0
        self.last_write_ms = 0.0

    def _buf(self, pool: dict, key: str, t: torch.Tensor, pinned: bool, device=None) -> torch.Tensor:
        b = pool.get(key)
        if b is None or b.shape != t.shape or b.dtype != t.dtype:
            b = (torch.empty(t.shape, dtype=t.dtype, device=device) if device is not None
                 else torch.empty(t.shape, dtype=t.dtype, pin_memory=pinned))
            pool[key] = b
        return b

    def wait(self) -> None:
        """Block until the previous snapshot is fully written (re-raises its
        error)."""
        if self._thread is not None:
            self._thread.join()
            self._thread = None
        if self._error is not None:
            e, self._error = self._error, None
            raise RuntimeError(f"{self.name} failed") from e

    def busy(self) -> bool:
        return self._thread is not None and self._thread.is_alive()

    def try_submit(self, tensors: dict[str, torch.Tensor], write) -> float | None:
        """``submit`` unless the previous snapshot is still being written
        (then nothing is staged: None) -- for best-effort snapshots taken
        under a lock (the asynchronous aggregator)."""
        if self.busy():
            return None
        return self.submit(tensors, write)

    def submit(self, tensors: dict[str, torch.Tensor], write) -> float:
        """Snapshot ``tensors`` (device or host) as they are NOW and run
        ``write(host_tensors)`` on the background thread once they are on the
        host.  Device tensors are first copied device-to-device on the
        current stream (HBM rate: ~30 us for 90 MB), so the caller may
        overwrite them right away; the D2H copy of that private copy runs on
        the side stream.  Returns the milliseconds this call held the caller
        (the critical-path cost)."""
        t0 = time.perf_counter()
        self.wait()  # the staging buffers are about to be reused
        self.last_wait_ms = (time.perf_counter() - t0) * 1e3
        host = {}
        ev = None
        if self.cuda:
            cur = torch.cuda.current_stream(self.device)
            staged = {}
            for k, t in tensors.items():
                if t.is_cuda:
                    d = self._buf(self._dev, k, t, False, device=t.device)
                    d.copy_(t)
                    staged[k] = d
            t1 = time.perf_counter()
            self.last_d2d_issue_ms = (t1 - t0) * 1e3 - self.last_wait_ms
            self.stream.wait_stream(cur)
            with torch.cuda.stream(self.stream):
                for k, t in tensors.items():
                    if k in staged:
                        b = self._buf(self._host, k, t, True)
                        b.copy_(staged[k], non_blocking=True)
                        host[k] = b
                    else:
                        host[k] = t.detach().clone()
                ev = torch.cuda.Event()
                ev.record(self.stream)
        else:
            host = {k: t.detach().clone() for k, t in tensors.items()}

        def run():
            try:
                t1 = time.perf_counter()
                if ev is not None:
                    ev.synchronize()
                write(host)
                self.last_write_ms = (time.perf_counter() - t1) * 1e3
            except BaseException as e:  # noqa: BLE001 - re-raised by wait()
                self._error = e

        # not a daemon: the interpreter joins it before finalising.  A daemon
        # writer still inside a torch / numpy call (GIL released) when the
        # process exits is force-unwound through noexcept C++ frames at
        # finalisation -> std::terminate, SIGABRT after a successful run (seen
        # as "terminate called without an active exception", ~1 in 60
        # two-rank runs, traced to this thread with a terminate-handler
        # backtrace).
        self._thread = threading.Thread(target=run, name=self.name, daemon=False)
        self._thread.start()
        self.last_stage_ms = (time.perf_counter() - t0) * 1e3
        return self.last_stage_ms


def publish(root: str, name: str, store=None, world: int = 1, key: str = "", keep: int = 2,
            timeout_s: float = 600.0) -> None:
    """Rank 0, after writing its own files of checkpoint ``root/name``: wait
    until every rank reported its files (store keys ``<key>/<rank>``), then
    point LATEST at it and prune older checkpoints (the newest ``keep``
    stay)."""
    if store is not None and world > 1:
        keys = [f"{key}/{r}" for r in range(world)]
        # short polls, not one long store.wait: the c10d store client
        # serialises its operations, and the rank watchdog's heartbeats go
        # through the same client -- a blocking wait for a slow or
        # dead peer's key would silence this rank's heartbeat as well
        end = time.time() + timeout_s
        while not store.check(keys):
            if time.time() > end:
                raise TimeoutError(f"checkpoint {name}: not every rank reported its files in {timeout_s:.0f} s")
            time.sleep(PUBLISH_POLL_S)
    atomic_write(os.path.join(root, LATEST), name.encode())
    rounds = sorted((d for d in os.listdir(root) if d.startswith("round_") and d != name),
                    key=lambda d: int(d.split("_")[1]) if d.split("_")[1].isdigit() else -1)
    for d in rounds[: max(0, len(rounds) - (keep - 1))]:
        shutil.rmtree(os.path.join(root, d), ignore_errors=True)


