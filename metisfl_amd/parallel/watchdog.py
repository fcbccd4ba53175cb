"""Per-rank heartbeats for the collective federation (SURVEY §5.3 MI355X plan).

A learner process that dies or hangs inside a collective would block every
other rank until the collective timeout.  Each rank publishes a heartbeat
(monotonic counter) into the process group's rendezvous store every
``interval_s``; every rank watches the others and, when a peer's heartbeat
has not advanced for ``timeout_s``, runs ``on_failure`` -- by default it
exits the process with code 75 so that an elastic launcher
(``torchrun --max-restarts N``) restarts the job, which then resumes from the
last federation checkpoint (CollectiveFederation.save_checkpoint / resume).

Fault injection for tests: ``pause()`` stops this rank's heartbeats while
the process keeps running (a hung learner).
"""
from __future__ import annotations

import os
import threading
import time

from metisfl_amd.utils.metis_logger import MetisLogger

EXIT_PEER_LOST = 75


def _default_failure(rank: int, peer: int) -> None:
    """Exit with EXIT_PEER_LOST.  With METISFL_WATCHDOG_REPORT_DIR set (the
    driver sets it), first record which peer went silent: a HUNG rank never
    exits by itself, so the driver learns from these reports which of the
    ranks it has to stop is the failed one (driver_session._recover_collective)."""
    MetisLogger.error("rank %d: peer rank %d lost its heartbeat; exiting for an elastic restart", rank, peer)
    d = os.environ.get("METISFL_WATCHDOG_REPORT_DIR")
    if d:
        try:
            import json
            os.makedirs(d, exist_ok=True)
            with open(os.path.join(d, f"lost_by_rank{rank}.json"), "w") as f:
                json.dump({"rank": rank, "peer": peer}, f)
        except OSError:
            pass
    os._exit(EXIT_PEER_LOST)


class RankWatchdog:
    def __init__(self, comm, interval_s: float = 2.0, timeout_s: float = 30.0, on_failure=None,
                 store=None, prefix: str = "metisfl_hb"):
        self.comm = comm
        self.interval = interval_s
        self.timeout = timeout_s
        self.on_failure = on_failure or _default_failure
        self.prefix = prefix
        if store is None and comm.distributed:
            import torch.distributed as dist
            store = dist.distributed_c10d._get_default_store()
        self.store = store
        self._beat = 0
        self._paused = threading.Event()
        self._stop = threading.Event()
        self._last_seen: dict[int, tuple[int, float]] = {}
        self.lost: list[int] = []
        self._thread = threading.Thread(target=self._loop, name="rank-watchdog", daemon=True)

    def start(self) -> "RankWatchdog":
        if self.store is not None:
            self._publish()
            self._thread.start()
        return self

    def stop(self) -> None:
        """Stop and join the heartbeat thread -- before the process group (and
        its store) is destroyed: a store call racing the teardown aborts the
        process (std::terminate)."""
        self._stop.set()
        if self._thread.is_alive():
            self._thread.join(timeout=5 * self.interval + 5)

    def pause(self) -> None:  # fault injection
        self._paused.set()

    def _publish(self) -> None:
        self._beat += 1
        self.store.set(f"{self.prefix}/{self.comm.rank}", str(self._beat))

    def check_peers(self) -> list[int]:
        now = time.monotonic()
        lost = []
        for peer in range(self.comm.world):
            if peer == self.comm.rank or peer in self.lost:
                continue
            try:
                v = int(self.store.get(f"{self.prefix}/{peer}").decode() or 0) \
                    if self.store.check([f"{self.prefix}/{peer}"]) else 0
            except Exception:  # noqa: BLE001 - store unreachable counts as silence
                v = -1
            prev = self._last_seen.get(peer)
            if prev is None or v != prev[0]:
                self._last_seen[peer] = (v, now)
            elif now - prev[1] > self.timeout:
                lost.append(peer)
        return lost

    def _loop(self) -> None:
        while not self._stop.wait(self.interval):
            if not self._paused.is_set():
                try:
                    self._publish()
                except Exception:  # noqa: BLE001
                    pass
            for peer in self.check_peers():
                self.lost.append(peer)
                self.on_failure(self.comm.rank, peer)
