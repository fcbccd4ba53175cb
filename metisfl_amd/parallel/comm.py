"""Process-group plumbing: one process per GPU, RCCL over xGMI.

The reference moves every model through the controller over gRPC
(controller.cc:696-793: one serialized RunTaskRequest per learner, a fresh
channel per request).  On one MI355X node the data plane is instead a set of
RCCL collectives between the learner processes (torch.distributed backend
``nccl`` IS RCCL on ROCm); the gRPC services remain the control plane for
remote learners and API parity.  CPU-only runs (tests) use ``gloo`` with the
identical code path.

``MFL_COMM_BACKEND=gloo`` on a GPU host keeps the compute on the GPU and runs
the collectives over gloo, staged through host memory: several ranks can then
share ONE GPU (RCCL refuses two ranks on the same device), which is how the
multi-rank paths -- the hierarchical co-located sum + all-reduce, rank 0's
asynchronous service thread -- are rehearsed with real HIP graphs and streams
on a one-GPU box (tests/test_multirank_gpu.py).  Ranks map to
``LOCAL_RANK % device_count``.  A rehearsal mode, not a data plane: every
collective pays a device <-> host round trip.
"""
from __future__ import annotations

import datetime
import os

import torch
import torch.distributed as dist


class Comm:
    def __init__(self, backend: str | None = None, timeout_s: float = 1800.0):
        self.rank = int(os.environ.get("RANK", "0"))
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.local_rank = int(os.environ.get("LOCAL_RANK", str(self.rank)))
        # host-staged gloo on GPU ranks (module docstring)
        self.staged = backend is None and os.environ.get("MFL_COMM_BACKEND") == "gloo" and torch.cuda.is_available()
        use_cuda = torch.cuda.is_available() and backend != "gloo"
        if use_cuda:
            idx = self.local_rank % torch.cuda.device_count() if self.staged else self.local_rank
            torch.cuda.set_device(idx)
            self.device = torch.device("cuda", idx)
        else:
            self.device = torch.device("cpu")
        self.backend = "gloo" if self.staged else (backend or ("nccl" if use_cuda else "gloo"))
        self.owned = False
        if self.world > 1 and not dist.is_initialized():
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            kw = {}
            if self.backend == "nccl":
                kw["device_id"] = self.device
            dist.init_process_group(self.backend, rank=self.rank, world_size=self.world,
                                    timeout=datetime.timedelta(seconds=timeout_s), **kw)
            self.owned = True
        self.pg = dist.group.WORLD if self.world > 1 else None

    @property
    def distributed(self) -> bool:
        return self.world > 1

    def barrier(self) -> None:
        if self.distributed:
            if self.backend == "nccl":
                dist.barrier(device_ids=[self.local_rank])
            else:
                dist.barrier()

    # host staging of a device tensor for the gloo rehearsal mode
    def _host(self, t: torch.Tensor) -> torch.Tensor:
        return t.cpu() if self.staged and t.is_cuda else t

    @staticmethod
    def _back(t: torch.Tensor, h: torch.Tensor) -> None:
        if h is not t:
            t.copy_(h)

    def all_reduce_(self, t: torch.Tensor) -> None:
        if self.distributed:
            h = self._host(t)
            dist.all_reduce(h, op=dist.ReduceOp.SUM)
            self._back(t, h)

    def broadcast_(self, t: torch.Tensor, src: int = 0) -> None:
        if self.distributed:
            h = self._host(t)
            dist.broadcast(h, src=src)
            self._back(t, h)

    def send(self, t: torch.Tensor, dst: int, group=None) -> None:
        """Point-to-point send (``group``: e.g. the asynchronous protocol's own)."""
        dist.send(self._host(t), dst=dst, group=group)

    def recv(self, t: torch.Tensor, src: int, group=None) -> None:
        # (staged: a host landing buffer, nothing to copy down first)
        h = torch.empty(t.shape, dtype=t.dtype) if self.staged and t.is_cuda else t
        dist.recv(h, src=src, group=group)
        self._back(t, h)

    def broadcast_bytes(self, data: bytes | None, src: int = 0) -> bytes:
        """Small host blob (keys, configs) from ``src`` to every rank."""
        if not self.distributed:
            return data or b""
        n = torch.tensor([len(data) if self.rank == src else 0], dtype=torch.int64, device=self.device)
        self.broadcast_(n, src=src)
        buf = torch.empty(int(n.item()), dtype=torch.uint8, device=self.device)
        if self.rank == src:
            buf.copy_(torch.frombuffer(bytearray(data), dtype=torch.uint8))
        self.broadcast_(buf, src=src)
        return bytes(buf.cpu().numpy().tobytes())

    def all_gather_rows(self, row: torch.Tensor) -> torch.Tensor:
        """Gather one small 1-D tensor per rank -> [world, n] (on row.device)."""
        if not self.distributed:
            return row.reshape(1, -1).clone()
        # flat output: gloo's allgather_base wants chunks shaped like the input
        dev = torch.device("cpu") if self.staged else row.device
        out = torch.empty(self.world * row.numel(), dtype=row.dtype, device=dev)
        dist.all_gather_into_tensor(out, self._host(row.contiguous().reshape(-1)))
        return out.view(self.world, row.numel()).to(row.device)

    def all_max(self, x: float) -> float:
        if not self.distributed:
            return x
        t = torch.tensor([x], dtype=torch.float64, device=self.device)
        h = self._host(t)
        dist.all_reduce(h, op=dist.ReduceOp.MAX)
        return float(h.item())

    def close(self) -> None:
        if self.owned and dist.is_initialized():
            # every rank reaches the teardown together: a gloo rank destroying
            # its pairs while a peer's last collective is still draining was
            # seen to abort the peer ("terminate called without an active
            # exception", 1 in ~4 three-rank runs)
            if self.distributed:
                try:
                    dist.barrier()
                except RuntimeError:
                    pass  # a peer is already gone (lost-rank paths): tear down anyway
            dist.destroy_process_group()
            self.owned = False
