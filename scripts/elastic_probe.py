"""Where does the host block in CoLocatedLearners.train_elastic?  Times every
graph replay and epoch reshuffle of a slow (batch 256) and two fast (batch 16)
co-located learners."""
import time

import numpy as np
import torch

from metisfl_amd.models.colocated import CoLocatedLearners
from metisfl_amd.models.net import DeviceDataset
from metisfl_amd.models.resnet import ResNet18
from metisfl_amd.ops.optim import OptimizerSpec

log = []
_orig_rs = DeviceDataset.reshuffle
_orig_replay = torch.cuda.CUDAGraph.replay


def rs(self):
    t = time.perf_counter()
    _orig_rs(self)
    log.append(("reshuffle", self.batch_size, (time.perf_counter() - t) * 1e3))


def rp(self):
    t = time.perf_counter()
    _orig_replay(self)
    log.append(("replay", 0, (time.perf_counter() - t) * 1e3))


DeviceDataset.reshuffle = rs
torch.cuda.CUDAGraph.replay = rp
nets, dss = [], []
for j, b in enumerate((16, 16, 256)):
    net = ResNet18(batch_size=b, device="cuda", seed=7, optimizer=OptimizerSpec("momentum_sgd", 0.005, 0.75))
    rng = np.random.default_rng(j)
    m = 4096
    nets.append(net)
    dss.append(net.make_dataset(rng.standard_normal((m, 32, 32, 3)).astype(np.float32), rng.integers(0, 10, m), seed=j))
group = CoLocatedLearners(nets, dss)
group.train([8, 8, 8], [0, 0, 0])
torch.cuda.synchronize()
log.clear()
done, tq = [], []


def on_finish(j):
    done.append(j)
    log.append(("finish", j, time.perf_counter()))
    if len(done) == 2:
        tq.append(time.perf_counter())


t0 = time.perf_counter()
ms, ran, part = group.train_elastic([16, 16, 64], [8, 8, 8], lambda: len(done) >= 2, on_finish, poll_steps=16,
                                    poll_s=0.0)
t1 = time.perf_counter()
print("return after quorum ms", (t1 - tq[0]) * 1e3, "total", (t1 - t0) * 1e3, ran, part)
for e in log:
    if e[0] == "finish":
        print("finish", e[1], (e[2] - t0) * 1e3)
    else:
        print(e)
