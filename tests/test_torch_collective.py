"""User PyTorch models (TorchModelDef) on the collective data plane
(models/torch_net.py): the module's floating-point parameters
and buffers are views of one flat buffer, so FedAvg over co-located learners
(K1), the all-reduce, FedRec and the driver's ``DataPlane: rccl`` run on them
unchanged.  References: metisfl/models/pytorch/pytorch_model_ops.py:83-131,
examples/pytorch/dummy.py:18-103."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _ionosphere(g, n=48):
    rng = np.random.default_rng(g)
    x = rng.uniform(-1, 1, (n, 34)).astype(np.float32)
    y = (x @ np.random.default_rng(7).standard_normal(34) > 0).astype(np.int64)
    return x, y


def _nets(model_def, L, batch=8, opt=None):
    from metisfl_amd.models.torch_net import TorchNet
    from metisfl_amd.ops.optim import OptimizerSpec
    opt = opt or OptimizerSpec("momentum_sgd", 0.05, momentum=0.5)
    nets, dss, tds = [], [], []
    for g in range(L):
        net = TorchNet(model_def, batch, device="cpu", optimizer=opt, seed=g)
        x, y = _ionosphere(g, 40 + 8 * g)
        nets.append(net)
        dss.append(net.make_dataset(x, y, seed=g))
        xt, yt = _ionosphere(100 + g, 16)
        tds.append(net.make_dataset(xt, yt, seed=g, shuffle=False))
    return nets, dss, tds


def test_module_state_is_the_flat_buffer():
    """Parameters, gradients and BatchNorm buffers are views of model32 /
    grad32: writing the flat buffer changes the module's forward, a backward
    fills the flat gradient, and the fused optimizer step moves the module."""
    from examples.models.torch_models import BrainAge2DCNN
    from metisfl_amd.models.torch_net import TorchNet
    net = TorchNet(BrainAge2DCNN(filters=(4, 8)), 2, device="cpu")
    st = net.state
    names = [s.name for s in st.specs]
    assert any("running_mean" in n for n in names) and any(s.trainable for s in st.specs)
    assert all(not s.trainable for s in st.specs if "running" in s.name)
    for n, p in net.module.named_parameters():
        v = st.view(n)
        assert p.data_ptr() == v.data_ptr() and p.grad.data_ptr() == st.grad(n).data_ptr()
    for n, b in net.module.named_buffers():
        if torch.is_floating_point(b):
            assert b.data_ptr() == st.view(n).data_ptr()
    x = torch.randn(2, 1, 16, 16)
    before = net.module(x).detach().clone()
    st.model32.mul_(0.5)
    assert not torch.allclose(before, net.module(x))
    ds = net.make_dataset(torch.randn(4, 1, 16, 16).numpy(), np.array([60.0, 61.0, 70.0, 50.0], np.float32))
    p0 = st.params32.clone()
    net.train_steps(ds, 2)
    assert not torch.equal(p0, st.params32) and int(st.step.item()) == 2
    assert np.isfinite(net.train_stats()["loss"])


def test_colocated_torch_learners_fedavg():
    """3 co-located Ionosphere MLP learners, synchronous FedAvg: every round's
    community model is the NUM_TRAINING_EXAMPLES-weighted average of the
    local models and every replica holds it."""
    from examples.models.torch_models import IonosphereMLP
    from metisfl_amd.parallel.comm import Comm
    from metisfl_amd.parallel.federation import CollectiveFederation, FederationConfig
    nets, dss, tds = _nets(IonosphereMLP(), 3)
    cfg = FederationConfig(batch_size=8, local_epochs=2)
    fed = CollectiveFederation(Comm(backend="gloo"), nets, dss, cfg, test_ds=tds)
    locs = []
    orig = fed.aggregate

    def spy(meta):
        locs.append([n.state.model32.double().clone() for n in nets])
        return orig(meta)
    fed.aggregate = spy
    for r in range(3):
        rec = fed.run_round()
        w = np.array(rec.weights)
        sizes = np.array([d.n for d in dss], dtype=np.float64)
        assert np.allclose(w, sizes / sizes.sum())
        ref = sum(wi * x for wi, x in zip(w, locs[r]))
        got = nets[0].state.model32.double()
        assert float((got - ref).abs().max()) <= 1e-6
        assert all(torch.equal(n.state.model32, nets[0].state.model32) for n in nets[1:])
        assert rec.community_eval and all(0.0 <= e["accuracy"] <= 1.0 for e in rec.community_eval)
        assert list(rec.learner_meta[:, 1]) == [2 * d.steps_per_epoch for d in dss]


def test_torch_learners_async_fedrec():
    from examples.models.torch_models import IonosphereMLP
    from metisfl_amd.parallel.async_federation import AsyncCollectiveFederation
    from metisfl_amd.parallel.comm import Comm
    from metisfl_amd.parallel.federation import FederationConfig
    nets, dss, tds = _nets(IonosphereMLP(), 3)
    cfg = FederationConfig(protocol="asynchronous", batch_size=8, local_epochs=1)
    fed = AsyncCollectiveFederation(Comm(backend="gloo"), nets, dss, cfg, test_ds=tds)
    fed.run_until(max_updates=9)
    assert fed.version >= 9
    ref = fed.community_reference()
    assert np.abs(fed.community().double().numpy() - ref).max() <= 1e-5 * (np.abs(ref).max() + 1e-12)


def _run_example(args, wd, timeout=900):
    p = subprocess.run([sys.executable] + args + ["--device", "cpu", "--workdir", wd], cwd=ROOT,
                       capture_output=True, text=True, timeout=timeout, env=dict(os.environ, PYTHONPATH=ROOT))
    assert p.returncode == 0, (p.stdout[-3000:], p.stderr[-3000:])
    return json.load(open(os.path.join(wd, "experiment.json")))


def test_neuroimaging_brainage_on_the_collective_plane(tmp_path):
    """examples/neuroimaging.py --env brainage_test_localhost_synchronous.yaml
    with DataPlane: rccl: the BrainAge 3D CNN (a TorchModelDef) trains on the
    collective ranks (gloo here) to the file's round budget."""
    cfg = os.path.join(ROOT, "examples", "config", "brainage", "brainage_test_localhost_synchronous.yaml")
    wd = str(tmp_path / "ni")
    st = _run_example(["examples/neuroimaging.py", "--env", cfg, "--rounds", "3", "--samples", "6",
                       "--shape", "16", "16", "16", "--data-plane", "rccl"], wd)
    md = st["federation_runtime_metadata"]["metadata"]
    assert max(int(m["global_iteration"]) for m in md) >= 3
    log = open(os.path.join(wd, "learner_localhost-1.log")).read()
    assert "[collective] round 3" in log, log[-2000:]


def test_pytorch_dummy_async_on_the_collective_plane(tmp_path):
    """examples/pytorch_dummy.py (the reference's examples/pytorch/dummy.py,
    Ionosphere MLP) with the asynchronous protocol on DataPlane: rccl reaches
    its community-version budget."""
    wd = str(tmp_path / "pd")
    st = _run_example(["examples/pytorch_dummy.py", "--learners", "3", "--rounds", "6", "--protocol", "Asynchronous",
                       "--data-plane", "rccl"], wd)
    md = st["federation_runtime_metadata"]["metadata"]
    assert max(int(m["global_iteration"]) for m in md) >= 6
    log = open(os.path.join(wd, "learner_localhost:0.log")).read()
    line = [l for l in log.splitlines() if l.startswith("[collective-async]")][-1]
    assert "over 3 learners" in line and "stop: rounds" in line, line
