"""The bench's hot path pinned against eager execution: the full-width fp32
ResNet-18 at batch 32 (the BASELINE config) with its 8-update captured
hipGraph (models/net.py ``graph_steps``, MFL_GRAPH_STEPS) against 8 eager
``_train_body`` calls, and co-located learners (one HIP stream each,
models/colocated.py) against the same learners run one after another.

lr = 0 keeps the weights fixed, so nothing is amplified chaotically: every
update sees the same model, and the comparisons are per-update loss /
accuracy sums, the last update's gradient buffer and the BatchNorm running
statistics (which integrate all 8 updates).  A second replay of the same
graph must agree again: the halo convs' split-K arrival tickets and the BN
accumulators must re-arm across replays."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

B = 32


def _net(seed=7, lr=0.0, conv_products=None):
    from metisfl_amd.models.resnet import ResNet18
    from metisfl_amd.ops.optim import OptimizerSpec
    return ResNet18(batch_size=B, device="cuda", optimizer=OptimizerSpec("momentum_sgd", lr, momentum=0.75),
                    seed=seed, conv_products=conv_products)


def _data(n=512, seed=0):
    rng = np.random.default_rng(seed)
    return rng.standard_normal((n, 32, 32, 3)).astype(np.float32), rng.integers(0, 10, n)


def _rel(a, b):
    a, b = a.double(), b.double()
    return float((a - b).abs().max() / max(1e-30, float(b.abs().max())))


def _frozen(net):
    st = net.state
    return torch.cat([st.view(s.name).reshape(-1) for s in st.specs if not s.trainable])


def test_k8_graph_replay_matches_eager_full_width():
    x, y = _data()
    g = _net()
    e = _net()
    assert g.graph_steps == 8, "the bench's graph length"
    g.zero_grad_in_optimizer = e.zero_grad_in_optimizer = False  # the last update's gradient stays readable
    dg = g.make_dataset(x, y, seed=1)
    de = e.make_dataset(x, y, seed=1)
    assert torch.equal(dg.perm, de.perm)
    g.prepare_graphs(dg, 16)
    assert g._train_graph_k is not None
    for rep in range(2):
        g.reset_train_stats()
        e.reset_train_stats()
        g._train_graph_k.replay()
        for _ in range(8):
            e._train_body(de)
        torch.cuda.synchronize()
        assert int(g.state.step.cpu()) == int(e.state.step.cpu()) == 8 * (rep + 1)
        sg, se = g.stats.cpu(), e.stats.cpu()
        assert float(sg[2]) == float(se[2]) == 8 * B
        assert abs(float(sg[0]) - float(se[0])) <= 1e-5 * abs(float(se[0])), (rep, sg, se)  # loss sum
        assert abs(float(sg[1]) - float(se[1])) <= 1.0  # correct predictions (a near-tie may flip)
        rg = _rel(g.state.grad32, e.state.grad32)
        rb = _rel(_frozen(g), _frozen(e))
        print(f"replay {rep}: loss {float(sg[0]) / (8 * B):.5f}, grad rel {rg:.2e}, BN running stats rel {rb:.2e}")
        assert rg <= 1e-5, rg
        assert rb <= 1e-5, rb
        assert torch.equal(g.state.model32[: g.state.n_params], e.state.model32[: e.state.n_params])  # lr 0


def _pair_ring():
    """The LDS ring the co-located group selects (process-wide, before any
    capture): the sequential references run the same kernels."""
    from metisfl_amd.models.colocated import CoLocatedLearners
    if CoLocatedLearners.pair_ring:
        CoLocatedLearners._set_pair_ring(int(CoLocatedLearners.pair_ring))


@pytest.mark.parametrize("n", [4, 8])
def test_colocated_streams_match_sequential_learners(n):
    """n learners replaying their graphs concurrently on n streams compute
    what the same n learners compute one after another (no shared scratch,
    no cross-stream race) -- 8 is the bench's group, more streams than the
    4 hardware queues (GPU_MAX_HW_QUEUES), with the 2-stage pair ring.
    lr 0: bitwise (forward, BN running statistics, loss sums).  16 updates
    at the bench's learning rate: the split-K weight gradients accumulate
    with fp32 atomics in arrival order, so two SEQUENTIAL runs already differ
    and the difference grows chaotically; the co-located run must stay
    within a few times that run-to-run spread."""
    from metisfl_amd.models.colocated import CoLocatedLearners
    _pair_ring()

    def make(lr):
        out = []
        for j in range(n):
            net = _net(seed=11 + j, lr=lr)
            x, y = _data(256, 20 + j)
            out.append((net, net.make_dataset(x, y, seed=j)))
        return out

    for lr in (0.0, 0.005):
        seq, seq2, co = make(lr), make(lr), make(lr)
        for grp in (seq, seq2):
            for net, ds in grp:
                net.train_steps(ds, 16)
        group = CoLocatedLearners([n_ for n_, _ in co], [d for _, d in co])
        assert len(group.streams) == n and len({s.stream_id for s in group.streams}) == n
        ms = group.train([16] * n, [0] * n)
        torch.cuda.synchronize()
        assert len(ms) == n and all(m > 0 for m in ms)
        for (a, _), (a2, _), (b, _) in zip(seq, seq2, co):
            assert int(a.state.step.cpu()) == int(b.state.step.cpu()) == 16
            r = _rel(b.state.model32, a.state.model32)
            spread = _rel(a2.state.model32, a.state.model32)
            ls = abs(b.train_stats()["loss"] - a.train_stats()["loss"])
            print(f"lr {lr}: co-located vs sequential rel {r:.2e}, sequential run-to-run {spread:.2e}, "
                  f"loss diff {ls:.2e}")
            if lr == 0.0:
                assert r == 0.0 and ls <= 1e-6, (r, ls)
            else:
                assert r <= max(5 * spread, 1e-5), (r, spread)


def test_colocated_federation_round_matches_sequential_fedavg():
    """One CollectiveFederation round of the bench's shape (8 co-located
    learners on one GPU, hierarchical FedAvg: one weighted-sum launch) against
    the same federation whose learners train one after another on the default
    stream.  lr 0: the community model (weights, and the BN running
    statistics the round averages) is bitwise equal; lr 0.005: within the
    run-to-run spread of two sequential federations."""
    from metisfl_amd.parallel.comm import Comm
    from metisfl_amd.parallel.federation import CollectiveFederation, FederationConfig
    _pair_ring()

    def fed_round(lr, sequential):
        nets, dss = [], []
        for j in range(8):
            net = _net(seed=31 + j, lr=lr)
            x, y = _data(256, 40 + j)
            nets.append(net)
            dss.append(net.make_dataset(x, y, seed=j))
        cfg = FederationConfig(batch_size=B, local_epochs=2, evaluate_test=False, evaluate_community=False)
        fed = CollectiveFederation(Comm(), nets, dss, cfg)
        assert fed.group is not None and len(fed.group.streams) == 8
        if sequential:
            def one_after_another(nsteps, offsets):
                for net, ds, k, off in zip(nets, dss, nsteps, offsets):
                    net.train_steps(ds, k, step_offset=off)
                torch.cuda.synchronize()
                return [1.0] * len(nets)
            fed.group.train = one_after_another
        rec = fed.run_round()
        assert rec.num_local_updates == [16] * 8
        torch.cuda.synchronize()
        return fed.net.state.model32.clone(), [n.train_stats()["loss"] for n in nets]

    for lr in (0.0, 0.005):
        a, la = fed_round(lr, True)
        a2, _ = fed_round(lr, True)
        b, lb = fed_round(lr, False)
        r, spread = _rel(b, a), _rel(a2, a)
        print(f"lr {lr}: 8 co-located vs sequential community rel {r:.2e}, sequential run-to-run {spread:.2e}")
        if lr == 0.0:
            # (the per-step loss sums are fp32 atomics: ulp-level order effects)
            assert torch.equal(a, b) and max(abs(x - y) / max(1.0, abs(y)) for x, y in zip(la, lb)) <= 2e-6
        else:
            assert r <= max(5 * spread, 1e-5), (r, spread)
