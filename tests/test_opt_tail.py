"""Optimizer tails (models/layers.py OptTailScheduler, conv32.h OptTail):
the optimizer step of the variables whose backward has finished rides in
later paired backward launches, the step's last launch updates the rest.
The update is elementwise, so the result must equal the single optimizer
launch: bitwise on the host path, and on the GPU through the bench's
K-update graph (lr 0: bitwise forward; lr > 0: within the run-to-run spread
of the split-K weight-gradient atomics)."""
import numpy as np
import pytest
import torch


def _pair(device, chunk, monkeypatch, B=4, width=0.25, lr=0.05, kind="momentum_sgd", dtype="fp32"):
    from metisfl_amd.models.layers import OptTailScheduler
    from metisfl_amd.models.resnet import ResNet18
    from metisfl_amd.ops.optim import OptimizerSpec
    spec = OptimizerSpec(kind, lr, momentum=0.75) if kind == "momentum_sgd" else OptimizerSpec(kind, lr)
    nets = [ResNet18(batch_size=B, device=device, seed=3, width_mult=width, optimizer=spec, dtype=dtype)
            for _ in range(2)]
    return nets, OptTailScheduler


def _data(n, seed=0):
    rng = np.random.default_rng(seed)
    return rng.standard_normal((n, 32, 32, 3)).astype(np.float32), rng.integers(0, 10, n)


def test_scheduler_chunks_cover_the_ready_range_top_down():
    from metisfl_amd.models.layers import OptTailScheduler
    from metisfl_amd.models.resnet import ResNet18
    st = ResNet18(batch_size=2, width_mult=0.25).state
    s = OptTailScheduler(st, True)
    s.chunk = 1000
    assert s.take() is None  # nothing final yet
    lo4 = st.offset_of_prefix("layer4.")
    s.mark_ready(lo4)
    got, prev = [], st.n_params
    while True:
        r = s.take()
        if r is None:
            break
        n = r.numel
        assert 0 < n <= 1000 + 64
        assert r.p.data_ptr() == st.params32[prev - n:].data_ptr()
        got.append(n)
        prev -= n
    assert prev == lo4 == s.done and sum(got) == st.n_params - lo4


@pytest.mark.parametrize("kind,chunk", [("momentum_sgd", 3000), ("momentum_sgd", 10 ** 9), ("adam", 5000),
                                        ("vanilla_sgd", 2000)])
def test_opt_tails_are_bitwise_on_host(kind, chunk, monkeypatch):
    (base, tail), S = _pair("cpu", chunk, monkeypatch, kind=kind)
    x, y = _data(16)
    dsb = base.make_dataset(x, y, seed=1)
    dst = tail.make_dataset(x, y, seed=1)
    monkeypatch.setattr(S, "chunk", 0)
    for _ in range(3):
        base._train_body(dsb)
    monkeypatch.setattr(S, "chunk", chunk)
    taken = []
    orig = S.take

    def spy(self, everything=False):
        r = orig(self, everything)
        if r is not None:
            taken.append(r.numel)
        return r
    monkeypatch.setattr(S, "take", spy)
    for _ in range(3):
        tail._train_body(dst)
    assert taken, "no optimizer tail was scheduled"
    assert torch.equal(base.state.model32, tail.state.model32)
    if base.state.m is not None:
        assert torch.equal(base.state.m, tail.state.m)
    assert int(base.state.step) == int(tail.state.step) == 3
    assert float(tail.state.grad32.abs().max()) == 0.0


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_opt_tails_graph_full_width(monkeypatch, dtype):
    B = 32
    (base, tail), S = _pair("cuda", 0, monkeypatch, B=B, width=1.0, lr=0.0, dtype=dtype)
    x, y = _data(512)
    dsb = base.make_dataset(x, y, seed=1)
    dst = tail.make_dataset(x, y, seed=1)
    monkeypatch.setattr(S, "chunk", 0)
    base.prepare_graphs(dsb, 16)
    monkeypatch.setattr(S, "chunk", 1 << 20)
    tail.prepare_graphs(dst, 16)
    for _ in range(2):
        base._train_graph_k.replay()
        tail._train_graph_k.replay()
    torch.cuda.synchronize()
    # lr 0: nothing moves, the mirror stays the split of the master, every
    # gradient range was consumed and re-zeroed
    assert torch.equal(base.state.model32, tail.state.model32)
    mirror = "psplit" if dtype == "fp32" else "p16"
    assert torch.equal(getattr(base.state, mirror), getattr(tail.state, mirror))
    assert float(tail.state.grad32.abs().max()) == 0.0
    assert int(tail.state.step) == 16


@pytest.mark.gpu
def test_opt_tails_train_like_one_launch(monkeypatch):
    """16 updates at the bench's learning rate: the split-K weight gradients
    accumulate with fp32 atomics in arrival order, so two runs of the SAME
    configuration already differ and the difference grows chaotically; the
    tail run must stay within a few times that run-to-run spread."""
    B = 32
    (base, tail), S = _pair("cuda", 0, monkeypatch, B=B, width=1.0, lr=0.005)
    (base2, _), _ = _pair("cuda", 0, monkeypatch, B=B, width=1.0, lr=0.005)
    x, y = _data(512)
    monkeypatch.setattr(S, "chunk", 0)
    for n in (base, base2):
        n.train_steps(n.make_dataset(x, y, seed=1), 16)
    monkeypatch.setattr(S, "chunk", 1 << 20)
    tail.train_steps(tail.make_dataset(x, y, seed=1), 16)
    torch.cuda.synchronize()

    def rel(u, v):
        u, v = u.double(), v.double()
        return float((u - v).norm() / v.norm())
    r = rel(tail.state.params32, base.state.params32)
    spread = rel(base2.state.params32, base.state.params32)
    print(f"tail vs one launch rel {r:.2e}, run-to-run {spread:.2e}")
    assert r <= max(5 * spread, 1e-5), (r, spread)
    from metisfl_amd.ops import optim as opt_ops
    ref = torch.empty_like(tail.state.psplit)
    opt_ops.split_pack(tail.state.params32, ref)
    assert torch.equal(ref, tail.state.psplit)
