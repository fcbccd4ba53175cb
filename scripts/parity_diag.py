"""Per-tensor gradient error of the fp32 ResNet-18 step against the fp64
torch.nn oracle, next to torch's own fp32 error (the noise floor), sorted by
the ratio.  python scripts/parity_diag.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from metisfl_amd.models.resnet import ResNet18  # noqa: E402
from metisfl_amd.ops.optim import OptimizerSpec  # noqa: E402
from tests.torch_resnet_ref import reference_step  # noqa: E402


def rel(a, b):
    a, b = a.double().cpu().flatten(), b.double().cpu().flatten()
    return float((a - b).norm() / (b.norm() + 1e-300))


def main():
    rng = np.random.default_rng(0)
    B = 32
    x = rng.standard_normal((B, 32, 32, 3)).astype(np.float32)
    y = rng.integers(0, 10, B)
    net = ResNet18(batch_size=B, device="cuda", optimizer=OptimizerSpec("vanilla_sgd", 0.0), seed=4)
    values = net.state.to_numpy()
    ds = net.make_dataset(x, y, shuffle=False)
    net.zero_grad_in_optimizer = False
    net._train_body(ds)
    torch.cuda.synchronize()
    x8 = F.pad(torch.as_tensor(x), (0, 5))
    _, g64, _ = reference_step(values, x8, torch.as_tensor(y))
    _, g32, _ = reference_step(values, x8, torch.as_tensor(y), dtype=torch.float32)
    rows = []
    for n, r in g64.items():
        e, f = rel(net.state.grad(n), r), rel(g32[n], r)
        rows.append((e / max(f, 1e-12), e, f, float(r.norm()), n))
    rows.sort(reverse=True)
    for q, e, f, nrm, n in rows[:25]:
        print(f"{n:40s} ours {e:9.2e}  torch32 {f:9.2e}  ratio {q:8.1f}  |g| {nrm:9.3e}")


if __name__ == "__main__" and len(sys.argv) == 1:
    main()


def forward_check():
    """Block outputs of the executor vs the fp64 oracle's (forward hooks)."""
    from tests.torch_resnet_ref import TorchResNet18
    rng = np.random.default_rng(0)
    B = 32
    x = rng.standard_normal((B, 32, 32, 3)).astype(np.float32)
    y = rng.integers(0, 10, B)
    net = ResNet18(batch_size=B, device="cuda", optimizer=OptimizerSpec("vanilla_sgd", 0.0), seed=4)
    values = net.state.to_numpy()
    ds = net.make_dataset(x, y, shuffle=False)
    net.zero_grad_in_optimizer = False
    net._train_body(ds)
    torch.cuda.synchronize()
    m = TorchResNet18().double()
    m.load_from(values)
    m.train()
    outs = {}
    m.stem.register_forward_hook(lambda mod, i, o: outs.__setitem__("stem_z", o))
    for bi, b in enumerate(m.blocks):
        b.register_forward_hook(lambda mod, i, o, bi=bi: outs.__setitem__(f"block{bi}", o))
        b.conv1.register_forward_hook(lambda mod, i, o, bi=bi: outs.__setitem__(f"block{bi}.z1", o))
    xx = F.pad(torch.as_tensor(x), (0, 5)).double().permute(0, 3, 1, 2)
    logits = m(xx)
    for o in outs.values():
        o.retain_grad()
    F.cross_entropy(logits, torch.as_tensor(y)).backward()
    nhwc = lambda t: t.permute(0, 2, 3, 1)
    print("stem z", rel(net.stem.z, nhwc(outs["stem_z"])))
    for bi, b in enumerate(net.blocks):
        print(f"block{bi} z1 {rel(b.c1.z, nhwc(outs[f'block{bi}.z1'])):9.2e}  out {rel(b.c2.y, nhwc(outs[f'block{bi}'])):9.2e}")
    nb = len(net.blocks)
    print("head dx", rel(net.head.dx.view(net.blocks[-1].out_shape), nhwc(outs[f"block{nb - 1}"].grad)))
    for bi in range(nb - 1, 0, -1):
        print(f"d block{bi - 1} out", rel(net.dacts[bi], nhwc(outs[f"block{bi - 1}"].grad)))


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "fwd":
    forward_check()


def sums_check():
    """Fused BN-backward sums left by one forward+backward (no optimizer, so
    the accumulators survive) vs host sums from the model's own buffers."""
    from metisfl_amd.ops import nn as K
    rng = np.random.default_rng(0)
    B = 32
    x = rng.standard_normal((B, 32, 32, 3)).astype(np.float32)
    y = rng.integers(0, 10, B)
    net = ResNet18(batch_size=B, device="cuda", optimizer=OptimizerSpec("vanilla_sgd", 0.0), seed=4)
    ds = net.make_dataset(x, y, shuffle=False)
    st = net.state
    st.grad32.zero_()
    net.ws.bn_acc.zero_()
    K.gather_batch(ds.x, ds.y, ds.perm, st.step, ds.steps_per_epoch, net.B, net.xb, net.yb)
    out = net.forward(net.xb, train=True)
    dlast = net.head.forward_backward(out, net.yb, net.stats, train=True)
    net.backward(dlast)
    net.ws.join()
    torch.cuda.synchronize()
    layers = [(b.c2, net.dacts[i + 1]) for i, b in enumerate(net.blocks[:-1])]
    layers.append((net.blocks[-1].c2, dlast.view(net.blocks[-1].out_shape)))
    for i, b in enumerate(net.blocks):
        layers.append((b.c1, b.da))
    for c, dy in layers:
        C = c.shp.Co
        acc = net.ws.acc(c.acc_b).view(-1, 2 * C).sum(0).cpu()
        ref = torch.zeros(2 * C, dtype=torch.float64)
        K._bnb_sums_cpu(dy.cpu(), K.BnBwdTarget(c.z.cpu(), c.y.cpu() if c.relu else None,
                                                 c.mean.cpu(), c.invstd.cpu(), ref))
        print(f"{c.name:18s} reps {acc.numel() // (2 * C) if False else net.ws.acc(c.acc_b).numel() // (2 * C)} "
              f"sum dy {rel(acc[:C], ref[:C]):9.2e}  sum dy*xh {rel(acc[C:], ref[C:]):9.2e}")


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "sums":
    sums_check()


def bwd_check():
    """Per-conv dz (grad of conv output) and per-block da (grad of conv2's
    input) of one forward+backward vs the fp64 oracle and torch fp32."""
    from metisfl_amd.ops import nn as K
    from tests.torch_resnet_ref import TorchResNet18
    rng = np.random.default_rng(0)
    B = 32
    x = rng.standard_normal((B, 32, 32, 3)).astype(np.float32)
    y = rng.integers(0, 10, B)
    net = ResNet18(batch_size=B, device="cuda", optimizer=OptimizerSpec("vanilla_sgd", 0.0), seed=4)
    values = net.state.to_numpy()
    ds = net.make_dataset(x, y, shuffle=False)
    st = net.state
    st.grad32.zero_()
    net.ws.bn_acc.zero_()
    K.gather_batch(ds.x, ds.y, ds.perm, st.step, ds.steps_per_epoch, net.B, net.xb, net.yb)
    out = net.forward(net.xb, train=True)
    dlast = net.head.forward_backward(out, net.yb, net.stats, train=True)
    net.backward(dlast)
    net.ws.join()
    torch.cuda.synchronize()
    grads = {}
    for dt in (torch.float64, torch.float32):
        m = TorchResNet18().to(dt)
        m.load_from(values)
        m.train()
        outs = {}
        for bi, b in enumerate(m.blocks):
            b.conv1.register_forward_hook(lambda mod, i, o, bi=bi: outs.__setitem__(f"{bi}.z1", o))
            b.conv2.register_forward_hook(lambda mod, i, o, bi=bi: outs.__setitem__(f"{bi}.z2", o))
            b.conv2.register_forward_hook(lambda mod, i, o, bi=bi: outs.__setitem__(f"{bi}.a", i[0]))
        xx = F.pad(torch.as_tensor(x), (0, 5)).to(dt).permute(0, 3, 1, 2)
        logits = m(xx)
        for o in outs.values():
            o.retain_grad()
        F.cross_entropy(logits, torch.as_tensor(y)).backward()
        grads[dt] = {k: v.grad.permute(0, 2, 3, 1) for k, v in outs.items()}
    g64, g32 = grads[torch.float64], grads[torch.float32]
    for bi in range(len(net.blocks) - 1, -1, -1):
        b = net.blocks[bi]
        for k, ours in ((f"{bi}.z2", b.c2.dz), (f"{bi}.a", b.da), (f"{bi}.z1", b.c1.dz)):
            print(f"{k:6s} ours {rel(ours, g64[k]):9.2e}  torch32 {rel(g32[k], g64[k]):9.2e}")


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "bwd":
    bwd_check()


def flip_check():
    """ReLU mask disagreements between the executor's forward and the fp64
    oracle's (elements whose sign differs: the backward masks then differ)."""
    from tests.torch_resnet_ref import TorchResNet18
    rng = np.random.default_rng(0)
    B = 32
    x = rng.standard_normal((B, 32, 32, 3)).astype(np.float32)
    y = rng.integers(0, 10, B)
    net = ResNet18(batch_size=B, device="cuda", optimizer=OptimizerSpec("vanilla_sgd", 0.0), seed=4)
    values = net.state.to_numpy()
    ds = net.make_dataset(x, y, shuffle=False)
    net.zero_grad_in_optimizer = False
    net._train_body(ds)
    torch.cuda.synchronize()
    m = TorchResNet18().double()
    m.load_from(values)
    m.train()
    outs = {}
    for bi, b in enumerate(m.blocks):
        b.register_forward_hook(lambda mod, i, o, bi=bi: outs.__setitem__(f"{bi}.out", o))
        b.conv2.register_forward_hook(lambda mod, i, o, bi=bi: outs.__setitem__(f"{bi}.a", i[0]))
    m(F.pad(torch.as_tensor(x), (0, 5)).double().permute(0, 3, 1, 2).contiguous())
    for bi, b in enumerate(net.blocks):
        for k, ours in ((f"{bi}.a", b.c1.y), (f"{bi}.out", b.c2.y)):
            r = outs[k].permute(0, 2, 3, 1)
            o = ours.double().cpu()
            flips = ((o > 0) != (r > 0))
            print(f"{k:6s} flips {int(flips.sum()):4d}  |y| at flips {r[flips].abs().max().item() if flips.any() else 0:9.2e}"
                  f"  min |y|>0 {r[r > 0].min().item():9.2e}")


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "flips":
    flip_check()
