"""GPU diagnostic: ResNet-18 (full width, batch 32) GPU kernels vs the CPU
reference ops, layer by layer, after one eager step; then determinism of
eager vs eager vs graph over a few steps."""
import torch

from metisfl_amd.models.layers import BasicBlock, ConvBN
from metisfl_amd.models.resnet import ResNet18
from metisfl_amd.ops.optim import OptimizerSpec


def make(dev, lr=0.005):
    return ResNet18(batch_size=32, device=dev,
                    optimizer=OptimizerSpec("momentum_sgd", learning_rate=lr, momentum=0.75), seed=3)


def convbns(net):
    out = [net.stem]
    for b in net.blocks:
        out += b.sublayers()
    return out


def cos(a, b):
    a, b = a.double().flatten(), b.double().flatten()
    return float((a @ b) / (a.norm() * b.norm() + 1e-30))


def main():
    g = torch.Generator().manual_seed(0)
    x = torch.randn(256, 32, 32, 3, generator=g)
    y = torch.randint(0, 10, (256,), generator=g)
    cpu, gpu = make("cpu", 0.0), make("cuda", 0.0)
    cpu.zero_grad_in_optimizer = gpu.zero_grad_in_optimizer = False
    dc = cpu.make_dataset(x, y, shuffle=False)
    dg = gpu.make_dataset(x, y, shuffle=False)
    cpu._train_body(dc)
    gpu._train_body(dg)
    torch.cuda.synchronize()
    for lc, lg in zip(convbns(cpu), convbns(gpu)):
        msg = [lc.name, str(lc.shp.args()), f"P{lc.P}"]
        for attr in ("z", "y", "dz", "mean", "invstd"):
            a, b = getattr(lc, attr), getattr(lg, attr).cpu()
            fin = bool(torch.isfinite(b.float()).all())
            msg.append(f"{attr}:{cos(a.float(), b.float()):.4f}{'' if fin else '(NONFINITE)'}")
        a, b = lc.dw, lg.dw.cpu()
        msg.append(f"dw:{cos(a, b):.4f}{'' if torch.isfinite(b).all() else '(NONFINITE)'}")
        print(" ".join(msg))
    print("head dx", cos(cpu.head.dx.float(), gpu.head.dx.float().cpu()))
    print("stats cpu", cpu.stats.tolist(), "gpu", gpu.stats.cpu().tolist())

    nets = [make("cuda") for _ in range(3)]
    ds = [n.make_dataset(x, y, shuffle=False) for n in nets]
    steps = 8
    for i in range(steps):
        nets[0]._train_body(ds[0])
        nets[1]._train_body(ds[1])
        torch.cuda.synchronize()
        print("step", i, "norm", nets[0].state.model32.norm().item(),
              "finite", bool(torch.isfinite(nets[0].state.model32).all()))
    nets[2].train_steps(ds[2], steps)
    torch.cuda.synchronize()
    a, b, c = (n.state.model32 for n in nets)
    print("eager-eager max diff", (a - b).abs().max().item())
    print("eager-graph max diff", (a - c).abs().max().item())


if __name__ == "__main__":
    main()
