"""Does ONE hipGraph holding two learners' independent K-update chains run
them concurrently on one stream (one in-order hardware queue)?  Compares, for
G co-located learners: G streams of per-learner K-update graphs (production)
against G/2 streams each replaying a graph with two learners' chains forked
on two capture side streams and joined at the end.

python scripts/pair_graph_probe.py --groups 8 --updates 256
"""
import argparse
import gc
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from metisfl_amd.models.colocated import configure_regime  # noqa: E402
from metisfl_amd.models.resnet import ResNet18  # noqa: E402
from metisfl_amd.ops.optim import OptimizerSpec  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--groups", type=int, default=8)
    ap.add_argument("--updates", type=int, default=256)
    a = ap.parse_args()
    G = a.groups
    configure_regime(G)
    from metisfl_amd.models.colocated import CoLocatedLearners
    CoLocatedLearners.apply_kernel_regime(G)
    nets, dss = [], []
    gen = torch.Generator(device="cuda").manual_seed(0)
    for i in range(G):
        net = ResNet18(batch_size=32, device="cuda", seed=7 + i, optimizer=OptimizerSpec("momentum_sgd", 0.005, 0.75))
        x = torch.randn((1024, 32, 32, 3), generator=gen, device="cuda")
        y = torch.randint(0, 10, (1024,), generator=gen, device="cuda")
        nets.append(net)
        dss.append(net.make_dataset(x, y, seed=i))
    for net, ds in zip(nets, dss):
        net.train_steps(ds, 16)  # per-learner graphs (1- and K-update)
    torch.cuda.synchronize()
    K = nets[0].graph_steps

    # pair graphs: learners 2p and 2p+1, K updates each, on two forked capture streams
    pair_graphs = []
    for p in range(G // 2):
        A, B = nets[2 * p], nets[2 * p + 1]
        da, db = dss[2 * p], dss[2 * p + 1]
        cap = torch.cuda.Stream()
        sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
        g = torch.cuda.CUDAGraph()
        gc.collect()
        with torch.cuda.graph(g, stream=cap, capture_error_mode="thread_local"):
            sa.wait_stream(cap)
            sb.wait_stream(cap)
            with torch.cuda.stream(sa):
                for _ in range(K):
                    A._train_body(da)
            with torch.cuda.stream(sb):
                for _ in range(K):
                    B._train_body(db)
            cap.wait_stream(sa)
            cap.wait_stream(sb)
        pair_graphs.append(g)
    torch.cuda.synchronize()

    reps = a.updates // K
    for mode in ("streams", "pairs", "streams", "pairs"):
        streams = [torch.cuda.Stream() for _ in range(G if mode == "streams" else G // 2)]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            if mode == "streams":
                for g_, s in enumerate(streams):
                    with torch.cuda.stream(s):
                        nets[g_]._train_graph_k.replay()
            else:
                for p, s in enumerate(streams):
                    with torch.cuda.stream(s):
                        pair_graphs[p].replay()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print(f"G={G} {mode}: {dt * 1e3 / (reps * K * G):.4f} ms per update", flush=True)


if __name__ == "__main__":
    main()
