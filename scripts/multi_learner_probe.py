"""Throughput of G co-resident ResNet-18 learners on one GPU: each learner
keeps its own model, workspace and captured K-update graph; the graphs are
replayed on G streams (concurrent HIP queues) instead of back to back.

python scripts/multi_learner_probe.py --groups 1 2 4 8 --updates 256
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for _i, _a in enumerate(sys.argv):  # before HIP initialises
    if _a == "--hw-queues":
        os.environ["GPU_MAX_HW_QUEUES"] = sys.argv[_i + 1]

import torch  # noqa: E402

from metisfl_amd.models.resnet import ResNet18  # noqa: E402
from metisfl_amd.ops.optim import OptimizerSpec  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--groups", type=int, nargs="+", default=[1, 2, 4, 8])
    ap.add_argument("--updates", type=int, default=256, help="per learner")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--dtype", default="fp32", choices=("fp32", "bf16"))
    ap.add_argument("--serial", action="store_true", help="one stream (baseline)")
    ap.add_argument("--hw-queues", type=int, default=0)
    ap.add_argument("--stagger-us", type=float, default=0.0,
                    help="delay stream g's first launch by (g %% 4) x this many microseconds (phase offset)")
    ap.add_argument("--cu-mask", choices=("none", "contig", "interleave"), default="none",
                    help="confine learner g's stream to 256/G CUs (hipExtStreamCreateWithCUMask): a contiguous "
                         "CU-id range, or CU ids with id %% G == g")
    ap.add_argument("--pair-ring", type=int, default=-1,
                    help="conv32 paired-launch LDS ring stages (-1: what CoLocatedLearners selects for the group)")
    ap.add_argument("--conv-products", default=None, choices=("bf16x3", "exact"))
    ap.add_argument("--prio-split", action="store_true", help="alternate learner stream priorities")
    a = ap.parse_args()
    gmax = max(a.groups)
    from metisfl_amd.models.colocated import CoLocatedLearners, configure_regime
    configure_regime(gmax)  # the production regime for gmax co-located learners (plans, halo-conv stages)
    ring = a.pair_ring if a.pair_ring >= 0 else (int(CoLocatedLearners.pair_ring or 0)
                                                 if gmax >= CoLocatedLearners.pair_ring_min_learners else 0)
    if ring:
        CoLocatedLearners._set_pair_ring(ring)
    print(f"pair ring {ring or 'build default'}, conv products {a.conv_products or 'default'}", flush=True)
    nets, dss = [], []
    gen = torch.Generator(device="cuda").manual_seed(0)
    for i in range(gmax):
        net = ResNet18(batch_size=a.batch, device="cuda", seed=7 + i, dtype=a.dtype,
                       conv_products=a.conv_products,
                       optimizer=OptimizerSpec("momentum_sgd", 0.005, momentum=0.75))
        ns = max(1024, 16 * a.batch)  # >= 2 x K steps per epoch: the K-update graph gets captured
        x = torch.randn((ns, 32, 32, 3), generator=gen, device="cuda")
        y = torch.randint(0, 10, (ns,), generator=gen, device="cuda")
        nets.append(net)
        dss.append(net.make_dataset(x, y, seed=i))
    for net, ds in zip(nets, dss):  # capture (1-step and K-step graphs)
        net.train_steps(ds, 16)
    torch.cuda.synchronize()
    if a.prio_split:
        # alternate stream priorities: HIP keeps hardware queues per priority,
        # so the two halves do not share in-order queues
        lo, hi = torch.cuda.Stream.priority_range()
        print(f"stream priorities {lo} / {hi} alternating", flush=True)
        streams = [torch.cuda.Stream(priority=hi if g % 2 else lo) for g in range(gmax)]
    else:
        streams = [torch.cuda.Stream() for _ in range(gmax)]
    masked = {}
    if a.cu_mask != "none":
        import ctypes
        hip = ctypes.CDLL("libamdhip64.so")
        ncu = torch.cuda.get_device_properties(0).multi_processor_count
        for G in a.groups:
            per = ncu // G
            lst = []
            for g in range(G):
                bits = [0] * ((ncu + 31) // 32)
                for cu in range(ncu):
                    mine = (cu // per == g) if a.cu_mask == "contig" else (cu % G == g)
                    if mine:
                        bits[cu // 32] |= 1 << (cu % 32)
                arr = (ctypes.c_uint32 * len(bits))(*bits)
                h = ctypes.c_void_p()
                err = hip.hipExtStreamCreateWithCUMask(ctypes.byref(h), ctypes.c_uint32(len(bits)), arr)
                assert err == 0, f"hipExtStreamCreateWithCUMask: {err}"
                lst.append(torch.cuda.ExternalStream(h.value))
            masked[G] = lst
        print(f"CU-masked streams ({a.cu_mask}), {ncu} CUs", flush=True)
    K = nets[0].graph_steps
    for G in a.groups:
        for mode in (["serial"] if a.serial else []) + ["streams"]:
            reps = a.updates // K
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            if mode == "streams" and a.stagger_us > 0:
                cyc = int(a.stagger_us * 2100)  # ~2.1 GHz shader clock
                for g in range(G):
                    if g % 4:
                        with torch.cuda.stream(masked[G][g] if masked else streams[g]):
                            torch.cuda._sleep(cyc * (g % 4))
            for r in range(reps):
                for g in range(G):
                    if mode == "streams":
                        with torch.cuda.stream(masked[G][g] if masked else streams[g]):
                            nets[g]._train_graph_k.replay()
                    else:
                        nets[g]._train_graph_k.replay()
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            upd = reps * K * G
            print(f"G={G} {mode}: {dt * 1e3 / (reps * K):.3f} ms per {G}-learner step, "
                  f"{dt * 1e3 / upd:.4f} ms per update, {upd * a.batch / dt:.0f} samples/s", flush=True)


if __name__ == "__main__":
    main()
