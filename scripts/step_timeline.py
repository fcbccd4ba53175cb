"""Per-launch timeline of the training step from a rocprofv3 kernel trace:
    python scripts/step_timeline.py <run_kernel_trace.csv> [--first gather_kernel]
Splits the dispatch stream into steps (each starts with the batch gather),
keeps the steps whose launch sequence is the most common one, and prints per
position the mean duration, the mean gap since the previous launch ended and
the kernel -- where a step's time goes layer by layer, and how much of it is
dispatch gaps."""
import argparse
import csv
import re
from collections import Counter


def short(name: str) -> str:
    m = re.search(r"(\w+_kernel)(I[^E]*E)?", name)
    base = m.group(1) if m else name[:40]
    tpl = re.findall(r"Li(\d+)E", name[:160])
    return base + ("<" + ",".join(tpl[:5]) + ">" if tpl else "")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--first", default="gather_kernel")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    steps, cur = [], None
    for r in rows:
        nm = r["Kernel_Name"]
        if a.first in nm:
            cur = []
            steps.append(cur)
        if cur is not None:
            cur.append((short(nm), int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    sig = Counter(tuple(k for k, _, _ in s) for s in steps)
    common, n = sig.most_common(1)[0]
    sel = [s for s in steps if tuple(k for k, _, _ in s) == common][1:]  # drop the first (cold)
    L = len(common)
    dur = [0.0] * L
    gap = [0.0] * L
    span = 0.0
    for s in sel:
        for i, (_, t0, t1) in enumerate(s):
            dur[i] += (t1 - t0) / 1e3
            if i:
                gap[i] += (t0 - s[i - 1][2]) / 1e3
        span += (s[-1][2] - s[0][1]) / 1e3
    k = max(1, len(sel))
    print(f"{len(sel)} steps of {L} launches (of {len(steps)} steps seen); mean span {span / k:.1f} us, "
          f"kernels {sum(dur) / k:.1f} us, gaps {sum(gap) / k:.1f} us")
    print(f"{'#':>3s} {'dur_us':>8s} {'gap_us':>7s}  kernel")
    for i in range(L):
        print(f"{i:3d} {dur[i] / k:8.2f} {gap[i] / k:7.2f}  {common[i]}")


if __name__ == "__main__":
    main()
