"""Kernel statistics from a rocprofv3 SQLite (rocpd) database:
    python scripts/rocpd_stats.py <results.db> [--steps N]
prints per-kernel calls / total ms / mean us / share (and per-step numbers
when --steps is given), like rocprofv3 --stats' kernel_stats.csv."""
import argparse
import sqlite3
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--steps", type=int, default=0)
    ap.add_argument("--width", type=int, default=74)
    a = ap.parse_args()
    con = sqlite3.connect(a.db)
    cur = con.cursor()
    rows = cur.execute("""select s.kernel_name, d.start, d.end from rocpd_kernel_dispatch d
                          join rocpd_info_kernel_symbol s on d.kernel_id = s.id""").fetchall()
    agg = defaultdict(lambda: [0, 0])
    for name, st, en in rows:
        agg[name][0] += 1
        agg[name][1] += en - st
    tot = sum(v[1] for v in agg.values())
    print(f"{'kernel':{a.width}s} {'calls':>7s} {'ms':>9s} {'avg_us':>8s} {'%':>6s}")
    for name, (n, ns) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print(f"{name[:a.width]:{a.width}s} {n:7d} {ns / 1e6:9.2f} {ns / n / 1e3:8.2f} {100 * ns / tot:6.1f}")
    calls = sum(v[0] for v in agg.values())
    line = f"total {tot / 1e6:.1f} ms, {calls} launches"
    if a.steps:
        line += f"; per step: {tot / 1e6 / a.steps:.3f} ms, {calls / a.steps:.1f} launches"
    print(line)


if __name__ == "__main__":
    main()
