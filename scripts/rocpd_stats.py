"""Kernel statistics from a rocprofv3 rocpd database (ROCm 7 default
output): per kernel name calls / total / mean, grid, VGPRs, LDS, plus the
concurrency of the trace (sum of kernel time / union of busy time).

    python scripts/rocpd_stats.py <results.db> [--top 30] [--min-start-frac 0.3]
"""
import argparse
import re
import sqlite3


def short(name: str) -> str:
    name = name.replace("(anonymous namespace)::", "")
    name = re.sub(r"\((?!anonymous).*$", "", name)
    return name[:90]


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--min-start-frac", type=float, default=0.0,
                    help="skip the first fraction of the trace (warmup / capture)")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, start, end, duration, grid_x, grid_y, grid_z, workgroup_x, vgpr_count, "
                     "accum_vgpr_count, lds_size, queue_id from kernels order by start").fetchall()
    t0, t1 = rows[0][1], max(r[2] for r in rows)
    cut = t0 + a.min_start_frac * (t1 - t0)
    rows = [r for r in rows if r[1] >= cut]
    agg = {}
    for n, s, e, d, gx, gy, gz, wx, vg, ag, lds, q in rows:
        k = short(n)
        x = agg.setdefault(k, [0, 0, (gx // max(1, wx)) * gy * gz, wx, vg, ag, lds, set()])
        x[0] += 1
        x[1] += d
        x[7].add(q)
    tot = sum(x[1] for x in agg.values())
    # union of busy intervals
    busy, cur_s, cur_e = 0, None, None
    for _, s, e, *_ in rows:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    span = max(r[2] for r in rows) - rows[0][1]
    print(f"{len(rows)} launches, kernel time {tot / 1e6:.2f} ms, busy union {busy / 1e6:.2f} ms, "
          f"span {span / 1e6:.2f} ms, concurrency {tot / max(1, busy):.2f}")
    print(f"{'kernel':90s} {'calls':>7s} {'ms':>9s} {'avg_us':>8s} {'%':>5s} {'wgs':>6s} {'thr':>4s} "
          f"{'vgpr':>4s} {'agpr':>4s} {'lds':>6s} q")
    for k, x in sorted(agg.items(), key=lambda kv: -kv[1][1])[:a.top]:
        print(f"{k:90s} {x[0]:7d} {x[1] / 1e6:9.2f} {x[1] / x[0] / 1e3:8.2f} {100 * x[1] / tot:5.1f} "
              f"{x[2]:6d} {x[3]:4d} {x[4]:4d} {x[5]:4d} {x[6]:6d} {len(x[7])}")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
