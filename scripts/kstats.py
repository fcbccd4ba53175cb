"""Summarise a rocprofv3 kernel_stats.csv: top kernels, per-step totals."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
tot = sum(int(r["TotalDurationNs"]) for r in rows)
calls = sum(int(r["Calls"]) for r in rows)
print(f"{'kernel':72s} {'calls':>7s} {'ms':>8s} {'avg_us':>8s} {'%':>6s}")
for r in rows[: int(sys.argv[3]) if len(sys.argv) > 3 else 25]:
    print(f"{r['Name'][:72]:72s} {int(r['Calls']):7d} {int(r['TotalDurationNs'])/1e6:8.2f} "
          f"{float(r['AverageNs'])/1e3:8.2f} {float(r['Percentage']):6.1f}")
print(f"total {tot/1e6:.1f} ms, {calls} launches; per step: {tot/1e6/steps:.3f} ms, {calls/steps:.1f} launches")
