"""Per-step totals of a whole-step PMC run (scripts/pmc_step.sh): sums every
counter over the dispatches of the timed steps and divides by the number of
steps; per kernel class too.  python scripts/pmc_step_summary.py gpurun_out/pmc_step 40"""
import collections
import csv
import glob
import sys

root, steps = sys.argv[1], float(sys.argv[2])
tot = collections.Counter()
per = collections.defaultdict(collections.Counter)
for f in glob.glob(f"{root}/p*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "")
        short = name.split("(")[0].split("<")[0].split("::")[-1][:40]
        v = float(r["Counter_Value"])
        tot[r["Counter_Name"]] += v
        per[short][r["Counter_Name"]] += v
print("per step:")
for k in sorted(tot):
    v = tot[k] / steps
    unit = " KB" if k in ("FETCH_SIZE", "WRITE_SIZE") else ""
    print(f"  {k:22s} {v:16.1f}{unit}")
h, m = tot.get("TCC_HIT_sum", 0), tot.get("TCC_MISS_sum", 0)
if h + m:
    print(f"  L2 hit rate {h / (h + m):.3f}")
print("per kernel class (per step): FETCH MB, WRITE MB, MFMA, VALU, LDS")
rows = []
for k, c in per.items():
    rows.append((c.get("FETCH_SIZE", 0) / 1024 / steps, c.get("WRITE_SIZE", 0) / 1024 / steps,
                 c.get("SQ_INSTS_MFMA", 0) / steps, c.get("SQ_INSTS_VALU", 0) / steps,
                 c.get("SQ_INSTS_LDS", 0) / steps, k))
for r in sorted(rows, reverse=True)[:20]:
    print(f"  {r[5]:40s} {r[0]:9.1f} {r[1]:9.1f} {r[2]:12.0f} {r[3]:12.0f} {r[4]:12.0f}")
