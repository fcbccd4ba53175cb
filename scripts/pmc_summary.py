"""Per-kernel averages of rocprofv3 --pmc counter_collection.csv files
(several passes merged by dispatch id): python scripts/pmc_summary.py a.csv [b.csv ...] [--filter conv32]"""
import collections
import csv
import sys

files = [a for a in sys.argv[1:] if not a.startswith("--")]
flt = next((a.split("=", 1)[1] for a in sys.argv[1:] if a.startswith("--filter=")), "")
per = collections.defaultdict(lambda: collections.defaultdict(list))
grid = {}
for f in files:
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        if flt and flt not in name:
            continue
        key = (name.replace("(anonymous namespace)::", "").split("(")[0][-60:], r["Grid_Size"])
        per[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
for (name, g), cs in sorted(per.items()):
    avg = {k: sum(v) / len(v) for k, v in cs.items()}
    waves = avg.get("SQ_WAVES", 0) or 1
    parts = [f"{name:60s} grid={g:>8s}"]
    for k in sorted(avg):
        v = avg[k]
        if k in ("SQ_WAVES", "GRBM_GUI_ACTIVE", "SQ_BUSY_CYCLES"):
            parts.append(f"{k.replace('SQ_', '')}={v:.0f}")
        else:
            parts.append(f"{k.replace('SQ_', '')}/w={v / waves:.0f}")
    print(" ".join(parts))
