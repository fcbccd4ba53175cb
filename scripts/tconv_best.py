"""Best (config, splits) per shape and kind from tconv_check logs (co-located column)."""
import re
import sys

best = {}
for f in sys.argv[1:]:
    for ln in open(f):
        m = re.match(r"N=(\d+)\s+(\d+)x(\d+)\s+C=\s*(\d+) (wgrad|dgrad) cfg (\d+) splits\s+(\d+) \| 1-stream\s+([\d.]+) us.*"
                     r"8 on 4 streams\s+([\d.]+) us", ln)
        if not m:
            continue
        key = (int(m.group(4)), m.group(5))
        t1, tc = float(m.group(8)), float(m.group(9))
        if key not in best or tc < best[key][0]:
            best[key] = (tc, t1, f.split("/")[-1], int(m.group(6)), int(m.group(7)))
for k in sorted(best):
    tc, t1, f, cfg, sp = best[k]
    print(f"C={k[0]:4d} {k[1]}: conc {tc:6.2f} us (1-stream {t1:6.2f}) cfg {cfg} splits {sp} [{f}]")
