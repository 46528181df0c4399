"""Diagnostics: per-kernel durations and the idle gap before each kernel, from a rocprofv3
--kernel-trace CSV (the last `n` dispatches), grouped by kernel name."""
import csv
import sys
from collections import defaultdict

path, n = sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 256
rows = list(csv.DictReader(open(path)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
rows = rows[-n:]
dur, gap = defaultdict(list), defaultdict(list)
prev_end = None
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    k = r["Kernel_Name"][:60]
    dur[k].append((e - s) / 1e3)
    if prev_end is not None:
        gap[k].append((s - prev_end) / 1e3)
    prev_end = max(prev_end or 0, e)
span = (int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])) / 1e3
print(f"{len(rows)} dispatches over {span:.1f} us")
for k in dur:
    d, g = dur[k], gap.get(k, [0])
    print(f"{len(d):5d} x {k:60s} dur {sum(d) / len(d):7.2f} us  gap before {sum(g) / len(g):7.2f} us (max {max(g):6.2f})")
