"""Diagnostics: one step's anatomy from a rocprofv3 --kernel-trace CSV of
scripts/dp_fork_probe.py: the last 16 steps (a step starts at each encoder launch), per step
the kernels in start order with their queue (stream) id, start offset, duration and the idle
time of the device (no kernel running on any queue) before each; then the median step
period and the median per-position start / duration over those steps."""
import csv
import statistics as st
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
first = sys.argv[2] if len(sys.argv) > 2 else "enc_latent"   # a substring of the step's first kernel
nsteps = int(sys.argv[3]) if len(sys.argv) > 3 else 16
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
name = lambda r: r["Kernel_Name"].split("(")[0].replace("void ", "").replace("vaeb::", "").replace("bf::", "")[:60]
qid = lambda r: r.get("Queue_Id") or r.get("Stream_Id") or "?"
starts = [i for i, r in enumerate(rows) if first in r["Kernel_Name"]]
steps = [rows[a:b] for a, b in zip(starts[-nsteps - 1:-1], starts[-nsteps:])]
per = defaultdict(list)
periods = []
for si, s in enumerate(steps):
    t0 = int(s[0]["Start_Timestamp"])
    periods.append((int(steps[si + 1][0]["Start_Timestamp"]) - t0) / 1e3 if si + 1 < len(steps) else None)
    busy_end = t0
    for k, r in enumerate(s):
        a, b = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        idle = max(0, a - busy_end) / 1e3
        busy_end = max(busy_end, b)
        per[(k, name(r), qid(r))].append(((a - t0) / 1e3, (b - a) / 1e3, idle))
print(f"{len(steps)} steps; median period {st.median([p for p in periods if p]):.2f} us")
print(f"{'#':>2} {'kernel':60s} {'queue':>6} {'start':>7} {'dur':>6} {'idle before':>11}")
for (k, n, q), v in sorted(per.items()):
    print(f"{k:2d} {n:60s} {q:>6} {st.median(x[0] for x in v):7.2f} {st.median(x[1] for x in v):6.2f} "
          f"{st.median(x[2] for x in v):11.2f}")
