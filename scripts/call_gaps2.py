"""Reads a rocprofv3 kernel_trace.csv of scripts/call_trace.py (update_many(20) calls) and prints,
for the last three calls, every kernel's start relative to the call's first kernel and the idle gap
before it (calls are split at idle gaps > 50 us)."""
import csv
import glob
import sys

f = sorted(glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True))[0]
rows = list(csv.DictReader(open(f)))
ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:40]) for r in rows)
calls, cur, prev = [], [], None
for k in ks:
    if prev is not None and k[0] - prev > 50_000:
        calls.append(cur)
        cur = []
    cur.append(k)
    prev = max(prev or 0, k[1])
calls.append(cur)
for c in calls[-3:]:
    t0 = c[0][0]
    prev_end = None
    tot_gap = 0.0
    print(f"---- call: {len(c)} kernels, span {(max(e for _, e, _ in c) - t0) / 1e3:.1f} us")
    for i, (s, e, name) in enumerate(c):
        gap = (s - prev_end) / 1e3 if prev_end else 0.0
        tot_gap += max(gap, 0.0)
        if i < 8 or gap > 2.0:
            print(f"  #{i:3d} t={(s - t0) / 1e3:8.1f} us  dur={(e - s) / 1e3:6.1f}  gap={gap:6.1f}  {name}")
        prev_end = e
    print(f"  sum of gaps {tot_gap:.1f} us")
