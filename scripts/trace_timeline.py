"""Diagnostics: prints the kernels of the last N launches of a rocprofv3 kernel trace as a
timeline (start / end relative to the first, duration, name) -- for multi-stream steps."""
import csv
import glob
import sys

f = sorted(glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True))[0]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 20
rows = list(csv.DictReader(open(f)))
ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Queue_Id", ""), r["Kernel_Name"]) for r in rows)
ks = ks[-n:]
t0 = ks[0][0]
for s, e, qid, name in ks:
    print(f"{(s - t0) / 1e3:9.1f} {(e - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f}  q{qid:>3}  {name[:90]}")
