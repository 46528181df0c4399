"""Diagnostics (round 6): per-kernel effective clock from one rocprofv3 run with --pmc
GRBM_GUI_ACTIVE SQ_BUSY_CYCLES and --kernel-trace: for each kernel, the mean GRBM_GUI_ACTIVE
per dispatch over the mean dispatch duration.  Usage: clock_per_kernel.py DIR"""
import collections
import csv
import glob
import sys

d = sys.argv[1]
cnt = collections.defaultdict(lambda: collections.defaultdict(float))
names = {}
for p in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(p)):
        key = r.get("Dispatch_Id") or r.get("Correlation_Id")
        cnt[key][r["Counter_Name"]] += float(r["Counter_Value"])
        names[key] = r["Kernel_Name"]
dur = {}
for p in glob.glob(d + "/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(p)):
        key = r.get("Dispatch_Id") or r.get("Correlation_Id")
        dur[key] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
agg = collections.defaultdict(lambda: [0, 0.0, 0.0, 0.0])
for k, c in cnt.items():
    if k not in dur or dur[k] <= 0:
        continue
    a = agg[names[k]]
    a[0] += 1
    a[1] += c.get("GRBM_GUI_ACTIVE", 0.0)
    a[2] += c.get("SQ_BUSY_CYCLES", 0.0)
    a[3] += dur[k]
for n, (m, g, s, t) in sorted(agg.items(), key=lambda kv: -kv[1][3]):
    if m < 3:
        continue
    print(f"{n[:90]:90s} n={m:4d} dur {t / m * 1e6:8.1f} us  GRBM {g / m:10.0f}  GRBM/dur {g / t / 1e9:5.2f} GHz-eq  SQ_BUSY/dur {s / t / 1e9:6.2f}")
