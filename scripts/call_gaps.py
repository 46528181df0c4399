"""Reads a rocprofv3 kernel_trace.csv of scripts/call_trace.py and prints, for the last
calls, each kernel's start relative to the call's first kernel and the gap before it."""
import csv
import glob
import sys

f = sorted(glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True))[0]
rows = list(csv.DictReader(open(f)))
ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:40]) for r in rows)
# calls start with set_order_kernel
starts = [i for i, k in enumerate(ks) if "set_order" in k[2]]
for c in starts[-3:]:
    t0 = ks[c][0]
    prev_end = None
    print("---- call")
    for s, e, name in ks[c:c + 1 + 4 * 20 + 2]:
        gap = (s - prev_end) / 1e3 if prev_end else 0
        if gap > 2.5 or "set_order" in name or prev_end is None or "enc_latent" in name:
            print(f"  t={(s - t0) / 1e3:8.1f} us  dur={(e - s) / 1e3:6.1f}  gap={gap:6.1f}  {name}")
        prev_end = e
    print(f"  last end t={(prev_end - t0) / 1e3:.1f} us")
rt = sorted(glob.glob(sys.argv[1] + "/**/*hip_api_trace.csv", recursive=True))
if rt:
    rows = list(csv.DictReader(open(rt[0])))
    calls = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Function"]) for r in rows)
    last = [c for c in calls if c[2] in ("hipGraphLaunch", "hipStreamSynchronize", "hipLaunchKernel",
                                          "hipModuleLaunchKernel", "hipExtModuleLaunchKernel")][-12:]
    t0 = last[0][0]
    for s, e, fn in last:
        print(f"  api {fn:24s} t={(s - t0) / 1e3:8.1f} us dur={(e - s) / 1e3:7.1f}")
