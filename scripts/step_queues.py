"""Diagnostics: per-step kernel timeline of a config-5 graph replay from a rocprofv3 kernel trace
(steps start at the encoder GEMM followed by the heads launch): kernel, HW queue, start / end
offsets in us, and the idle gap before each launch on its queue."""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
name = lambda r: r["Kernel_Name"].split("(")[0].replace("void ", "").replace("vaeb::", "").replace("bf::", "").replace("hf::", "")[:52]
qid = lambda r: r.get("Queue_Id") or r.get("Stream_Id") or "?"
starts = [i for i, r in enumerate(rows[:-1]) if "EpiBiasAct" in r["Kernel_Name"] and "EpiHeadsLatent" in rows[i + 1]["Kernel_Name"]]
for a, b in list(zip(starts, starts[1:]))[5:7]:
    t0 = int(rows[a]["Start_Timestamp"])
    last = {}
    for r in rows[a:b]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        q = qid(r)
        gap = (s - last[q]) / 1e3 if q in last else 0.0
        last[q] = e
        print(f"{name(r):52s} q{q:>3} {(s - t0) / 1e3:8.2f} {(e - t0) / 1e3:8.2f} gap {gap:6.2f}")
    print("period", (int(rows[b]["Start_Timestamp"]) - t0) / 1e3)
