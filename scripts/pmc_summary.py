#!/usr/bin/env python3
"""Fold rocprofv3 `--pmc` counter CSVs into per-launch averages per kernel.

Usage: pmc_summary.py OUT.json DIR [DIR ...]
Each DIR is one rocprofv3 `-d` output directory of a separate `--pmc` pass; every
`*counter_collection.csv` under it is read.  Values are summed per (dispatch, counter)
and averaged over the dispatches of each kernel.  FETCH_SIZE / WRITE_SIZE stay in the
counters' KB unit; `FETCH_SIZE_corrected` doubles FETCH_SIZE, because on gfx950 it
tallies 128-B wide reads at 64 B (MI355X_MICROARCH.md §HBM); `hbm_bytes_per_launch` =
(2 x FETCH_SIZE + WRITE_SIZE) x 1024.
"""
import collections
import csv
import glob
import json
import os
import sys


def fold(dirs):
    per = collections.defaultdict(lambda: collections.defaultdict(float))   # (kernel, dispatch) -> counter -> v
    for d in dirs:
        for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(path) as f:
                for row in csv.DictReader(f):
                    key = (row["Kernel_Name"], d + ":" + row.get("Dispatch_Id", row.get("Correlation_Id", "")))
                    per[key][row["Counter_Name"]] += float(row["Counter_Value"])
    out = collections.defaultdict(lambda: collections.defaultdict(list))
    for (kern, _), cs in per.items():
        for c, v in cs.items():
            out[kern][c].append(v)
    res = {}
    for kern, cs in out.items():
        r = {c: sum(v) / len(v) for c, v in cs.items()}
        r["launches"] = max(len(v) for v in cs.values())
        if "FETCH_SIZE" in r:
            r["FETCH_SIZE_corrected"] = 2.0 * r["FETCH_SIZE"]
        if "FETCH_SIZE" in r and "WRITE_SIZE" in r:
            r["hbm_bytes_per_launch"] = (2.0 * r["FETCH_SIZE"] + r["WRITE_SIZE"]) * 1024.0
        res[kern] = r
    return res


def main():
    if len(sys.argv) < 3:
        print(__doc__)
        sys.exit(2)
    res = fold(sys.argv[2:])
    with open(sys.argv[1], "w") as f:
        json.dump(res, f, indent=1, sort_keys=True)
    for k, v in sorted(res.items()):
        print(k[:90], {c: round(x, 1) for c, x in v.items() if c in ("FETCH_SIZE", "WRITE_SIZE", "launches")})


if __name__ == "__main__":
    main()
