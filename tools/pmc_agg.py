#!/usr/bin/env python3
"""Per-kernel totals of rocprofv3 --pmc passes (counter_collection.csv), compact enough to copy
back from the GPU box: for each kernel (bare name; the fused scan k_nearest_wave32<.., true> is
`k_nearest_wave32@fleet`) and counter, the dispatch count, the summed counter value and the
summed traced duration -- over the planner's own launches only (grids at least 1/8 of the
kernel's largest: the bench's scene setup runs the same kernels on a few configurations).

usage: python tools/pmc_agg.py PASS_DIR [PASS_DIR ...] > out.json"""
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import short  # noqa: E402


def main():
    rows = {}
    for d in sys.argv[1:]:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(f) as fh:
                for r in csv.DictReader(fh):
                    k = short(r.get("Kernel_Name", ""))
                    s, e = float(r.get("Start_Timestamp", 0) or 0), float(r.get("End_Timestamp", 0) or 0)
                    rows.setdefault(k, []).append((r.get("Counter_Name"),
                                                   int(float(r.get("Grid_Size", 0) or 0)),
                                                   float(r.get("Counter_Value", 0) or 0),
                                                   (e - s) / 1e3 if e > s else 0.0))
    out = {}
    for k, rs in rows.items():
        big = max(g for _, g, _, _ in rs)
        agg = {}
        for c, g, v, us in rs:
            if g * 8 < big:
                continue
            a = agg.setdefault(c, {"dispatches": 0, "sum": 0.0, "dur_us": 0.0})
            a["dispatches"] += 1
            a["sum"] += v
            a["dur_us"] += us
        out[k] = agg
    json.dump(out, sys.stdout, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
