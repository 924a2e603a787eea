#!/usr/bin/env python3
"""Average launch durations of the planner's kernels in a rocprofv3 kernel trace, split into the
launches that overlapped work of another engine (pipelined steps: another queue busy during the
launch) and those that ran alone (bench.py's one-at-a-time kernel-timing pass), so that the bench
line's event-timed `avg_launch_ms` can be checked against the trace of the same command.
Launches of a few hundred threads (the bench's scene setup) are left out, as in bench.py.

usage: python tools/trace_split.py RUN_kernel_trace.csv [kernel ...]
Kernels are named as tools/pmc_summary.py names them (the fused-rounds scan is
`k_nearest_wave32@fleet`).
"""
import csv
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import short  # noqa: E402


def main():
    path = sys.argv[1]
    want = sys.argv[2:] or ["k_edges", "k_fl_edges", "k_nearest_wave32", "k_nearest_wave32@fleet"]
    rows = list(csv.DictReader(open(path)))
    # every dispatch as (start, end, queue): a launch "overlapped" if any dispatch of another
    # queue (another engine's stream) ran during it
    allx = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"]) for r in rows)
    starts = [x[0] for x in allx]

    def overlapped(a, b, q):
        import bisect
        i = bisect.bisect_left(starts, b)
        return any(x < b and a < y and qq != q for x, y, qq in allx[max(0, i - 4000):i])

    out = {}
    for k in want:
        ks = [r for r in rows if short(r["Kernel_Name"]) == k]
        if not ks:
            continue
        big = max(int(r["Grid_Size_X"]) for r in ks)
        ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"]) for r in ks
              if int(r["Grid_Size_X"]) * 8 >= big]
        alone, over = [], []
        for a, b, q in ks:
            (over if overlapped(a, b, q) else alone).append((b - a) * 1e-6)
        out[k] = {"launches": len(ks),
                  "alone": {"n": len(alone), "avg_ms": sum(alone) / len(alone) if alone else None},
                  "overlapped": {"n": len(over), "avg_ms": sum(over) / len(over) if over else None},
                  "all_avg_ms": sum(alone + over) / len(ks)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
