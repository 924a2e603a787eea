#!/usr/bin/env python3
"""Sum rocprofv3 counter_collection.csv values per kernel over the pass dirs of pmc_passes.sh.
usage: python tools/pmc_report.py OUTDIR [kernel-substring ...]"""
import csv
import glob
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import short  # noqa: E402


def main():
    out = sys.argv[1]
    want = sys.argv[2:] or ["k_nearest_wave32", "k_edges"]
    tot = defaultdict(lambda: defaultdict(float))
    n = defaultdict(lambda: defaultdict(int))
    for f in glob.glob(os.path.join(out, "p*", "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            k = short(row["Kernel_Name"])
            if k in want:
                tot[k][row["Counter_Name"]] += float(row["Counter_Value"])
                n[k][row["Counter_Name"]] += 1
    for k in want:
        print(k)
        for c in sorted(tot[k]):
            print("  %-24s %16.4g  (dispatches %d)" % (c, tot[k][c], n[k][c]))


if __name__ == "__main__":
    main()
