#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes (counter_collection.csv) into profiles/<tag>_pmc_hbm.json.

Usage: python tools/pmc_summary.py OUT.json NOTE PASS_DIR [PASS_DIR ...]
Each PASS_DIR is one `rocprofv3 --pmc <COUNTER> --kernel-trace -d PASS_DIR -o run
--output-format csv -- python3 bench.py ...` run (one TCC counter per pass: FETCH_SIZE and
WRITE_SIZE do not fit one pass on gfx950).  Kernel names are reduced to the bare function name
(template arguments and parameters stripped; the fleet scan k_nearest_wave32<.., true> is
`k_nearest_wave32@fleet`).  Values are per dispatch, in KiB as rocprofv3
reports them; bench.py applies the gfx950 correction (x2 on FETCH_SIZE) when it reads them.
"""
import csv
import glob
import json
import os
import re
import sys


def short(name):
    # the fused-rounds instantiation of the scan (k_nearest_wave32<UW, SW, true>) is its own
    # entry: its launches serve a whole fleet
    fleet = re.search(r"k_nearest_wave32<[^>]*, true>", name) is not None
    name = short_base(name)
    return name + "@fleet" if fleet else name


def short_base(name):
    name = name.replace("(anonymous namespace)::", "")
    name = re.sub(r"\(.*$", "", name)
    name = re.sub(r"<.*$", "", name)
    name = name.replace("void ", "").strip()
    return name.split("::")[-1]


def main():
    out, note, dirs = sys.argv[1], sys.argv[2], sys.argv[3:]
    disp = {}
    for d in dirs:
        files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
        for f in files:
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    k = short(row.get("Kernel_Name", ""))
                    start = float(row.get("Start_Timestamp", 0) or 0)
                    end = float(row.get("End_Timestamp", 0) or 0)
                    disp.setdefault(k, []).append({
                        "counter": row.get("Counter_Name"),
                        "grid": int(float(row.get("Grid_Size", 0) or 0)),
                        # the raw counter value (KiB for FETCH_SIZE / WRITE_SIZE)
                        "value_KiB": float(row.get("Counter_Value", 0) or 0),
                        "dur_us": (end - start) / 1e3 if end > start else None,
                    })
    json.dump({"note": note, "dispatches": disp}, open(out, "w"), indent=1)
    print("%s: %s" % (out, {k: len(v) for k, v in disp.items()}))


if __name__ == "__main__":
    main()
