#!/usr/bin/env python3
"""Per-kernel VGPRs / scratch / occupancy / LDS of libtcmp's own kernels (hipcc
-Rpass-analysis=kernel-resource-usage), one line each.  usage: python tools/resource.py [filter]"""
import re
import subprocess
import sys

src = "torque_constrained_motion_planning_amd/csrc"
out = subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-fPIC",
                      "-shared", "-w", "-Rpass-analysis=kernel-resource-usage", "-o",
                      "/tmp/tcmp_res.so", "tcmp_engine.hip"], cwd=src, capture_output=True,
                     text=True).stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        name = subprocess.run(["c++filt", m.group(1)], capture_output=True, text=True).stdout.strip()
        cur = {"name": name.replace("(anonymous namespace)::", "")}
        rows.append(cur)
        continue
    for key, pat in (("vgpr", r" VGPRs: (\d+)"), ("scratch", r"ScratchSize \[bytes/lane\]: (\d+)"),
                     ("occ", r"Occupancy \[waves/SIMD\]: (\d+)"), ("lds", r"LDS Size \[bytes/block\]: (\d+)"),
                     ("sspill", r"SGPRs Spill: (\d+)"), ("vspill", r"VGPRs Spill: (\d+)")):
        m = re.search(pat, line)
        if m and cur is not None:
            cur[key] = int(m.group(1))
flt = sys.argv[1] if len(sys.argv) > 1 else ""
for r in rows:
    if "rocprim" in r["name"] or flt not in r["name"]:
        continue
    print("vgpr %3s scratch %4s occ %s lds %6s sspill %3s vspill %3s  %s" % (
        r.get("vgpr"), r.get("scratch"), r.get("occ"), r.get("lds"), r.get("sspill"),
        r.get("vspill"), r["name"][:90]))
