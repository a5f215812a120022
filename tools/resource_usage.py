#!/usr/bin/env python3
"""Per-kernel register / occupancy table from hipcc -Rpass-analysis=kernel-resource-usage remarks.
usage: hipcc ... -Rpass-analysis=kernel-resource-usage -c x.hip 2>&1 | tools/resource_usage.py [filter]"""
import re
import subprocess
import sys

flt = sys.argv[1] if len(sys.argv) > 1 else ""
cur, rows = None, []
for line in sys.stdin:
    m = re.search(r"remark:\s+Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    m = re.search(r"remark:\s+(VGPRs|AGPRs|Occupancy \[waves/SIMD\]|VGPRs Spill|LDS Size \[bytes/block\]): (\d+)", line)
    if m and cur is not None:
        cur[m.group(1).split()[0] + ("_spill" if "Spill" in m.group(1) else "")] = int(m.group(2))
names = [r["name"] for r in rows]
try:
    dem = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True).stdout.split("\n")
except OSError:
    dem = names
for r, d in zip(rows, dem):
    if flt in d:
        print(f"v{r.get('VGPRs', 0):4d} a{r.get('AGPRs', 0):4d} spill{r.get('VGPRs_spill', 0):4d} occ{r.get('Occupancy', 0):2d}  {d[:150]}")
