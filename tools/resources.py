#!/usr/bin/env python3
"""Per-kernel register / occupancy table from `make -C dna-ldpc-codes_amd resources`
(-Rpass-analysis=kernel-resource-usage remarks), demangled names shortened.

    make -s -C dna-ldpc-codes_amd resources 2>&1 | python tools/resources.py [filter]
"""
import re
import subprocess
import sys

flt = sys.argv[1] if len(sys.argv) > 1 else ""
rows, cur = [], None
for ln in sys.stdin:
    m = re.search(r"Function Name: (\S+)", ln)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    m = re.search(r"(VGPRs|AGPRs|TotalSGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]): (\d+)", ln)
    if m and cur is not None:
        cur[m.group(1).split()[0]] = int(m.group(2))
names = subprocess.run(["c++filt"], input="\n".join(r["name"] for r in rows), capture_output=True, text=True).stdout.split("\n")
for r, n in zip(rows, names):
    n = re.sub(r"\(.*", "", n).replace("ldpc::dev::", "").replace("void ", "")
    if flt in n:
        print(f"{n:60s} VGPR {r.get('VGPRs', 0):4d} AGPR {r.get('AGPRs', 0):3d} SGPR {r.get('TotalSGPRs', 0):4d} "
              f"scratch {r.get('ScratchSize', 0):4d} occ {r.get('Occupancy', 0)}")
