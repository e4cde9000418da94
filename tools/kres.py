#!/usr/bin/env python3
"""Per-kernel resource usage (VGPR/AGPR/occupancy/spills/LDS) of one HIP
source compiled for gfx950:  python tools/kres.py mpc-mmd_amd/csrc/k_betacem.hip"""
import re
import subprocess
import sys

cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-ffp-contract=off", "-c",
       sys.argv[1], "-o", "/tmp/kres.o", "-Rpass-analysis=kernel-resource-usage"]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    m = re.search(r"remark:\s+([A-Za-z ]+?)(?: \[[^]]*\])?: (\d+)", line)
    if m and cur is not None:
        cur[m.group(1).strip()] = m.group(2)
for r in rows:
    n = re.sub(r"^_ZN6mpcmmd12_GLOBAL__N_1\d+", "", r["name"])
    g = lambda k: r.get(k, "?")
    print(f"{n[:40]:40s} vgpr {g('VGPRs'):>4} agpr {g('AGPRs'):>4} occ {g('Occupancy'):>2} "
          f"sspill {g('SGPRs Spill'):>5} vspill {g('VGPRs Spill'):>4} lds {g('LDS Size')}")
