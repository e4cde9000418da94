#!/usr/bin/env python3
"""Per-kernel instruction statistics of a HIP source's gfx950 assembly:
global loads, vmcnt(0) waits (serialised loads show as one wait per load),
branches, DPP moves, fp64 / MFMA counts.
    python tools/isa_stats.py mpc-mmd_amd/csrc/k_betacem.hip [name-filter]"""
import re
import subprocess
import sys

src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-ffp-contract=off",
                "--cuda-device-only", "-S", src, "-o", "/tmp/isa_stats.s"], check=True, capture_output=True)
lines = open("/tmp/isa_stats.s").read().split("\n")
starts = [(i, l.split(":")[0]) for i, l in enumerate(lines) if re.match(r"^_Z\S+: ", l) and "k_" in l]
for i, name in starts:
    if flt not in name:
        continue
    body = []
    for l in lines[i + 1:]:
        if l.strip().startswith("s_endpgm") or l.startswith(".Lfunc_end"):
            break
        body.append(l.strip())
    ins = [l.split()[0] for l in body if l and not l.startswith((";", ".")) and not l.endswith(":")]
    c = lambda p: sum(1 for x in ins if x.startswith(p))
    short = re.sub(r"^_ZN6mpcmmd12_GLOBAL__N_1\d+", "", name)[:40]
    print(f"{short:40s} instrs {len(ins):6d} gload {c('global_load'):4d} vmcnt0 "
          f"{sum(1 for l in body if 'vmcnt(0)' in l):4d} branch {c('s_cbranch'):4d} dpp {c('v_mov_b32_dpp'):4d} "
          f"f64 {c('v_fma_f64') + c('v_fmac_f64') + c('v_mul_f64') + c('v_add_f64'):5d} mfma {c('v_mfma'):4d}")
