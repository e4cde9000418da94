#!/usr/bin/env python3
"""Per-kernel resources (VGPR / AGPR / SGPR / spills / LDS / occupancy) from a
gfx950 assembly file:  python tools/kres.py /tmp/kb.s [name-filter]"""
import re
import sys

text = open(sys.argv[1]).read()
flt = sys.argv[2] if len(sys.argv) > 2 else ""
for m in re.finditer(r"\.amdhsa_kernel (\S+)\n(.*?)\.end_amdhsa_kernel", text, re.S):
    name, body = m.group(1), m.group(2)
    if flt not in name:
        continue
    g = lambda k: (re.search(r"\.amdhsa_" + k + r" (\d+)", body) or [0, "?"])[1]
    short = re.sub(r"^_ZN6mpcmmd12_GLOBAL__N_1\d+", "", name)[:60]
    # the comment block emitted after the kernel body carries the occupancy
    cm = re.search(re.escape(name) + r".*?; Occupancy: (\d+)", text, re.S)
    sp = re.search(re.escape(name) + r".*?; ScratchSize: (\d+)", text, re.S)
    print(f"{short:60s} vgpr {g('next_free_vgpr'):>4s} agpr_off {g('accum_offset'):>4s} sgpr {g('next_free_sgpr'):>4s} "
          f"lds {g('group_segment_fixed_size'):>6s} scratch {sp.group(1) if sp else '?':>5s} occ {cm.group(1) if cm else '?'}")
