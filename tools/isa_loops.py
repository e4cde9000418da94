#!/usr/bin/env python3
"""Instruction mix of every basic block of one kernel in a gfx950 assembly
file (hipcc -S --cuda-device-only), loop headers marked: where a kernel's
issue slots go.
    python tools/isa_loops.py FILE.s KERNEL-NAME-FILTER [min-instrs]"""
import re
import sys
from collections import Counter

path, flt = sys.argv[1], sys.argv[2]
lo = int(sys.argv[3]) if len(sys.argv) > 3 else 8
s = open(path).read()
m = [x for x in re.finditer(r"^(_Z\S+):\s", s, re.M) if flt in x.group(1)]
if not m:
    sys.exit(f"no kernel matching {flt}")
i = m[0].end()
body = s[i:s.index(".Lfunc_end", i)].split("\n")
blocks = []
for l in body:
    t = l.strip()
    if re.match(r"^\.LBB\d+_\d+:", t):
        blocks.append([t.split(":")[0] + (" LOOP" if "Loop Header" in t else (" in-loop" if "Loop:" in t else "")), []])
        continue
    if not t or t.startswith((".", ";")) or t.endswith(":"):
        continue
    if not blocks:
        blocks.append(["entry", []])
    blocks[-1][1].append(t.split()[0])
tot = Counter()
for name, ins in blocks:
    c = Counter(ins)
    tot.update(c)
    if len(ins) < lo:
        continue
    g = lambda *p: sum(n for k, n in c.items() if k.startswith(p))
    print(f"{name:28s} {len(ins):5d}  valu {g('v_'):4d} (trans {g('v_exp', 'v_log', 'v_rcp', 'v_rsq', 'v_sqrt', 'v_sin', 'v_cos'):3d}, "
          f"f64 {g('v_fma_f64', 'v_mul_f64', 'v_add_f64', 'v_fmac_f64'):3d}, pk {g('v_pk'):3d}, mfma {g('v_mfma'):3d})  "
          f"salu {g('s_') - g('s_waitcnt', 's_cbranch', 's_branch', 's_nop'):3d}  br {g('s_cbranch', 's_branch'):3d}  "
          f"ds {g('ds_'):3d}  vmem {g('global_', 'buffer_', 'flat_'):3d}  wait {g('s_waitcnt'):3d}")
print("total", sum(tot.values()))
