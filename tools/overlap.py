#!/usr/bin/env python3
"""Where the two-stream mmd_opt step spends its time (rocprofv3 kernel trace):
    python tools/overlap.py <kernel_trace.csv> FIRST_STEP NSTEPS [marker]
The window runs from the start of the FIRST_STEP-th launch of `marker`
(k_mother: one per outer step) to the start of the (FIRST_STEP + NSTEPS)-th.
Per kernel: total busy time, and "exclusive" time -- the stretches where it is
the only kernel on the GPU (the other stream is idle or waiting), which is
what shortening that kernel can take off the step.  Also the idle time (no
kernel running)."""
import csv
import re
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
first, nsteps = int(sys.argv[2]), int(sys.argv[3])
marker = sys.argv[4] if len(sys.argv) > 4 else "k_mother"
ks = []
for r in rows:
    short = re.sub(r"^.*?(k_\w+).*$", r"\1", r["Kernel_Name"])
    if short.startswith("__amd"):
        short = "copy/fill"
    ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short))
ks.sort()
marks = [s for s, e, n in ks if n == marker]
t0, t1 = marks[first], marks[first + nsteps]
ev = []
for s, e, n in ks:
    s, e = max(s, t0), min(e, t1)
    if e > s:
        ev.append((s, 1, n))
        ev.append((e, -1, n))
ev.sort(key=lambda x: (x[0], x[1]))
active = defaultdict(int)
busy, excl = defaultdict(float), defaultdict(float)
idle = 0.0
both = 0.0
last = t0
for t, d, n in ev:
    dt = (t - last) / 1e3
    names = [k for k, v in active.items() if v > 0]
    cnt = sum(active.values())
    if cnt == 0:
        idle += dt
    elif cnt == 1:
        excl[names[0]] += dt
    else:
        both += dt
    for k in names:
        busy[k] += dt * active[k] / max(cnt, 1)
    active[n] += d
    last = t
idle += (t1 - last) / 1e3
tot = (t1 - t0) / 1e3
print(f"window {tot / nsteps:.1f} us per step ({nsteps} steps); idle {idle / nsteps:.1f}, "
      f">=2 kernels {both / nsteps:.1f}, one kernel {sum(excl.values()) / nsteps:.1f} us per step")
print(f"{'kernel':24s} {'busy(shared) us/step':>22s} {'alone us/step':>14s}")
for k in sorted(busy, key=lambda k: -excl[k]):
    print(f"{k:24s} {busy[k] / nsteps:22.1f} {excl[k] / nsteps:14.1f}")
