#!/usr/bin/env python3
"""Per-launch durations from a rocprofv3 --kernel-trace CSV, in launch order:
    python tools/ktrace.py <kernel_trace.csv> [name-filter ...]
Prints, per kernel name matching a filter, its launches' durations (us) in
order (e.g. the 20 k_bkernel launches of one outer step, beta-iteration by
beta-iteration)."""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
flt = sys.argv[2:] or [""]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
by = {}
for r in rows:
    name = r["Kernel_Name"]
    short = re.sub(r"^.*?(k_\w+).*$", r"\1", name)
    if any(f in short for f in flt):
        by.setdefault(short, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in by.items():
    print(f"{k} ({len(v)} launches):")
    for i in range(0, len(v), 20):
        print("  " + " ".join(f"{x:6.1f}" for x in v[i:i + 20]))
