#!/usr/bin/env python3
"""Copy one measurement run's outputs (gpurun_out/, from `tools/gpu.sh round
TAG`, `tools/prof.sh TAG_cvar --workload cvar` and a CARLA kernel trace) into
profiles/ under the round's tag:
    python tools/collect_profiles.py TAG
bench line, GPU test log, rocprofv3 kernel stats (mmd_opt, cvar, CARLA), the
PMC counter tables, per-kernel HBM traffic, and the CARLA per-tick breakdown
from the kernel trace (kernel sum per tick vs the bench's wall clock)."""
import csv
import json
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
G = os.path.join(ROOT, "gpurun_out")
# PROFILES_OUT: write elsewhere (the GPU box: gpurun_out/profiles_TAG, so only
# the summaries travel back)
P = os.environ.get("PROFILES_OUT", os.path.join(ROOT, "profiles"))


def run(*a):
    return subprocess.run([sys.executable, *a], capture_output=True, text=True, check=True).stdout


def main():
    tag = sys.argv[1]
    out = lambda name: os.path.join(P, f"{tag}_{name}")  # noqa: E731
    os.makedirs(P, exist_ok=True)
    shutil.copy(os.path.join(G, f"bench_default_{tag}.json"), out("bench_default.json"))
    if os.path.exists(os.path.join(G, "gpu_tests.log")):
        shutil.copy(os.path.join(G, "gpu_tests.log"), out("gpu_tests.log"))
    traffic = {}
    for wl, d in (("mmdopt", f"prof_{tag}"), ("cvar", f"prof_{tag}_cvar")):
        src = os.path.join(G, d)
        if not os.path.isdir(src):
            continue
        shutil.copy(os.path.join(src, "stats", "run_kernel_stats.csv"), out(f"rocprof_kernel_stats_{wl}.csv"))
        open(out(f"pmc_counters_{wl}.txt"), "w").write(run(os.path.join(ROOT, "tools", "pmc_table.py"), src))
        tj = out(f"pmc_traffic_{wl}.json")
        run(os.path.join(ROOT, "tools", "pmc_traffic.py"), os.path.join(src, "pmc3", "run_counter_collection.csv"),
            os.path.join(src, "pmc4", "run_counter_collection.csv"), tj)
        traffic[wl] = json.load(open(tj))
    kt = os.path.join(G, f"kt_carla_{tag}")
    if os.path.isdir(kt):
        shutil.copy(os.path.join(kt, "run_kernel_stats.csv"), out("rocprof_kernel_stats_carla.csv"))
        # per-tick breakdown: every kernel's total over the traced run / ticks
        rows = list(csv.DictReader(open(os.path.join(kt, "run_kernel_stats.csv"))))
        line = [json.loads(l) for l in open(os.path.join(G, f"kt_carla_{tag}.log")) if l.startswith("{")][-1]
        ticks = line["ticks"] + 2  # timed + warmup ticks (the trace also holds the profiled and two-stream ticks)
        total_ms = sum(float(r["TotalDurationNs"]) for r in rows) / 1e6
        with open(out("carla_tick_breakdown.txt"), "w") as f:
            f.write(f"CARLA configs[4] (n = {line['num_reduced_set']}): rocprofv3 kernel trace of "
                    f"`bench.py --workload carla` -- {line['ticks']} timed ticks at {line['ms_per_tick_mmd_plus_cvar']:.2f} ms "
                    f"for mmd_opt + cvar, {line['per_cost']['mmd_opt']['ms_per_tick']:.2f} ms for an mmd_opt tick "
                    f"(wall clock, no per-launch events).\n")
            f.write(f"Kernel time over the whole traced run: {total_ms:.1f} ms for the timed + warmup ticks, the "
                    f"det solves, the profiled tick and the two-stream ticks.\n\n")
            f.write(f"{'kernel':60s} {'calls':>6s} {'avg us':>8s} {'total ms':>9s}\n")
            for r in rows:
                f.write(f"{r['Name'][:60]:60s} {int(r['Calls']):6d} {float(r['AverageNs']) / 1e3:8.1f} "
                        f"{float(r['TotalDurationNs']) / 1e6:9.2f}\n")
    print("written", sorted(x for x in os.listdir(P) if x.startswith(tag)))


if __name__ == "__main__":
    main()
