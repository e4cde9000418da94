"""Per-kernel table of the PMC passes written by tools/prof.sh.

    python tools/pmc_table.py gpurun_out/prof_TAG

Averages every counter over the dispatches of each library kernel and prints
one row per kernel (kernel names reduced to the library's short names)."""
import collections
import csv
import glob
import os
import sys


def short(name):
    if "k_" not in name:
        return None
    return name[name.find("k_") + 2:].split("(")[0].split("<")[0]


def main():
    root = sys.argv[1]
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    cnt = collections.defaultdict(collections.Counter)
    for path in glob.glob(os.path.join(root, "pmc*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(path)):
            k = short(r["Kernel_Name"])
            if k is None:
                continue
            tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
            cnt[k][r["Counter_Name"]] += 1
    for k in sorted(tot):
        row = {c.replace("SQ_", ""): tot[k][c] / cnt[k][c] for c in sorted(tot[k])}
        print(k, " ".join(f"{c}={v:.3g}" for c, v in row.items()))


if __name__ == "__main__":
    main()
