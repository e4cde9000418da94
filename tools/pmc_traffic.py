"""Per-kernel HBM bytes per launch from two rocprofv3 PMC passes
(FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950).

    python tools/pmc_traffic.py FETCH_CSV WRITE_CSV OUT_JSON

FETCH_SIZE on gfx950 reports half the bytes of wide coalesced reads
(MI355X_MICROARCH.md, HBM section), so traffic = 2 x FETCH_SIZE + WRITE_SIZE,
both in KiB per dispatch as rocprofv3 reports them.  Kernel names are reduced
to the library's short names (k_bkernel -> bkernel)."""
import collections
import csv
import json
import sys


def per_kernel(path, counter):
    tot = collections.defaultdict(float)
    cnt = collections.Counter()
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        name = r["Kernel_Name"]
        if "k_" not in name:
            continue
        short = name[name.find("k_") + 2:].split("(")[0].split("<")[0]
        tot[short] += float(r["Counter_Value"])
        cnt[short] += 1
    return {k: tot[k] / cnt[k] for k in tot}


def main():
    fetch = per_kernel(sys.argv[1], "FETCH_SIZE")
    write = per_kernel(sys.argv[2], "WRITE_SIZE")
    out = {k: (2.0 * fetch.get(k, 0.0) + write.get(k, 0.0)) * 1024.0 for k in set(fetch) | set(write)}
    json.dump(out, open(sys.argv[3], "w"), indent=1, sort_keys=True)
    for k in sorted(out):
        print(f"{k:14s} fetch {fetch.get(k, 0) / 1024:10.2f} MiB  write {write.get(k, 0) / 1024:10.2f} MiB  "
              f"traffic {out[k] / 2**20:10.2f} MiB/launch")


if __name__ == "__main__":
    main()
