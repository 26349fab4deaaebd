"""Turn two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE) of a bench workload into
profiles/traffic_<workload>.json: average HBM bytes per launch of each named kernel.

Corrections follow /opt/skills/guides/MI355X_MICROARCH.md (HBM section): FETCH_SIZE and
WRITE_SIZE are in KiB; FETCH_SIZE is doubled on gfx950 (128-B requests tallied at 64 B).
Usage: python scripts/pmc_traffic.py <fetch_dir> <write_dir> <out.json> <kernel-substring>...
(the first kernel's entry is also written at the top level, for older readers; a name ending in "(" matches
that kernel only, not the kernels it prefixes — "k_wifi_rx(" against k_wifi_rx_sort — and is keyed without it)
"""
import csv
import glob
import json
import os
import sys


def per_dispatch(d, counter, kernel):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    vals = {}
    for f in files:
        for row in csv.DictReader(open(f)):
            if row.get("Counter_Name") != counter or kernel not in row.get("Kernel_Name", ""):
                continue
            key = (f, row.get("Dispatch_Id"))
            vals[key] = vals.get(key, 0.0) + float(row["Counter_Value"])
    if not vals:
        raise SystemExit(f"no {counter} rows for {kernel} in {d}")
    return sum(vals.values()) / len(vals), len(vals)


def main():
    fdir, wdir, out = sys.argv[1:4]
    kernels = sys.argv[4:]
    res = {"correction": "FETCH_SIZE KiB x1024 x2 (gfx950), WRITE_SIZE KiB x1024", "kernels": {}}
    for k in kernels:
        fetch_kib, nf = per_dispatch(fdir, "FETCH_SIZE", k)
        write_kib, nw = per_dispatch(wdir, "WRITE_SIZE", k)
        rd = 2.0 * fetch_kib * 1024.0
        wr = write_kib * 1024.0
        res["kernels"][k.rstrip("(")] = {"fetch_bytes_per_launch": rd, "write_bytes_per_launch": wr,
                             "hbm_bytes_per_launch": rd + wr, "dispatches": [nf, nw]}
    first = res["kernels"][kernels[0].rstrip("(")]
    res.update({"kernel": kernels[0].rstrip("("), **first})
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
