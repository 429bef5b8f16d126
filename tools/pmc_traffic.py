#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into HBM bytes per launch.

gfx950 corrections (MI355X_MICROARCH.md §HBM, cdna_hip_programming.md §7):
  * FETCH_SIZE and WRITE_SIZE are in KiB (x1024);
  * FETCH_SIZE reports exactly half of the bytes of a wide (16 B/lane) coalesced
    streaming read, so it is doubled;
  * WRITE_SIZE is exact for 16 B/lane streaming stores.
FETCH_SIZE (3 TCC slots) and WRITE_SIZE (2) cannot share a pass: collect them in
two separate rocprofv3 runs and pass both directories.

usage: pmc_traffic.py OUT.json --fetch DIR --write DIR [--kernel SUBSTR] [--algo-bytes N] [--stat median|mean]
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict


def read_counters(d):
    vals = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> [per dispatch]
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    for path in files:
        with open(path) as f:
            per = defaultdict(float)
            rows = list(csv.DictReader(f))
        acc = defaultdict(float)
        names = {}
        for r in rows:
            key = (r.get("Dispatch_Id") or r.get("Correlation_Id"), r["Counter_Name"])
            acc[key] += float(r["Counter_Value"])
            names[key[0]] = r["Kernel_Name"]
        for (disp, ctr), v in acc.items():
            vals[names[disp]][ctr].append(v)
        del per
    return vals, files


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--kernel", default="")
    ap.add_argument("--algo-bytes", type=float, default=None)
    ap.add_argument("--note", default="")
    ap.add_argument("--stat", choices=("median", "mean"), default="median",
                    help="per-dispatch statistic: mean when one launch covers buckets of different sizes")
    a = ap.parse_args()
    fv, ff = read_counters(a.fetch)
    wv, wf = read_counters(a.write)
    kernels = {}
    for k in sorted(set(fv) | set(wv)):
        if a.kernel and a.kernel not in k:
            continue
        fetch = fv.get(k, {}).get("FETCH_SIZE", [])
        write = wv.get(k, {}).get("WRITE_SIZE", [])
        if not fetch or not write:
            continue
        # median dispatch (the first dispatches of a process include cold-cache effects); mean for
        # launches of different sizes (a list's buckets), against the mean algorithmic bytes
        if a.stat == "mean":
            fm, wm = sum(fetch) / len(fetch), sum(write) / len(write)
        else:
            fm = sorted(fetch)[len(fetch) // 2]
            wm = sorted(write)[len(write) // 2]
        hbm = (2 * fm + wm) * 1024
        e = {"dispatches_fetch": len(fetch), "dispatches_write": len(write), "FETCH_SIZE_KiB_median": fm,
             "WRITE_SIZE_KiB_median": wm, "read_bytes_corrected": 2 * fm * 1024, "write_bytes": wm * 1024,
             "hbm_bytes_per_launch": hbm, "statistic": a.stat + " over dispatches"}
        if a.algo_bytes:
            e["algorithmic_bytes_per_launch"] = a.algo_bytes
            e["traffic_over_algorithmic"] = hbm / a.algo_bytes
        kernels[k] = e
    out = {"source": {"fetch_files": [os.path.relpath(p) for p in ff], "write_files": [os.path.relpath(p) for p in wf]},
           "corrections": "FETCH_SIZE x2 (gfx950 half-count on wide streaming reads), KiB x1024",
           "note": a.note, "kernels": kernels}
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
