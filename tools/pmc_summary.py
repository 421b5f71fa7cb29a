#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes (run_pmc.sh) into per-kernel, per-launch averages.

FETCH_SIZE is doubled (gfx950: it reports half the bytes of wide coalesced reads,
MI355X_MICROARCH.md "HBM [CDNA4]"); WRITE_SIZE is taken as is. Both are in KiB in rocprofv3.

usage: pmc_summary.py OUT.json EVENTS_PER_LAUNCH gpurun_out/pmc/p1 [p2 ...]
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

KERNELS = {"k_part": r"ek::k_part<", "k_agg": r"ek::k_agg<", "k_stats": r"ek::k_stats[<(]",
           "k_finalize": r"ek::k_finalize<"}


def main():
    out, events, dirs = sys.argv[1], int(sys.argv[2]), sys.argv[3:]
    vals = defaultdict(lambda: defaultdict(list))   # kernel -> counter -> per-dispatch values
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                name = r.get("Kernel_Name", "")
                for k, pat in KERNELS.items():
                    if re.search(pat, name):
                        vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    res = {"note": "per-launch averages; FETCH_SIZE doubled per the gfx950 correction; sizes converted KiB -> bytes",
           "events_per_launch": events, "kernels": {}}
    for k, cs in vals.items():
        e = {c: sum(v) / len(v) for c, v in cs.items()}
        e["dispatches"] = {c: len(v) for c, v in cs.items()}
        fetch = e.get("FETCH_SIZE")
        write = e.get("WRITE_SIZE")
        if fetch is not None:
            e["hbm_read_bytes_per_launch"] = 2 * fetch * 1024
        if write is not None:
            e["hbm_write_bytes_per_launch"] = write * 1024
        if fetch is not None and write is not None:
            e["hbm_bytes_per_launch"] = e["hbm_read_bytes_per_launch"] + e["hbm_write_bytes_per_launch"]
        e["events_per_launch"] = events
        res["kernels"][k] = e
    json.dump(res, open(out, "w"), indent=1, sort_keys=True)
    print(json.dumps(res, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
