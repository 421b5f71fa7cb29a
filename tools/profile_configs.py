#!/usr/bin/env python3
"""Per-config rocprofv3 summaries -> profiles/<round>_* (round = $EKGPU_ROUND, default r03):
  <round>_kernels_<cfg>.csv  rocprofv3 --kernel-trace --stats of `bench.py --config <cfg> --steps S --warmup W`
  <round>_pmc_<cfg>.json     FETCH_SIZE / WRITE_SIZE passes (each its own run, --steps 1 --warmup 1): HBM bytes of the
                         engine's kernels (ek::*) and of the runtime copy / fill kernels dispatched inside the pushes,
                         per step; FETCH_SIZE doubled (gfx950: it reports half the bytes of
                         wide coalesced reads, MI355X_MICROARCH.md "HBM"), sizes KiB -> bytes.
usage: profile_configs.py <cfg> <events_per_gpu> <steps_in_pmc_runs> <trace_dir> <pmc_fetch_dir> <pmc_write_dir>
"""
import csv
import glob
import json
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ROUND = os.environ.get("EKGPU_ROUND", "r05")


COPY_KERNELS = ("__amd_rocclr_copyBuffer", "__amd_rocclr_fillBuffer")


def counters(d):
    """Per-kernel sums of every counter over the engine's dispatches: the ek:: kernels, and the runtime's copy / fill
    kernels (hipMemcpyAsync / hipMemsetAsync, e.g. the event-buffer append) dispatched between the first and the last
    ek:: kernel of the process — the step's own copies; the synthetic-input setup before the first push is excluded."""
    per = defaultdict(lambda: defaultdict(float))
    n = defaultdict(lambda: defaultdict(int))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        rows = list(csv.DictReader(open(f)))
        ek_ids = [int(r["Dispatch_Id"]) for r in rows if "ek::" in r.get("Kernel_Name", "")]
        if not ek_ids:
            continue
        lo, hi = min(ek_ids), max(ek_ids)
        for r in rows:
            name = r.get("Kernel_Name", "")
            did = int(r["Dispatch_Id"])
            if "ek::" not in name and not (any(c in name for c in COPY_KERNELS) and lo <= did <= hi):
                continue
            k = name.split("(")[0].replace("void ", "")
            per[k][r["Counter_Name"]] += float(r["Counter_Value"])
            n[k][r["Counter_Name"]] += 1
    return per, n


def main():
    cfg, events, steps, tdir, fdir, wdir = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), sys.argv[4], sys.argv[5], sys.argv[6]
    stats = glob.glob(os.path.join(tdir, "**", "*kernel_stats.csv"), recursive=True)
    if stats:
        shutil.copy(stats[0], os.path.join(ROOT, "profiles", f"{ROUND}_kernels_{cfg}.csv"))
    f, fn = counters(fdir)
    w, wn = counters(wdir)
    kern = {}
    tot_r = tot_w = 0.0
    for k in sorted(set(f) | set(w)):
        rd = 2 * f[k].get("FETCH_SIZE", 0.0) * 1024
        wr = w[k].get("WRITE_SIZE", 0.0) * 1024
        disp = max(fn[k].get("FETCH_SIZE", 0), wn[k].get("WRITE_SIZE", 0), 1)
        kern[k] = {"read_bytes_per_step": rd / steps, "write_bytes_per_step": wr / steps, "dispatches": disp}
        tot_r += rd
        tot_w += wr
    out = {"config": cfg, "events_per_gpu": events, "steps_profiled": steps,
           "note": "PMC passes over `steps_profiled` pushes (warmup + timed); FETCH_SIZE doubled (gfx950), KiB -> bytes",
           "hbm_read_bytes_per_step": tot_r / steps, "hbm_write_bytes_per_step": tot_w / steps,
           "hbm_bytes_per_step": (tot_r + tot_w) / steps, "kernels": kern}
    json.dump(out, open(os.path.join(ROOT, "profiles", f"{ROUND}_pmc_{cfg}.json"), "w"), indent=1)
    print(cfg, f"{out['hbm_bytes_per_step'] / 1e9:.3f} GB/step", {k: round((v['read_bytes_per_step'] + v['write_bytes_per_step']) / 1e9, 3) for k, v in kern.items()})


if __name__ == "__main__":
    main()
