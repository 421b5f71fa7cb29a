#!/usr/bin/env python3
"""Per-kernel averages per dispatch of rocprofv3 --pmc passes (tools/gpu/run_pmc_cfg.sh):
usage: pmc_kernels.py gpurun_out/pmc_<cfg> [kernel-substring]. FETCH_SIZE doubled (gfx950), sizes in bytes."""
import csv, glob, os, sys
from collections import defaultdict

d, pat = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else "ek::")
vals = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    per = defaultdict(float)
    for r in csv.DictReader(open(f)):
        name = r.get("Kernel_Name", "")
        if pat not in name and not (pat == "ek::" and "__amd_rocclr_" in name):   # the engine's copies / fills too
            continue
        per[(name.split("(")[0].replace("void ", ""), r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
    for (k, _, c), v in per.items():
        vals[k][c].append(v)
for k in sorted(vals):
    out = {}
    for c, v in sorted(vals[k].items()):
        a = sum(v) / len(v)
        if c == "FETCH_SIZE": a *= 2 * 1024
        elif c == "WRITE_SIZE": a *= 1024
        out[c] = round(a)
    print(k[:70], out)
