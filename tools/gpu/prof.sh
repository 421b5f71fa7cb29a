#!/bin/bash
# rocprofv3 kernel-trace summary of `bench.py --config $1` (GPU box): gpurun_out/prof_$1/ + the top kernels printed.
# Usage: tools/gpu/prof.sh <config> [steps]
set -o pipefail
cfg=$1; steps=${2:-5}
cd "$(dirname "$0")/../.."
R=$PWD
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_$cfg" -o run -- \
    python3 "$R/bench.py" --config "$cfg" --steps "$steps" --warmup 2 --no-cpu --no-ingest > "$R/gpurun_out/prof_$cfg.log" 2>&1
rc=$?
f=$(find "$R/gpurun_out/prof_$cfg" -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && python3 - "$f" "$steps" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
steps = int(sys.argv[2]) + 2
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:14]:
    print(f'{float(r["TotalDurationNs"]) / steps / 1e6:8.3f} ms/step  {int(r["Calls"]) / steps:7.1f} calls/step  avg {float(r["AverageNs"]) / 1e3:9.1f} us  {r["Name"][:90]}')
PY
exit $rc
