#!/bin/bash
# GPU: key-major + small-window parity, bench lines, then rocprofv3 kernel stats of the range-mode configs
cd "$(dirname "$0")/../.."; mkdir -p gpurun_out/km
export TMPDIR=/tmp
CONFIGS="${CONFIGS:-C4a C5 C4b}" bash tools/gpu/run_km.sh || exit $?
for c in ${CONFIGS:-C4a C5 C4b}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/km/$c.prof -o run -- python3 bench.py --config $c --steps 5 --warmup 1 --no-cpu --no-ingest > gpurun_out/km/$c.prof.log 2>&1 || { echo "$c trace failed"; tail -3 gpurun_out/km/$c.prof.log; exit 1; }
  f=$(find gpurun_out/km/$c.prof -name '*kernel_stats.csv' | head -1); echo "== $c"; head -8 "$f" | cut -d, -f1-4 | cut -c1-160
done
