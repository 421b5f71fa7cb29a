#!/bin/bash
# kernel traces (start / end per dispatch) of a few configs -> gpurun_out/r5trace/<cfg>
cd "$(dirname "$0")/../.."; mkdir -p gpurun_out/r5trace
export TMPDIR=/tmp
for c in ${CONFIGS:-C4a C5 C3}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r5trace/$c -o run -- python3 bench.py --config $c --steps 3 --warmup 1 --no-cpu --no-ingest > gpurun_out/r5trace/$c.log 2>&1 || { echo "$c trace failed"; tail -3 gpurun_out/r5trace/$c.log; exit 1; }
  echo "$c done"
done
