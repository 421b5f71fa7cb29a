#!/bin/bash
# round-6 evidence per config: rocprofv3 kernel trace + stats, FETCH_SIZE and WRITE_SIZE passes (each its own run)
# -> gpurun_out/r6prof/<cfg>/...; the profiles are written here by tools/profile_configs.py (EKGPU_ROUND=r06)
cd "$(dirname "$0")/../.."; mkdir -p gpurun_out/r6prof
export TMPDIR=/tmp
for c in ${CONFIGS:-C2 C3 C4a C4b C5 C1}; do
  d=gpurun_out/r6prof/$c; mkdir -p $d
  ing=--no-ingest
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $d/trace -o run -- python3 bench.py --config $c --steps 5 --warmup 1 --no-cpu $ing > $d/trace.log 2>&1 || { echo "$c trace failed"; tail -3 $d/trace.log; exit 1; }
  timeout -k 10 -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $d/fetch -o run -- python3 bench.py --config $c --steps 1 --warmup 1 --no-cpu $ing > $d/fetch.log 2>&1 || { echo "$c fetch failed"; exit 1; }
  timeout -k 10 -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $d/write -o run -- python3 bench.py --config $c --steps 1 --warmup 1 --no-cpu $ing > $d/write.log 2>&1 || { echo "$c write failed"; exit 1; }
  echo "$c done"
done
