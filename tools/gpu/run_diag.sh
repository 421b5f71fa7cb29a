#!/bin/bash
cd "$(dirname "$0")/../.."; mkdir -p gpurun_out/diag; export TMPDIR=/tmp
for d in 0 1 2 3; do
  EKGPU_DEBUG_AGG=$d timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/diag/d$d -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu > gpurun_out/diag/d$d.log 2>&1 || exit $?
done
