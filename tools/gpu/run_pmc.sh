#!/bin/bash
# PMC counter passes (separate runs; no tracing domains combined with --pmc)
cd "$(dirname "$0")/../.."; mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
rocprofv3 -L > gpurun_out/pmc/counters_list.txt 2>&1 || true
i=0
for set in "$@"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d gpurun_out/pmc/p$i -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu > gpurun_out/pmc/p$i.log 2>&1
  rc=$?; echo "pass $i ($set) rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
