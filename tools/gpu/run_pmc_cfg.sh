#!/bin/bash
# PMC passes of one bench config, each set its own run: run_pmc_cfg.sh <cfg> "<counters 1>" ["<counters 2>" ...]
cd "$(dirname "$0")/../.."; cfg=$1; shift
mkdir -p gpurun_out/pmc_$cfg
export TMPDIR=/tmp
i=0
for set in "$@"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d gpurun_out/pmc_$cfg/p$i -o run -- python3 bench.py --config $cfg --steps 1 --warmup 1 --no-cpu --no-ingest > gpurun_out/pmc_$cfg/p$i.log 2>&1
  rc=$?; echo "pass $i ($set) rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
