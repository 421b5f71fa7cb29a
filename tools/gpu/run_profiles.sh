#!/bin/bash
# rocprofv3 kernel-trace summary + PMC traffic passes of the C2 bench (each pass its own run)
cd "$(dirname "$0")/../.."; mkdir -p gpurun_out/prof gpurun_out/pmc
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/prof.log 2>&1 || exit $?
echo "kernel-trace ok"
i=0
for set in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_LDS GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 -s KILL 120 rocprofv3 --pmc $set --output-format csv -d gpurun_out/pmc/p$i -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu > gpurun_out/pmc/p$i.log 2>&1
  rc=$?; echo "pass $i ($set) rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
