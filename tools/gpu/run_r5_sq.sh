#!/bin/bash
# SQ instruction-mix / stall counters of one config's kernels (one pass) -> gpurun_out/r5sq/<cfg>
cd "$(dirname "$0")/../.."; mkdir -p gpurun_out/r5sq
export TMPDIR=/tmp
c=${CFG:-C4b}
timeout -k 10 -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU --output-format csv -d gpurun_out/r5sq/$c -o run -- python3 bench.py --config $c --steps 1 --warmup 1 --no-cpu --no-ingest > gpurun_out/r5sq/$c.log 2>&1
rc=$?; tail -3 gpurun_out/r5sq/$c.log; exit $rc
