#!/bin/bash
# What the driver runs at round end: smoke(), then the default bench (with the CPU-baseline leg)
cd "$(dirname "$0")/../.."; mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
SECONDS=0; timeout -k 10 600 python bench.py > gpurun_out/bench_default.log 2> gpurun_out/bench_default.err
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_default.log; echo "bench wall $SECONDS s"; exit $rc
