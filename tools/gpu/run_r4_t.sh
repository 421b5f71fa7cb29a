#!/bin/bash
# selected GPU test files / nodes (TESTS), verbose log, with its own time limit
cd "$(dirname "$0")/../.."; mkdir -p gpurun_out
timeout -k 10 ${TLIMIT:-500} python -u -m pytest ${TESTS} -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4_t.log 2>&1
rc=$?; tail -25 gpurun_out/r4_t.log; exit $rc
