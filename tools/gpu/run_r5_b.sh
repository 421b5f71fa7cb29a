#!/bin/bash
# round 5: incremental windows (processing time, WHERE over the last rows, FILTER) + the touched suites, then the
# key-major fault-address diagnostic
cd "$(dirname "$0")/../.."; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_inc_processing_gpu.py tests/test_incremental_gpu.py tests/test_window_error_gpu.py \
  tests/test_first_row_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r5_b_tests.log 2>&1
rc=$?; tail -25 gpurun_out/r5_b_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu/run_r5_km_addr.sh
