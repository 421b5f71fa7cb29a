#!/bin/bash
# round 5: v2 sliding windows (processing time; event time with delay) + state / incremental suites, then the
# key-major fold trace (debug build)
cd "$(dirname "$0")/../.."; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_state_window_gpu.py tests/test_inc_processing_gpu.py tests/test_state_gpu.py \
  tests/test_processing_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r5_c_tests.log 2>&1
rc=$?; tail -25 gpurun_out/r5_c_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu/run_r5_km_trace.sh
