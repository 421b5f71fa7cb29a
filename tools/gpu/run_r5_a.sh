#!/bin/bash
# round 5: processing-time incremental windows + the touched suites (production build), then the key-major gather
# diagnostic (debug build: the gather synchronised and checked on its own, wave starts of the walk printed)
cd "$(dirname "$0")/../.."; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_inc_processing_gpu.py tests/test_processing_gpu.py tests/test_incremental_gpu.py \
  tests/test_state_gpu.py tests/test_shared_source_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r5_a_tests.log 2>&1
rc=$?; tail -25 gpurun_out/r5_a_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu/run_r5_km_print.sh
