#!/bin/bash
# range-mode parity (event buffer paths) + full-size C4a / C5, then the C5 / C4a bench lines
cd "$(dirname "$0")/../.."; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_range_gpu.py tests/test_processing_gpu.py tests/test_state_gpu.py \
  tests/test_sharding_gpu.py tests/test_keymajor_gpu.py tests/test_window_error_gpu.py tests/test_first_row_gpu.py \
  tests/test_state_window_gpu.py tests/test_group_keys.py \
  "tests/test_fullsize_parity_gpu.py::test_c4a_sliding_full_parity" "tests/test_fullsize_parity_gpu.py::test_c5_shard_full_parity" \
  -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4_range_tests.log 2>&1
rc=$?; tail -6 gpurun_out/r4_range_tests.log; [ $rc -eq 0 ] || exit $rc
CONFIGS="${CONFIGS:-C5 C4a}" bash tools/gpu/run_r4_quick.sh
