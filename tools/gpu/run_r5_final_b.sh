#!/bin/bash
# round-5 close, part B: every other GPU suite
cd "$(dirname "$0")/../.."; mkdir -p gpurun_out/r5final
timeout -k 10 1050 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  --deselect tests/test_keymajor_gpu.py --deselect tests/test_range_gpu.py --deselect tests/test_fullsize_gpu.py \
  --deselect tests/test_fullsize_parity_gpu.py --deselect tests/test_sharding_gpu.py \
  > gpurun_out/r5final/tests_b.log 2>&1
rc=$?; tail -4 gpurun_out/r5final/tests_b.log; exit $rc
