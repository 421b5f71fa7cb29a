#!/bin/bash
# round-6 close, part A: the heavy GPU suites (key-major, range, full size, sharding)
cd "$(dirname "$0")/../.."; mkdir -p gpurun_out/r6final
timeout -k 10 1100 python -u -m pytest tests/test_keymajor_gpu.py tests/test_range_gpu.py tests/test_fullsize_gpu.py \
  tests/test_fullsize_parity_gpu.py tests/test_sharding_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r6final/tests_a.log 2>&1
rc=$?; tail -4 gpurun_out/r6final/tests_a.log; exit $rc
