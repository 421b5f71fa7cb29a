#!/bin/bash
# round-6 close, part B: every other GPU suite, then smoke()
cd "$(dirname "$0")/../.."; mkdir -p gpurun_out/r6final
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  --deselect tests/test_keymajor_gpu.py --deselect tests/test_range_gpu.py --deselect tests/test_fullsize_gpu.py \
  --deselect tests/test_fullsize_parity_gpu.py --deselect tests/test_sharding_gpu.py \
  > gpurun_out/r6final/tests_b.log 2>&1
rc=$?; tail -4 gpurun_out/r6final/tests_b.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6final/smoke.log 2>&1; rc=$?; tail -3 gpurun_out/r6final/smoke.log; exit $rc
