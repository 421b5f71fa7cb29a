#!/bin/bash
# round 4: small-window kernel check — its parity tests, the C4b bench line and its kernel profile
cd "$(dirname "$0")/../.."; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_range_gpu.py tests/test_state_window_gpu.py tests/test_first_row_gpu.py \
  tests/test_determinism_gpu.py tests/test_state_gpu.py "tests/test_fullsize_parity_gpu.py::test_c4b_count_full_parity" \
  -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4_sw_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r4_sw_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config C4b --steps 10 --warmup 2 --no-cpu > gpurun_out/r4_c4b.json 2> gpurun_out/r4_c4b.err
rc=$?; cut -c1-400 gpurun_out/r4_c4b.json; [ $rc -eq 0 ] || { tail -5 gpurun_out/r4_c4b.err; exit $rc; }
bash tools/gpu/prof.sh C4b 5
