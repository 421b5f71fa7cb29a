#!/bin/bash
# Round-end check: GPU parity suite, smoke(), then the default bench line (with the CPU baseline legs).
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 540 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/bench_default.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_default.log | cut -c1-400; exit $rc
