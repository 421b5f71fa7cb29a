#!/bin/bash
# GPU check used through gpurun: parity tests, then a short bench. Stops at the first crash/timeout.
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }   # 1 = test failures (no fault): keep going
timeout -k 10 540 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -30 gpurun_out/pytest_gpu.log; ok $rc || exit $rc
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -5 gpurun_out/bench.log; exit $rc
