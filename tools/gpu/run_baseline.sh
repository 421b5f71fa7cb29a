#!/bin/bash
# GPU check: parity suite, short bench, rocprofv3 kernel-trace summary of the bench. Stops at the first fault.
cd "$(dirname "$0")/../.."; mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log | cut -c1-600; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/prof.log 2>&1
rc=$?; echo "prof rc=$rc"; exit $rc
