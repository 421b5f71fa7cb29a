#!/bin/bash
# GPU: range-mode parity tests (then the rest of the GPU suite when asked)
cd "$(dirname "$0")/../.."; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_range_gpu.py} -m gpu -x -v -s --timeout 200 --timeout-method thread > gpurun_out/pytest_range.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|Error|error" gpurun_out/pytest_range.log | tail -40; exit $rc
