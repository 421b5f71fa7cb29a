#!/bin/bash
# GPU: selected parity tests (TESTS=...; default the whole -m gpu suite), verbose, one log
cd "$(dirname "$0")/../.."; mkdir -p gpurun_out
timeout -k 10 ${TLIMIT:-900} python -u -m pytest ${TESTS:-tests} -m gpu -x -v -s --timeout ${PER_TEST:-300} --timeout-method thread > gpurun_out/pytest_sel.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|Error|error|^C[2345]|^ *[0-9]+ passed" gpurun_out/pytest_sel.log | tail -60; exit $rc
