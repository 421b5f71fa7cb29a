#!/bin/bash
# round 5: STRING / BOOLEAN JSON ingest (device dictionary) + BOOLEAN engine columns, then the ingest / engine suites
cd "$(dirname "$0")/../.."; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_ingest_strings_gpu.py tests/test_ingest_gpu.py -x -v --timeout 180 \
  --timeout-method thread > gpurun_out/r5_d_tests.log 2>&1
rc=$?; tail -40 gpurun_out/r5_d_tests.log; exit $rc
