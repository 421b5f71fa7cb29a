#!/bin/bash
# round 6: nested JSON paths / LIST columns / top-level arrays / number->STRING / subnormals + the existing ingest tests
cd "$(dirname "$0")/../.."; mkdir -p gpurun_out/r6json
timeout -k 10 400 python -u -m pytest tests/test_json_nested_gpu.py tests/test_ingest_gpu.py tests/test_ingest_strings_gpu.py -x -q \
  --timeout 200 --timeout-method thread > gpurun_out/r6json/tests.log 2>&1
rc=$?; tail -30 gpurun_out/r6json/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --config C1 --steps 20 --warmup 3 --no-cpu > gpurun_out/r6json/c1.json 2> gpurun_out/r6json/c1.err || { tail -5 gpurun_out/r6json/c1.err; exit 1; }
tail -1 gpurun_out/r6json/c1.json | cut -c1-600
