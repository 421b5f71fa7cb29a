#!/bin/bash
# GPU: key-major range path — parity tests (forced and default rule), range-mode regression, then C4a / C5 bench lines
cd "$(dirname "$0")/../.."; mkdir -p gpurun_out/km
timeout -k 10 900 python -u -m pytest tests/test_keymajor_gpu.py tests/test_range_gpu.py tests/test_abi.py -x -v \
  --timeout 300 --timeout-method thread > gpurun_out/km/tests.log 2>&1
rc=$?; tail -4 gpurun_out/km/tests.log; [ $rc -eq 0 ] || exit $rc
for c in ${CONFIGS:-C4a C5 C4b}; do
  timeout -k 10 300 python bench.py --config $c --steps 5 --warmup 2 --no-cpu --no-ingest > gpurun_out/km/$c.json 2> gpurun_out/km/$c.err
  rc=$?; echo "$c rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/km/$c.json) $(grep -o '"frac": [0-9.]*' gpurun_out/km/$c.json | head -1)"
  [ $rc -eq 0 ] || { tail -5 gpurun_out/km/$c.err; exit $rc; }
done
