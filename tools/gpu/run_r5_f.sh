#!/bin/bash
# device-planned grouping partition (C5): bench C5 / C4a, then the key-major and full-size C5 / C4a suites -> gpurun_out/r5f
cd "$(dirname "$0")/../.."; mkdir -p gpurun_out/r5f
for c in C5 C4a; do
  timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 3 --no-cpu --no-ingest > gpurun_out/r5f/$c.json 2> gpurun_out/r5f/$c.err || { tail -5 gpurun_out/r5f/$c.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r5f/$c.json')); r=d['roofline']; print('$c', round(d['ms_per_step'],4), 'dev', round(r.get('device_ms_per_step') or 0,4), {k[:12]: round(v['launch_ms'],4) for k,v in r.get('kernels',{}).items()})"
done
timeout -k 10 700 python -u -m pytest tests/test_keymajor_gpu.py tests/test_fullsize_parity_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5f/tests.log 2>&1
rc=$?; tail -4 gpurun_out/r5f/tests.log; exit $rc
