#!/bin/bash
# host-gap fixes: quick bench of the range / pane configs (no CPU baseline), then the range / key-major / processing
# suites -> gpurun_out/r5e
cd "$(dirname "$0")/../.."; mkdir -p gpurun_out/r5e
for c in ${CONFIGS:-C4b C3 C4a C5 C2}; do
  timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 3 --no-cpu --no-ingest > gpurun_out/r5e/$c.json 2> gpurun_out/r5e/$c.err || { tail -5 gpurun_out/r5e/$c.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r5e/$c.json')); r=d['roofline']; print('$c', round(d['ms_per_step'],4), 'dev', round(r.get('device_ms_per_step') or 0,4), {k[:12]: round(v['launch_ms'],4) for k,v in r.get('kernels',{}).items()})"
done
timeout -k 10 600 python -u -m pytest tests/test_range_gpu.py tests/test_keymajor_gpu.py tests/test_processing_gpu.py tests/test_engine_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r5e/tests.log 2>&1
rc=$?; tail -4 gpurun_out/r5e/tests.log; exit $rc
