#!/bin/bash
# k_small_win<HS> with capped candidate tables + redo launch: bench C4b / C4a, then the small-window suites -> gpurun_out/r5g
cd "$(dirname "$0")/../.."; mkdir -p gpurun_out/r5g
for c in C4b C4a; do
  timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 3 --no-cpu --no-ingest > gpurun_out/r5g/$c.json 2> gpurun_out/r5g/$c.err || { tail -5 gpurun_out/r5g/$c.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r5g/$c.json')); r=d['roofline']; print('$c', round(d['ms_per_step'],4), 'dev', round(r.get('device_ms_per_step') or 0,4), {k[:12]: round(v['launch_ms'],4) for k,v in r.get('kernels',{}).items()})"
done
EKGPU_SW_CAP=0 timeout -k 10 300 python bench.py --config C4b --steps 20 --warmup 3 --no-cpu --no-ingest > gpurun_out/r5g/C4b_nocap.json 2>&1 && python3 -c "import json; d=json.load(open('gpurun_out/r5g/C4b_nocap.json')); print('C4b nocap', round(d['ms_per_step'],4))"
timeout -k 10 700 python -u -m pytest tests/test_range_gpu.py tests/test_window_error_gpu.py tests/test_fullsize_parity_gpu.py tests/test_engine_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5g/tests.log 2>&1
rc=$?; tail -4 gpurun_out/r5g/tests.log; exit $rc
