#!/bin/bash
# k_grp_walk<HV = false> (no interpreter without HAVING): bench C5, then the key-major / full-size suites -> gpurun_out/r5h
cd "$(dirname "$0")/../.."; mkdir -p gpurun_out/r5h
timeout -k 10 300 python bench.py --config C5 --steps 20 --warmup 3 --no-cpu --no-ingest > gpurun_out/r5h/C5.json 2> gpurun_out/r5h/C5.err || { tail -5 gpurun_out/r5h/C5.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r5h/C5.json')); r=d['roofline']; print('C5', round(d['ms_per_step'],4), 'dev', round(r.get('device_ms_per_step') or 0,4), {k[:12]: round(v['launch_ms'],4) for k,v in r.get('kernels',{}).items()})"
timeout -k 10 800 python -u -m pytest tests/test_keymajor_gpu.py tests/test_fullsize_parity_gpu.py tests/test_window_error_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5h/tests.log 2>&1
rc=$?; tail -4 gpurun_out/r5h/tests.log; exit $rc
