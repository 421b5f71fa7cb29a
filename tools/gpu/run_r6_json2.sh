#!/bin/bash
# round 6: k_json_decode staged through LDS — JSON suites, then C1 bench A/B (twice)
cd "$(dirname "$0")/../.."; mkdir -p gpurun_out/r6json2
timeout -k 10 500 python -u -m pytest tests/test_json_nested_gpu.py tests/test_ingest_gpu.py tests/test_ingest_strings_gpu.py tests/test_bool_oracle.py -m gpu -x -q \
  --timeout 200 --timeout-method thread > gpurun_out/r6json2/tests.log 2>&1
rc=$?; tail -3 gpurun_out/r6json2/tests.log; [ $rc -eq 0 ] || exit $rc
for t in a b; do
  timeout -k 10 200 python bench.py --config C1 --steps 20 --warmup 3 --no-cpu > gpurun_out/r6json2/c1_$t.json 2> gpurun_out/r6json2/c1_$t.err || { tail -5 gpurun_out/r6json2/c1_$t.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/r6json2/c1_$t.json').read().strip().splitlines()[-1]); r=d['roofline']; print('c1', round(d['ms_per_step'],4), {k[:16]: round(v['launch_ms'],4) for k,v in r.get('kernels',{}).items()}, flush=True)"
done
