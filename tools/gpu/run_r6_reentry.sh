#!/bin/bash
# round 6 re-entry: this round's GPU suites on HEAD, then one bench line per config (fused sorted pass on / off for C2, C3)
cd "$(dirname "$0")/../.."; mkdir -p gpurun_out/r6re
timeout -k 10 900 python -u -m pytest tests/test_fused_gpu.py tests/test_async_gpu.py tests/test_route_gpu.py tests/test_json_nested_gpu.py \
  tests/test_state_window_gpu.py tests/test_group_keys.py tests/test_range_gpu.py tests/test_keymajor_gpu.py tests/test_state_gpu.py \
  tests/test_sharding_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6re/tests.log 2>&1
rc=$?; tail -3 gpurun_out/r6re/tests.log; [ $rc -eq 0 ] || exit $rc
run() { tag=$1; cfg=$2; shift; shift
  env "$@" timeout -k 10 200 python bench.py --config $cfg --steps 20 --warmup 3 --no-cpu --no-ingest > gpurun_out/r6re/$tag.json 2> gpurun_out/r6re/$tag.err || { tail -3 gpurun_out/r6re/$tag.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/r6re/$tag.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$tag', round(d['ms_per_step'],4), round(r.get('device_ms_per_step',0),4), {k[:14]: round(v['launch_ms'],4) for k,v in r.get('kernels',{}).items()}, flush=True)"
}
run c2 C2 X=1
run c2_fused C2 EKGPU_FUSED=1
run c3 C3 X=1
run c3_fused C3 EKGPU_FUSED=1
run c4a C4a X=1
run c4b C4b X=1
run c5 C5 X=1
