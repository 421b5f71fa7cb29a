#!/bin/bash
# round 6: k_finalize_ring with the pane loop unrolled by the prefetch depth (fixed queue slots) — hopping / ring suites,
# full-size C3 parity, C3 bench x3, C2 bench (the k_agg knob-free build)
cd "$(dirname "$0")/../.."; mkdir -p gpurun_out/r6ring2
timeout -k 10 500 python -u -m pytest tests/test_engine_gpu.py tests/test_hopping_gap.py tests/test_late_tolerance_gpu.py tests/test_window_error_gpu.py \
  tests/test_state_gpu.py tests/test_determinism_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6ring2/tests.log 2>&1
rc=$?; tail -3 gpurun_out/r6ring2/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_fullsize_parity_gpu.py -k "c3" -x -q --timeout 300 --timeout-method thread > gpurun_out/r6ring2/full.log 2>&1
rc=$?; tail -3 gpurun_out/r6ring2/full.log; [ $rc -eq 0 ] || exit $rc
run() { tag=$1; cfg=$2; shift; shift
  env "$@" timeout -k 10 200 python bench.py --config $cfg --steps 20 --warmup 3 --no-cpu --no-ingest > gpurun_out/r6ring2/$tag.json 2> gpurun_out/r6ring2/$tag.err || { tail -3 gpurun_out/r6ring2/$tag.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/r6ring2/$tag.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$tag', round(d['ms_per_step'],4), round(r.get('device_ms_per_step',0),4), {k[:14]: round(v['launch_ms'],4) for k,v in r.get('kernels',{}).items()}, flush=True)"
}
run c3 C3 X=1
run c3_ch1 C3 EKGPU_FIN_RING_CHUNKS=1
run c3_fused C3 EKGPU_FUSED=1
run c3b C3 X=1
run c2 C2 X=1
