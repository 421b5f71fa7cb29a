#!/bin/bash
# round 6: k_finalize_ring with its window descriptors and pane flags staged in LDS — pane-mode suites (small partitions:
# the new instantiation) + full-size C2 / C3 parity, then C3 / C2 A/B against EKGPU_AGG_SMALL=0, twice
cd "$(dirname "$0")/../.."; mkdir -p gpurun_out/r6rlds
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py tests/test_window_error_gpu.py tests/test_late_tolerance_gpu.py tests/test_fused_gpu.py \
  tests/test_alignment_gpu.py tests/test_hopping_gap.py tests/test_determinism_gpu.py tests/test_state_gpu.py tests/test_expr_args_gpu.py \
  tests/test_processing_gpu.py tests/test_sharding_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r6rlds/tests.log 2>&1
rc=$?; tail -2 gpurun_out/r6rlds/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_fullsize_parity_gpu.py -k "c2 or c3" -x -q --timeout 300 --timeout-method thread > gpurun_out/r6rlds/full.log 2>&1
rc=$?; tail -2 gpurun_out/r6rlds/full.log; [ $rc -eq 0 ] || exit $rc
run() { tag=$1; cfg=$2; shift; shift
  env "$@" timeout -k 10 200 python bench.py --config $cfg --steps 20 --warmup 3 --no-cpu --no-ingest > gpurun_out/r6rlds/$tag.json 2> gpurun_out/r6rlds/$tag.err || { tail -3 gpurun_out/r6rlds/$tag.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/r6rlds/$tag.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$tag', round(d['ms_per_step'],4), round(r.get('device_ms_per_step',0),4), {k[:14]: round(v['launch_ms'],4) for k,v in r.get('kernels',{}).items()}, flush=True)"
}
for i in 1 2; do
  run c3_new$i C3 X=1
  run c3_old$i C3 EKGPU_RING_LDS=0
done
