#!/bin/bash
# round 6: fused sorted pass (glds ts, deferred values) + k_km_walk<HS> — tests, C2/C3/C4a bench
cd "$(dirname "$0")/../.."; mkdir -p gpurun_out/r6d
timeout -k 10 300 python -u -m pytest tests/test_fused_gpu.py tests/test_async_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r6d/fused.log 2>&1
rc=$?; tail -2 gpurun_out/r6d/fused.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u -m pytest tests/test_keymajor_gpu.py tests/test_engine_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r6d/tests.log 2>&1
rc=$?; tail -2 gpurun_out/r6d/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u -m pytest tests/test_fullsize_parity_gpu.py -k "c2 or c3 or c4a" -x -q --timeout 300 --timeout-method thread > gpurun_out/r6d/full.log 2>&1
rc=$?; tail -2 gpurun_out/r6d/full.log; [ $rc -eq 0 ] || exit $rc
run() { tag=$1; cfg=$2; shift; shift
  env "$@" timeout -k 10 150 python bench.py --config $cfg --steps 20 --warmup 3 --no-cpu --no-ingest > gpurun_out/r6d/$tag.log 2>&1 || exit $?
  tail -1 gpurun_out/r6d/$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['roofline']['kernels']; print('$tag', round(d['ms_per_step'],4), {a[:12]: round(v['launch_ms'],4) for a,v in k.items()}, d['config'].get('fused_sorted_batches_last_step'), flush=True)"
}
run c2 C2 X=1
run c2_nofuse C2 EKGPU_FUSED=0
run c3 C3 X=1
run c4a C4a X=1
run c2b C2 X=1
