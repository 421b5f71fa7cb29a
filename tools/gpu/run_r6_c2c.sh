#!/bin/bash
# round 6 C2: the fused sorted pass (k_part MODE 3) — fused tests, pane-mode suites, full-size C2/C3 parity, bench
cd "$(dirname "$0")/../.."; mkdir -p gpurun_out/r6c2c
timeout -k 10 300 python -u -m pytest tests/test_fused_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r6c2c/fused.log 2>&1
rc=$?; tail -3 gpurun_out/r6c2c/fused.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u -m pytest tests/test_engine_gpu.py tests/test_window_error_gpu.py tests/test_late_tolerance_gpu.py \
  tests/test_alignment_gpu.py tests/test_state_gpu.py tests/test_hopping_gap.py tests/test_async_gpu.py tests/test_ingest_strings_gpu.py tests/test_ingest_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r6c2c/tests.log 2>&1
rc=$?; tail -3 gpurun_out/r6c2c/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_fullsize_parity_gpu.py -k "c2 or c3" -x -q --timeout 300 --timeout-method thread > gpurun_out/r6c2c/full.log 2>&1
rc=$?; tail -3 gpurun_out/r6c2c/full.log; [ $rc -eq 0 ] || exit $rc
run() { tag=$1; cfg=$2; shift; shift
  env "$@" timeout -k 10 150 python bench.py --config $cfg --steps 20 --warmup 3 --no-cpu --no-ingest > gpurun_out/r6c2c/$tag.log 2>&1 || exit $?
  tail -1 gpurun_out/r6c2c/$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['roofline']['kernels']; print('$tag', round(d['ms_per_step'],4), {a[:12]: round(v['launch_ms'],4) for a,v in k.items()}, d['config'].get('fused_sorted_batches_last_step'), flush=True)"
}
run c2 C2 X=1
run c2_nofuse C2 EKGPU_FUSED=0
run c3 C3 X=1
run c3_nofuse C3 EKGPU_FUSED=0
run c2b C2 X=1
