#!/bin/bash
# round 6 C2: k_agg G8 fold (aligned 8-row groups, 16-B loads) — pane-path tests, C2 full-size parity, bench C2/C3
cd "$(dirname "$0")/../.."; mkdir -p gpurun_out/r6c2b
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py tests/test_window_error_gpu.py tests/test_late_tolerance_gpu.py \
  tests/test_range_gpu.py tests/test_fullsize_parity_gpu.py -k "c2 or c3" -x -q --timeout 300 --timeout-method thread > gpurun_out/r6c2b/tests.log 2>&1
rc=$?; tail -3 gpurun_out/r6c2b/tests.log; [ $rc -eq 0 ] || exit $rc
run() { tag=$1; cfg=$2; shift; shift
  env "$@" timeout -k 10 150 python bench.py --config $cfg --steps 20 --warmup 3 --no-cpu --no-ingest > gpurun_out/r6c2b/$tag.log 2>&1 || exit $?
  tail -1 gpurun_out/r6c2b/$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['roofline']['kernels']; print('$tag', round(d['ms_per_step'],4), [round(v['launch_ms'],4) for v in k.values()], flush=True)"
}
run c2 C2 X=1
run c2_loads C2 EKGPU_DEBUG_AGG=34
run c3 C3 X=1
run c2b C2 X=1
