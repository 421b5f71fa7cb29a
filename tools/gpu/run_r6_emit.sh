#!/bin/bash
# round 6: k_agg early row reservation — pane-mode suites + full-size C2/C3 parity, then the C2 A/B
cd "$(dirname "$0")/../.."; mkdir -p gpurun_out/r6emit
timeout -k 10 500 python -u -m pytest tests/test_engine_gpu.py tests/test_window_error_gpu.py tests/test_late_tolerance_gpu.py tests/test_fused_gpu.py \
  tests/test_alignment_gpu.py tests/test_hopping_gap.py tests/test_determinism_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r6emit/tests.log 2>&1
rc=$?; tail -3 gpurun_out/r6emit/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_fullsize_parity_gpu.py -k "c2 or C2" -x -q --timeout 300 --timeout-method thread > gpurun_out/r6emit/full.log 2>&1
rc=$?; tail -3 gpurun_out/r6emit/full.log; [ $rc -eq 0 ] || exit $rc
run() { tag=$1; cfg=$2; shift; shift
  env "$@" timeout -k 10 200 python bench.py --config $cfg --steps 20 --warmup 3 --no-cpu --no-ingest > gpurun_out/r6emit/$tag.json 2> gpurun_out/r6emit/$tag.err || { tail -3 gpurun_out/r6emit/$tag.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/r6emit/$tag.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$tag', round(d['ms_per_step'],4), round(r.get('device_ms_per_step',0),4), {k[:14]: round(v['launch_ms'],4) for k,v in r.get('kernels',{}).items()}, flush=True)"
}
run new C2 X=1
run old C2 EKGPU_VARIANT=1
run nostore C2 EKGPU_DEBUG_AGG=64
run new2 C2 X=1
run old2 C2 EKGPU_VARIANT=1
run sb2048 C2 EKGPU_STATS_BLOCKS=2048
run sb4096 C2 EKGPU_STATS_BLOCKS=4096
