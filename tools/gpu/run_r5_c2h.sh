#!/bin/bash
# round 5 C2: k_agg without the HAVING evaluator (U=8 / U=4), k_stats grid sweep
cd "$(dirname "$0")/../.."; mkdir -p gpurun_out/c2h
B=$PWD/ekuiper-vioneta_amd
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py tests/test_window_error_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/c2h/tests.log 2>&1
rc=$?; tail -1 gpurun_out/c2h/tests.log; [ $rc -eq 0 ] || exit $rc
run() { tag=$1; shift
  env "$@" timeout -k 10 150 python bench.py --config C2 --steps 20 --warmup 3 --no-cpu > gpurun_out/c2h/$tag.log 2>&1 || exit $?
  tail -1 gpurun_out/c2h/$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['roofline']['kernels']; print('$tag', round(d['ms_per_step'],4), [round(v['launch_ms'],4) for v in k.values()])"
}
for i in 1 2; do
  run prod_$i X=1
  run u4_$i EKGPU_LIB=$B/build_v_u4/libekgpu.so
  run sb512_$i EKGPU_STATS_BLOCKS=512
  run sb2048_$i EKGPU_STATS_BLOCKS=2048
  run sb4096_$i EKGPU_STATS_BLOCKS=4096
done
