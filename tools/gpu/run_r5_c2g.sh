#!/bin/bash
# round 5 C2: k_agg walk variants (software pipeline U=4/8, U=4) against production — parity of each, then the bench
cd "$(dirname "$0")/../.."; mkdir -p gpurun_out/c2g
B=$PWD/ekuiper-vioneta_amd
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py tests/test_async_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/c2g/tests_prod.log 2>&1
rc=$?; tail -2 gpurun_out/c2g/tests_prod.log; [ $rc -eq 0 ] || exit $rc
for v in pipe4 pipe8; do
  EKGPU_LIB=$B/build_v_$v/libekgpu.so timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/c2g/tests_$v.log 2>&1
  rc=$?; tail -1 gpurun_out/c2g/tests_$v.log; [ $rc -eq 0 ] || exit $rc
done
run() { tag=$1; shift
  env "$@" timeout -k 10 150 python bench.py --config C2 --steps 20 --warmup 3 --no-cpu > gpurun_out/c2g/$tag.log 2>&1 || exit $?
  tail -1 gpurun_out/c2g/$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['roofline']['kernels']; print('$tag', round(d['ms_per_step'],4), [round(v['launch_ms'],4) for v in k.values()])"
}
for i in 1 2; do
  run prod_$i X=1
  run pipe4_$i EKGPU_LIB=$B/build_v_pipe4/libekgpu.so
  run pipe8_$i EKGPU_LIB=$B/build_v_pipe8/libekgpu.so
  run u4_$i EKGPU_LIB=$B/build_v_u4/libekgpu.so
done
