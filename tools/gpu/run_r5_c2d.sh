#!/bin/bash
# round 5 C2: one-reservation direct emission + XCD-ordered k_agg — parity (engine / full-size / HAVING / errors), then
# the C2 bench with the production build and the k_part / k_agg shape variants, and a kernel trace of the production step
cd "$(dirname "$0")/../.."; mkdir -p gpurun_out/c2d
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py tests/test_fullsize_parity_gpu.py tests/test_window_error_gpu.py \
  tests/test_expr_args_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/c2d/tests.log 2>&1
rc=$?; tail -5 gpurun_out/c2d/tests.log; [ $rc -eq 0 ] || exit $rc
run() { tag=$1; shift
  env "$@" timeout -k 10 150 python bench.py --config C2 --steps 20 --warmup 3 --no-cpu > gpurun_out/c2d/$tag.log 2>&1 || exit $?
  tail -1 gpurun_out/c2d/$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['roofline']['kernels']; print('$tag', round(d['ms_per_step'],4), [round(v['launch_ms'],4) for v in k.values()])"
}
B=$PWD/ekuiper-vioneta_amd
for i in 1 2; do
  run prod_$i X=1
  run agg4_$i EKGPU_LIB=$B/build_v_agg4/libekgpu.so
  run p2048_$i EKGPU_LIB=$B/build_v_p2048/libekgpu.so
  run p256_$i EKGPU_LIB=$B/build_v_p256/libekgpu.so
done
timeout -k 10 -s KILL 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c2d/trace -o run -- python3 bench.py --config C2 --steps 5 --warmup 2 --no-cpu --no-ingest > gpurun_out/c2d/trace.log 2>&1 || exit $?
python3 tools/trace_gaps.py $(ls gpurun_out/c2d/trace/*kernel_trace.csv | head -1)
