#!/bin/bash
# key-major state emission (k_km_expand) + shared ts statistics: parity, then C4a / C5 A/B lines
cd "$(dirname "$0")/../.."; mkdir -p gpurun_out
TESTS="${TESTS:-tests/test_keymajor_gpu.py tests/test_range_gpu.py tests/test_shared_source_gpu.py tests/test_window_error_gpu.py}"
timeout -k 10 900 python -u -m pytest $TESTS "tests/test_fullsize_parity_gpu.py::test_c4a_sliding_full_parity" \
  -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4_km_tests.log 2>&1
rc=$?; tail -6 gpurun_out/r4_km_tests.log; [ $rc -eq 0 ] || exit $rc
CONFIGS="C4a" ENVS="${KM_ENVS:-EKGPU_KM_STATES=1 EKGPU_KM_STATES=0}" bash tools/gpu/run_r4_quick.sh || exit 1
for flag in "" "--no-shared-stats"; do
  tag="C5${flag:+_noshare}"
  timeout -k 10 300 python bench.py --config C5 --steps 10 --warmup 2 --no-cpu $flag > gpurun_out/s_${tag}.json 2> gpurun_out/s_${tag}.err
  rc=$?
  python3 -c "import json; d=json.load(open('gpurun_out/s_${tag}.json')); print('$tag', round(d['ms_per_step'],4), {k:round(v['launch_ms'],4) for k,v in d['roofline']['kernels'].items()})" || { tail -5 gpurun_out/s_${tag}.err; exit 1; }
  [ $rc -eq 0 ] || exit $rc
done
