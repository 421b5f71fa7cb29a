#!/bin/bash
# shared-source ts statistics: parity tests, then C5 with and without the shared pass (alternating)
cd "$(dirname "$0")/../.."; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_shared_source_gpu.py tests/test_engine_gpu.py tests/test_processing_gpu.py \
  -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4_shared_tests.log 2>&1
rc=$?; tail -6 gpurun_out/r4_shared_tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for flag in "" "--no-shared-stats"; do
    tag="rep${rep}${flag:+_noshare}"
    timeout -k 10 300 python bench.py --config C5 --steps 10 --warmup 2 --no-cpu $flag > gpurun_out/s_C5_${tag}.json 2> gpurun_out/s_C5_${tag}.err
    rc=$?
    python3 -c "import json; d=json.load(open('gpurun_out/s_C5_${tag}.json')); print('C5 $tag', round(d['ms_per_step'],4), {k:round(v['launch_ms'],4) for k,v in d['roofline']['kernels'].items()})" || { tail -5 gpurun_out/s_C5_${tag}.err; exit 1; }
    [ $rc -eq 0 ] || exit $rc
  done
done
