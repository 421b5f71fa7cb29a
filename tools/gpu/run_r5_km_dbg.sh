#!/bin/bash
# round 5: the key-major order-statistic launch through the E/X merge walk, under the bound-checked debug build
# (EK_KM_CHECK: the first violated bound is reported instead of touched), then the production build's key-major tests.
cd "$(dirname "$0")/../.."; mkdir -p gpurun_out
EKGPU_KM_MERGE_SORT=1 EKGPU_LIB=$PWD/ekuiper-vioneta_amd/build_dbg/libekgpu_dbg.so \
  timeout -k 10 300 python -u -m pytest tests/test_keymajor_gpu.py -x -v --timeout 120 --timeout-method thread \
  -k "median_percentile" > gpurun_out/r5_km_dbg.log 2>&1
rc=$?; tail -30 gpurun_out/r5_km_dbg.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_keymajor_gpu.py tests/test_shared_source_gpu.py tests/test_state_gpu.py -x -q \
  --timeout 120 --timeout-method thread > gpurun_out/r5_km_prod.log 2>&1
rc=$?; tail -5 gpurun_out/r5_km_prod.log; exit $rc
