#!/bin/bash
# C3 register-ring finalize: hopping parity (KATs, pane-mode engine tests, full-size C3), then the C3 bench line with
# the ring and with k_finalize (EKGPU_FIN_RING=0), and the kernel profile
cd "$(dirname "$0")/../.."; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py tests/test_window_error_gpu.py tests/test_state_gpu.py \
  "tests/test_fullsize_parity_gpu.py::test_c3_shard_full_parity" -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r4_c3_tests.log 2>&1
rc=$?; tail -6 gpurun_out/r4_c3_tests.log; [ $rc -eq 0 ] || exit $rc
for ring in 1 0; do
  EKGPU_FIN_RING=$ring timeout -k 10 300 python bench.py --config C3 --steps 10 --warmup 2 --no-cpu > gpurun_out/r4_c3_ring$ring.json 2> gpurun_out/r4_c3_ring$ring.err
  rc=$?; python3 -c "import json,sys; d=json.load(open('gpurun_out/r4_c3_ring$ring.json')); print('ring=$ring', d['ms_per_step'], {k:(v['launch_ms'],v['launches_per_step']) for k,v in d['roofline']['kernels'].items()})" || { tail -5 gpurun_out/r4_c3_ring$ring.err; exit 1; }
  [ $rc -eq 0 ] || exit $rc
done
bash tools/gpu/prof.sh C3 5
