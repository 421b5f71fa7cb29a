#!/bin/bash
# GPU: grouping / range / state parity, full-size C5 + C4 parity, then C5 bench lines (fused append on / off)
cd "$(dirname "$0")/../.."; mkdir -p gpurun_out
TESTS="tests/test_sharding_gpu.py tests/test_keymajor_gpu.py tests/test_range_gpu.py tests/test_state_gpu.py tests/test_fullsize_parity_gpu.py" \
  TLIMIT=700 bash tools/gpu/run_tests.sh || exit 1
for f in 1 0; do
  EKGPU_APPEND_FUSED=$f timeout -k 10 240 python -u bench.py --config C5 --steps 10 --no-cpu > gpurun_out/c5_app$f.json 2> gpurun_out/c5_app$f.err || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/c5_app$f.json').read().strip().splitlines()[-1]);print('C5 fused=$f', round(d['ms_per_step'],3))"
done
