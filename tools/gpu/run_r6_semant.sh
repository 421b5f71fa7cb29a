#!/bin/bash
# round 6: state-window WHERE pushdown + nullable-key parity (GPU), then the C2 / C3 A/B and C4a / C5 traces
cd "$(dirname "$0")/../.."; mkdir -p gpurun_out/r6sem
timeout -k 10 400 python -u -m pytest tests/test_state_window_gpu.py tests/test_group_keys.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r6sem/tests.log 2>&1
rc=$?; tail -3 gpurun_out/r6sem/tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu/run_r6_c2ab.sh
