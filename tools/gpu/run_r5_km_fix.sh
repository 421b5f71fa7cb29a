#!/bin/bash
# round 5: key-major order statistics without the in-memory rank counting (runs > kKmSegMax fall back), E / X merge
# walk for every multi-window launch — the key-major suite once, production build
cd "$(dirname "$0")/../.."; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_keymajor_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r5_km_fix.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/r5_km_fix.log | tail -40; exit $rc
