#!/bin/bash
cd "$(dirname "$0")/../.."; mkdir -p gpurun_out
EKGPU_STREAM_PROF=1 timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/bench_sprof.log 2>&1
rc=$?; echo "rc=$rc"; grep "k_stream" gpurun_out/bench_sprof.log | tail -3; grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_sprof.log; exit $rc
