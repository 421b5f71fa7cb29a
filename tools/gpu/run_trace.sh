#!/bin/bash
# rocprofv3 kernel trace (+ stats) of the default C2 bench: per-kernel durations and inter-kernel gaps
cd "$(dirname "$0")/../.."; mkdir -p gpurun_out/prof
export TMPDIR=/tmp
rm -rf gpurun_out/prof/*
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps ${STEPS:-5} --warmup 2 --no-cpu > gpurun_out/prof.log 2>&1 || exit $?
tail -1 gpurun_out/prof.log | cut -c1-300
