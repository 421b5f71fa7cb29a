#!/bin/bash
# rocprofv3 kernel-trace summary of a short bench run
cd "$(dirname "$0")/../.."; mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps ${STEPS:-3} --warmup 1 --no-cpu > gpurun_out/prof.log 2>&1
rc=$?; echo "rc=$rc"; tail -3 gpurun_out/prof.log
find gpurun_out/prof -name "*stats*" | head
exit $rc
