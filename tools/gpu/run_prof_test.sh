#!/bin/bash
# rocprofv3 kernel-trace summary of one GPU test (TEST=path::name)
cd "$(dirname "$0")/../.."; mkdir -p gpurun_out/proft
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/proft -o run -- python3 -m pytest "$TEST" -m gpu -x -q -s > gpurun_out/proft.log 2>&1
rc=$?; echo "rc=$rc"; grep -E "^C[2345]|passed|failed" gpurun_out/proft.log; exit $rc
