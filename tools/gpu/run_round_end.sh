#!/bin/bash
# GPU: every config's bench line (single GPU + --sim-world 8) and the C5 rocprofv3 kernel summary
cd "$(dirname "$0")/../.."; mkdir -p gpurun_out
bash tools/gpu/run_bench_all.sh all || exit 1
bash tools/gpu/prof.sh C5 5
