#!/bin/bash
# per-config rocprofv3 kernel stats + PMC passes, then the shard-mode path on one GPU (--sim-world 8: rank 0 of 8)
cd "$(dirname "$0")/../.."; mkdir -p gpurun_out/dev
CONFIGS="${CONFIGS:-C2 C3 C4a C4b C5 C1}" bash tools/gpu/run_profiles_configs.sh || exit $?
for c in C2 C4a C5; do
  timeout -k 10 300 python bench.py --config $c --sim-world 8 --no-cpu --no-ingest --steps 5 --warmup 2 > gpurun_out/dev/${c}_sim8.json 2> gpurun_out/dev/${c}_sim8.err || { echo "$c sim8 failed"; tail -5 gpurun_out/dev/${c}_sim8.err; exit 1; }
  cut -c1-220 gpurun_out/dev/${c}_sim8.json
done
