#!/bin/bash
# round-4 evidence: per-config kernel traces + FETCH / WRITE passes (each its own run), the --sim-world 8 passes of the
# shard-mode configs, and the 2-rank rehearsal on one GPU (gloo)
cd "$(dirname "$0")/../.."
CONFIGS="${CONFIGS:-C2 C3 C4a C4b C5}" bash tools/gpu/run_profiles_configs.sh || exit 1
mkdir -p gpurun_out/pcs
export TMPDIR=/tmp
for c in ${SIM_CONFIGS:-C2 C4a C4b}; do
  timeout -k 10 -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pcs/$c/fetch -o run -- python3 bench.py --config $c --sim-world 8 --steps 1 --warmup 1 --no-cpu --no-ingest > gpurun_out/pcs/$c.fetch.log 2>&1 || { echo "$c sim fetch failed"; exit 1; }
  timeout -k 10 -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pcs/$c/write -o run -- python3 bench.py --config $c --sim-world 8 --steps 1 --warmup 1 --no-cpu --no-ingest > gpurun_out/pcs/$c.write.log 2>&1 || { echo "$c sim write failed"; exit 1; }
  echo "$c sim8 done"
done
bash tools/gpu/run_rehearse_ranks.sh
