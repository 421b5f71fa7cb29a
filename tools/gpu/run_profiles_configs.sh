#!/bin/bash
# rocprofv3 kernel stats + FETCH_SIZE / WRITE_SIZE passes per BASELINE config (each pass its own run)
cd "$(dirname "$0")/../.."; mkdir -p gpurun_out/pc
export TMPDIR=/tmp
for c in ${CONFIGS:-C2 C3 C4a C4b C5}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pc/$c/trace -o run -- python3 bench.py --config $c --steps 5 --warmup 1 --no-cpu --no-ingest > gpurun_out/pc/$c.trace.log 2>&1 || { echo "$c trace failed"; tail -3 gpurun_out/pc/$c.trace.log; exit 1; }
  timeout -k 10 -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pc/$c/fetch -o run -- python3 bench.py --config $c --steps 1 --warmup 1 --no-cpu --no-ingest > gpurun_out/pc/$c.fetch.log 2>&1 || { echo "$c fetch failed"; exit 1; }
  timeout -k 10 -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pc/$c/write -o run -- python3 bench.py --config $c --steps 1 --warmup 1 --no-cpu --no-ingest > gpurun_out/pc/$c.write.log 2>&1 || { echo "$c write failed"; exit 1; }
  echo "$c done"
done
