#!/bin/bash
# round-5 evidence per config: bench line (with the CPU baseline), rocprofv3 kernel trace + stats, FETCH_SIZE and
# WRITE_SIZE passes (each its own run) -> gpurun_out/r5prof/<cfg>/...; profiles written by tools/profile_configs.py
cd "$(dirname "$0")/../.."; mkdir -p gpurun_out/r5prof
export TMPDIR=/tmp
for c in ${CONFIGS:-C2}; do
  d=gpurun_out/r5prof/$c; mkdir -p $d
  timeout -k 10 400 python bench.py --config $c --steps 20 --warmup 3 > $d/bench.json 2> $d/bench.err || { tail -5 $d/bench.err; exit 1; }
  python3 -c "import json; d=json.load(open('$d/bench.json')); print('$c', round(d['ms_per_step'],4), round(d['value']/1e9,3), 'G/s frac', round(d['roofline']['frac'],4))"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $d/trace -o run -- python3 bench.py --config $c --steps 5 --warmup 1 --no-cpu --no-ingest > $d/trace.log 2>&1 || { echo "$c trace failed"; tail -3 $d/trace.log; exit 1; }
  timeout -k 10 -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $d/fetch -o run -- python3 bench.py --config $c --steps 1 --warmup 1 --no-cpu --no-ingest > $d/fetch.log 2>&1 || { echo "$c fetch failed"; exit 1; }
  timeout -k 10 -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $d/write -o run -- python3 bench.py --config $c --steps 1 --warmup 1 --no-cpu --no-ingest > $d/write.log 2>&1 || { echo "$c write failed"; exit 1; }
  echo "$c done"
done
