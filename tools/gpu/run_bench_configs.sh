#!/bin/bash
# GPU: bench line per BASELINE config (N=1), the shard-mode path (--sim-world 8, rank 0) and the default C2 line
cd "$(dirname "$0")/../.."; mkdir -p gpurun_out/bench
for c in C2 C3 C4a C4b C5; do
  timeout -k 10 300 python bench.py --config $c --steps ${STEPS:-10} --warmup 2 --no-cpu --no-ingest > gpurun_out/bench/$c.json 2> gpurun_out/bench/$c.err
  rc=$?; echo "$c rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench/$c.json) $(grep -o '"frac": [0-9.]*' gpurun_out/bench/$c.json | head -1)"
  [ $rc -eq 0 ] || { tail -5 gpurun_out/bench/$c.err; exit $rc; }
done
for c in C2 C4a C4b; do
  timeout -k 10 300 python bench.py --config $c --sim-world 8 --steps 5 --warmup 2 --no-cpu > gpurun_out/bench/${c}_sim8.json 2> gpurun_out/bench/${c}_sim8.err
  rc=$?; echo "$c sim8 rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench/${c}_sim8.json)"
  [ $rc -eq 0 ] || { tail -5 gpurun_out/bench/${c}_sim8.err; exit $rc; }
done
timeout -k 10 400 python bench.py > gpurun_out/bench/default.json 2> gpurun_out/bench/default.err
rc=$?; echo "default rc=$rc"; cut -c1-300 gpurun_out/bench/default.json; exit $rc
