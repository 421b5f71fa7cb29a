#!/bin/bash
# bench sweep over engine tuning knobs (env), 5 timed steps each; prints ms/step and per-phase ms
cd "$(dirname "$0")/../.."; mkdir -p gpurun_out
for cfg in "$@"; do
  env $cfg timeout -k 10 200 python3 bench.py --steps ${STEPS:-5} --warmup 2 --no-cpu > gpurun_out/sweep.log 2>&1 || exit $?
  echo "$cfg $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/sweep.log) $(grep -o '"phase_ms_per_step": {[^}]*}' gpurun_out/sweep.log)" | tee -a gpurun_out/sweep_all.log
done
