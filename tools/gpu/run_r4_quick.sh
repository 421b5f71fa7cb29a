#!/bin/bash
# quick bench lines: CONFIGS (default C3 C4b) with ENVS variants; prints ms/step and per-kernel launch times
cd "$(dirname "$0")/../.."; mkdir -p gpurun_out
for cfg in ${CONFIGS:-C3 C4b}; do
  for env in ${ENVS:-X=0}; do
    tag=$(echo "$env" | tr '/=' '__' | tail -c 40)
    env $env timeout -k 10 300 python bench.py --config $cfg --steps 10 --warmup 2 --no-cpu > gpurun_out/q_${cfg}_${tag}.json 2> gpurun_out/q_${cfg}_${tag}.err
    rc=$?
    python3 -c "import json; d=json.load(open('gpurun_out/q_${cfg}_${tag}.json')); print('$cfg $env', round(d['ms_per_step'],4), {k:round(v['launch_ms'],4) for k,v in d['roofline']['kernels'].items()})" || { tail -5 gpurun_out/q_${cfg}_${tag}.err; exit 1; }
    [ $rc -eq 0 ] || exit $rc
  done
done
