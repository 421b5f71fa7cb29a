#!/bin/bash
# A/B of two engine builds in one box (EKGPU_LIB = the alternative .so): C2 bench, alternating, per-phase times.
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
for i in 1 2 3; do
  for v in prev new; do
    if [ $v = prev ]; then export EKGPU_LIB=$PWD/build/libekgpu_prev.so; else unset EKGPU_LIB; fi
    timeout -k 10 150 python bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/ab_${v}_$i.log 2>&1 || exit $?
    tail -1 gpurun_out/ab_${v}_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$v', round(d['ms_per_step'],4), {k: round(x,4) for k,x in r['phase_ms_per_step'].items()})"
  done
done
