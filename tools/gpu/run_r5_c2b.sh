#!/bin/bash
# round 5 C2 study: k_agg time split by the diagnostic knobs (32: loads only; 2: no emission; 34: both)
cd "$(dirname "$0")/../.."; mkdir -p gpurun_out/c2b
for k in 0 32 2 34; do
  EKGPU_VARIANT=1 EKGPU_DEBUG_AGG=$k timeout -k 10 150 python bench.py --config C2 --steps 20 --warmup 3 --no-cpu > gpurun_out/c2b/k_$k.log 2>&1 || exit $?
  tail -1 gpurun_out/c2b/k_$k.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['roofline']['kernels']; print('knob $k', round(d['ms_per_step'],4), [round(v['launch_ms'],4) for v in k.values()])"
done
