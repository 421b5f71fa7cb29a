#!/bin/bash
# round 6: the cost of the engine's per-phase HIP events (EKGPU_PHASE_EVENTS=0 drops them) — C2 / C3 / C4a / C5, A/B twice
cd "$(dirname "$0")/../.."; mkdir -p gpurun_out/r6phev
run() { tag=$1; cfg=$2; shift; shift
  env "$@" timeout -k 10 200 python bench.py --config $cfg --steps 20 --warmup 3 --no-cpu --no-ingest > gpurun_out/r6phev/$tag.json 2> gpurun_out/r6phev/$tag.err || { tail -3 gpurun_out/r6phev/$tag.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/r6phev/$tag.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$tag', round(d['ms_per_step'],4), round(r.get('device_ms_per_step',0),4), flush=True)"
}
for i in 1 2; do
  for c in C2 C3 C4a C5; do
    run ${c}_ev$i $c X=1
    run ${c}_noev$i $c EKGPU_PHASE_EVENTS=0
  done
done
