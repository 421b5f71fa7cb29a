#!/bin/bash
# round-5 bench lines of every config (traffic from the committed profiles/r05_pmc_<cfg>.json) -> gpurun_out/r5bench
cd "$(dirname "$0")/../.."; mkdir -p gpurun_out/r5bench
: > gpurun_out/r5bench/bench.jsonl
for c in ${CONFIGS:-C2 C3 C4a C4b C5 C1}; do
  timeout -k 10 400 python bench.py --config $c --steps 20 --warmup 3 > gpurun_out/r5bench/$c.json 2> gpurun_out/r5bench/$c.err || { tail -5 gpurun_out/r5bench/$c.err; exit 1; }
  tail -1 gpurun_out/r5bench/$c.json >> gpurun_out/r5bench/bench.jsonl
  python3 -c "import json; d=json.load(open('gpurun_out/r5bench/$c.json')); r=d['roofline']; print('$c', round(d['ms_per_step'],4), round(d['value']/1e9,3), 'G/s frac', round(r['frac'],4), 'traffic', r.get('traffic'), r.get('traffic_source'), {k: (round(v['launch_ms'],4), round(v['achieved_gbs'] or 0)) for k,v in r.get('kernels',{}).items()})"
done
timeout -k 10 300 python bench.py > gpurun_out/r5bench/default.json 2> gpurun_out/r5bench/default.err || exit 1
tail -1 gpurun_out/r5bench/default.json
