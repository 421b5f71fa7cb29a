#!/bin/bash
# round-6 bench lines of every config (traffic from the committed profiles/r06_pmc_<cfg>.json) -> gpurun_out/r6bench
cd "$(dirname "$0")/../.."; mkdir -p gpurun_out/r6bench
: > gpurun_out/r6bench/bench.jsonl
for c in ${CONFIGS:-C2 C3 C4a C4b C5 C1}; do
  timeout -k 10 400 python bench.py --config $c --steps 20 --warmup 3 > gpurun_out/r6bench/$c.json 2> gpurun_out/r6bench/$c.err || { tail -5 gpurun_out/r6bench/$c.err; exit 1; }
  tail -1 gpurun_out/r6bench/$c.json >> gpurun_out/r6bench/bench.jsonl
  python3 -c "import json; d=json.loads(open('gpurun_out/r6bench/$c.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$c', round(d['ms_per_step'],4), round(d['value']/1e9,3), 'G/s frac', round(r['frac'],4), 'traffic', r.get('traffic'), r.get('traffic_source'), 'cpu', d.get('cpu_baseline',{}).get('value'), flush=True)"
done
timeout -k 10 300 python bench.py > gpurun_out/r6bench/default.json 2> gpurun_out/r6bench/default.err || exit 1
tail -1 gpurun_out/r6bench/default.json | cut -c1-300
