#!/bin/bash
# round-4 close: the whole GPU suite, then the bench line of every config (kernel traces of C4a / C5 under gpurun_out/tr)
cd "$(dirname "$0")/../.."; mkdir -p gpurun_out
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4_final_tests.log 2>&1
rc=$?; tail -4 gpurun_out/r4_final_tests.log; [ $rc -eq 0 ] || exit $rc
for c in C2 C3 C4a C4b C5; do
  timeout -k 10 400 python bench.py --config $c --steps 10 --warmup 2 > gpurun_out/final_$c.json 2> gpurun_out/final_$c.err || { tail -5 gpurun_out/final_$c.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/final_$c.json')); print('$c', round(d['ms_per_step'],4), round(d['value']/1e9,2), 'G/s', {k:round(v['launch_ms'],4) for k,v in d['roofline']['kernels'].items()}, d['cpu_baseline']['value'] if d.get('cpu_baseline') else None)"
done
