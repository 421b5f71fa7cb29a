#!/bin/bash
# Bench lines of every config on one GPU (with their CPU baselines) -> gpurun_out/r03_bench/<cfg>.json; then the
# shard-mode lines (--sim-world 8: rank 0 of an 8-GPU run, analytic global watermark) -> <cfg>_sim8.json.
# Usage: run_bench_all.sh [single|sim8|all]
cd "$(dirname "$0")/../.."
mode=${1:-all}
out=gpurun_out/r03_bench
mkdir -p $out
if [ "$mode" != "sim8" ]; then
    for cfg in C2 C3 C4a C4b C5 C1; do
        timeout -k 10 400 python -u bench.py --config $cfg --steps 10 --warmup 3 > $out/$cfg.txt 2>&1 || { echo "$cfg failed"; exit 1; }
        grep '"metric"' $out/$cfg.txt > $out/$cfg.json
        python3 -c "import json; d=json.load(open('$out/$cfg.json')); print('$cfg', round(d['ms_per_step'],3), 'ms', '%.3g'%d['value'], d['unit'], 'frac', round(d['roofline']['frac'],3), 'cpu', '%.3g'%d.get('cpu_baseline',{}).get('value',0))"
    done
    timeout -k 10 300 python -u bench.py --config C2 --disorder 50 --steps 10 --no-cpu > $out/C2_disorder50.txt 2>&1 && grep '"metric"' $out/C2_disorder50.txt > $out/C2_disorder50.json
fi
if [ "$mode" != "single" ]; then
    for cfg in C2 C3 C4a C4b C5; do
        timeout -k 10 400 python -u bench.py --config $cfg --sim-world 8 --steps 5 --warmup 2 --no-cpu --no-ingest > $out/${cfg}_sim8.txt 2>&1 || { echo "$cfg sim8 failed"; exit 1; }
        grep '"metric"' $out/${cfg}_sim8.txt > $out/${cfg}_sim8.json
        python3 -c "import json; d=json.load(open('$out/${cfg}_sim8.json')); print('$cfg sim8', round(d['ms_per_step'],3), 'ms rank0', d['config']['events_rank0'])"
    done
fi
