#!/bin/bash
# kernel-trace stats only, per CONFIGS (ENV applied to the bench)
cd "$(dirname "$0")/../.."; mkdir -p gpurun_out/tr
export TMPDIR=/tmp
for c in ${CONFIGS:-C4a}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/tr/$c -o run -- python3 bench.py --config $c --steps 5 --warmup 1 --no-cpu --no-ingest > gpurun_out/tr/$c.log 2>&1 || { echo "$c trace failed"; tail -3 gpurun_out/tr/$c.log; exit 1; }
  f=$(ls gpurun_out/tr/$c/*kernel_stats.csv 2>/dev/null | head -1); [ -z "$f" ] && f=$(find gpurun_out/tr/$c -name '*kernel_stats.csv' | head -1)
  python3 -c "
import csv,sys
r=list(csv.DictReader(open('$f')))
for x in r[:14]: print('$c', x['Name'][:70], x['Calls'], round(float(x['AverageNs'])/1e3,1), 'us', x['Percentage'])
"
done
