#!/bin/bash
# round 6: kernel traces of C5 / C4a / C3 on HEAD (top kernels per config)
cd "$(dirname "$0")/../.."; mkdir -p gpurun_out/r6tr
export TMPDIR=/tmp
for c in ${CONFIGS:-C5 C4a C3}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6tr/$c -o run -- python3 bench.py --config $c --steps 5 --warmup 1 --no-cpu --no-ingest > gpurun_out/r6tr/$c.log 2>&1 || { echo "$c trace failed"; tail -3 gpurun_out/r6tr/$c.log; exit 1; }
  f=$(find gpurun_out/r6tr/$c -name "*kernel_stats.csv" | head -1)
  python3 -c "
import csv; rows=list(csv.DictReader(open('$f')))
rows.sort(key=lambda r: -float(r['TotalDurationNs']))
for r in rows[:14]: print('$c', r['Name'][:60], r['Calls'], round(float(r['TotalDurationNs'])/6e6,4), 'ms/step', round(float(r['AverageNs'])/1e3,1), 'us avg')
"
done
