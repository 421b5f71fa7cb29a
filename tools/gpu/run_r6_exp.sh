#!/bin/bash
# round 6: k_km_expand with LDS-gathered flushes + k_finalize_ring's deferred reservation — key-major / range / state suites + full-size C4a parity, C4a bench, C4a WRITE_SIZE
cd "$(dirname "$0")/../.."; mkdir -p gpurun_out/r6exp
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_keymajor_gpu.py tests/test_range_gpu.py tests/test_nullable_median_gpu.py tests/test_engine_gpu.py tests/test_hopping_gap.py tests/test_window_error_gpu.py tests/test_late_tolerance_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6exp/tests.log 2>&1
rc=$?; tail -3 gpurun_out/r6exp/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_fullsize_parity_gpu.py -k "c4a or c3" -x -q --timeout 300 --timeout-method thread > gpurun_out/r6exp/full.log 2>&1
rc=$?; tail -3 gpurun_out/r6exp/full.log; [ $rc -eq 0 ] || exit $rc
for c in C3 C3; do
  timeout -k 10 200 python bench.py --config $c --steps 20 --warmup 3 --no-cpu --no-ingest > gpurun_out/r6exp/c3.json 2> gpurun_out/r6exp/c3.err || { tail -3 gpurun_out/r6exp/c3.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/r6exp/c3.json').read().strip().splitlines()[-1]); r=d['roofline']; print('c3', round(d['ms_per_step'],4), round(r.get('device_ms_per_step',0),4), {k[:14]: round(v['launch_ms'],4) for k,v in r.get('kernels',{}).items()}, flush=True)"
done
for t in a b; do
  timeout -k 10 200 python bench.py --config C4a --steps 20 --warmup 3 --no-cpu --no-ingest > gpurun_out/r6exp/c4a_$t.json 2> gpurun_out/r6exp/c4a_$t.err || { tail -3 gpurun_out/r6exp/c4a_$t.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/r6exp/c4a_$t.json').read().strip().splitlines()[-1]); r=d['roofline']; print('c4a', round(d['ms_per_step'],4), round(r.get('device_ms_per_step',0),4), flush=True)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6exp/tr -o run -- python3 bench.py --config C4a --steps 5 --warmup 1 --no-cpu --no-ingest > gpurun_out/r6exp/tr.log 2>&1 || { echo "trace failed"; exit 1; }
f=$(find gpurun_out/r6exp/tr -name "*kernel_stats.csv" | head -1); grep -E "k_km_expand|k_km_walk" $f | cut -c1-200
timeout -k 10 -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/r6exp/write -o run -- python3 bench.py --config C4a --steps 1 --warmup 1 --no-cpu --no-ingest > gpurun_out/r6exp/write.log 2>&1 || { echo "write pmc failed"; exit 1; }
python3 - <<'PY'
import csv, glob, collections
s = collections.defaultdict(float)
for f in glob.glob('gpurun_out/r6exp/write/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if 'k_km_expand' in r['Kernel_Name']: s[r['Counter_Name']] += float(r['Counter_Value'])
print('k_km_expand WRITE_SIZE bytes per step', {k: v * 1024 / 2 for k, v in s.items()})
PY
