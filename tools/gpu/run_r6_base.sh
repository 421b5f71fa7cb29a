#!/bin/bash
# round 6 (re-entry): the round's new GPU tests, then one bench line per config and a C2 kernel trace on HEAD
cd "$(dirname "$0")/../.."; mkdir -p gpurun_out/r6base
timeout -k 10 400 python -u -m pytest tests/test_fused_gpu.py tests/test_async_gpu.py tests/test_route_gpu.py -x -q \
  --timeout 120 --timeout-method thread > gpurun_out/r6base/tests.log 2>&1
rc=$?; tail -2 gpurun_out/r6base/tests.log; [ $rc -eq 0 ] || exit $rc
for c in C2 C3 C4a C4b C5; do
  timeout -k 10 200 python bench.py --config $c --steps 20 --warmup 3 --no-cpu --no-ingest > gpurun_out/r6base/$c.json 2> gpurun_out/r6base/$c.err || { tail -5 gpurun_out/r6base/$c.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/r6base/$c.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$c', round(d['ms_per_step'],4), 'frac', round(r['frac'],4), {k[:14]: round(v['launch_ms'],4) for k,v in r.get('kernels',{}).items()}, flush=True)"
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r6base/prof_c2 -o run -- python3 bench.py --config C2 --steps 10 --warmup 2 --no-cpu --no-ingest > gpurun_out/r6base/prof_c2.log 2>&1 || exit 1
find gpurun_out/r6base/prof_c2 -name "*kernel_stats.csv" | head -1 | xargs -I{} sh -c 'head -12 {}'
# k_agg diagnosis: no emission (2), loads only + no emission (34), no LDS atomics but emission (32)
for kn in 2 34 32; do
  EKGPU_DEBUG_AGG=$kn timeout -k 10 150 python bench.py --config C2 --steps 20 --warmup 3 --no-cpu --no-ingest > gpurun_out/r6base/dbg$kn.json 2> gpurun_out/r6base/dbg$kn.err || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/r6base/dbg$kn.json').read().strip().splitlines()[-1]); r=d['roofline']; print('dbg$kn', round(d['ms_per_step'],4), {k[:14]: round(v['launch_ms'],4) for k,v in r.get('kernels',{}).items()}, flush=True)"
done
