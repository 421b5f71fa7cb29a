#!/bin/bash
# round 6: phase events sampled in the bench (ek_set_phase_timing, one timed step in 4) — engine / async suites, then
# C2 / C3 / C4a / C5 lines with the per-kernel fields
cd "$(dirname "$0")/../.."; mkdir -p gpurun_out/r6samp
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py tests/test_async_gpu.py tests/test_fused_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r6samp/tests.log 2>&1
rc=$?; tail -2 gpurun_out/r6samp/tests.log; [ $rc -eq 0 ] || exit $rc
for c in C2 C3 C2 C3 C4a C5; do
  timeout -k 10 200 python bench.py --config $c --steps 20 --warmup 3 --no-cpu --no-ingest > gpurun_out/r6samp/$c.json 2> gpurun_out/r6samp/$c.err || { tail -3 gpurun_out/r6samp/$c.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/r6samp/$c.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$c', round(d['ms_per_step'],4), round(r['frac'],4), r['dominant_kernel'], {k[:14]: (round(v['launch_ms'],4), v['launches_per_step']) for k,v in r.get('kernels',{}).items()}, flush=True)"
done
