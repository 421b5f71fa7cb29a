#!/bin/bash
# round 6: fused event-buffer append (k_eb_copy) + LDS-staged k_msd_plan2 — range / key-major / sharding / state tests,
# then C4a / C5 bench and a C5 kernel trace
cd "$(dirname "$0")/../.."; mkdir -p gpurun_out/r6app
timeout -k 10 900 python -u -m pytest tests/test_range_gpu.py tests/test_keymajor_gpu.py tests/test_state_gpu.py tests/test_sharding_gpu.py \
  -x -q --timeout 300 --timeout-method thread > gpurun_out/r6app/tests.log 2>&1
rc=$?; tail -3 gpurun_out/r6app/tests.log; [ $rc -eq 0 ] || exit $rc
run() { tag=$1; cfg=$2; shift; shift
  env "$@" timeout -k 10 200 python bench.py --config $cfg --steps 20 --warmup 3 --no-cpu --no-ingest > gpurun_out/r6app/$tag.json 2> gpurun_out/r6app/$tag.err || { tail -3 gpurun_out/r6app/$tag.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/r6app/$tag.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$tag', round(d['ms_per_step'],4), round(r['device_ms_per_step'],4), {k[:14]: round(v['launch_ms'],4) for k,v in r.get('kernels',{}).items()}, flush=True)"
}
run c5 C5 X=1
run c4a C4a X=1
run c3ch4 C3 EKGPU_FIN_RING_CHUNKS=4
run c3 C3 X=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6app/tr_C5 -o run -- python3 bench.py --config C5 --steps 5 --warmup 1 --no-cpu --no-ingest > gpurun_out/r6app/tr_C5.log 2>&1 || { echo "C5 trace failed"; exit 1; }
echo traces done
