#!/bin/bash
# round 6 C2 diagnosis: k_agg under kbits 10/11/12 and the timing-only knobs (2: no emission, 32: loads only)
cd "$(dirname "$0")/../.."; mkdir -p gpurun_out/r6c2a
run() { tag=$1; shift
  env "$@" timeout -k 10 150 python bench.py --config C2 --steps 20 --warmup 3 --no-cpu --no-ingest > gpurun_out/r6c2a/$tag.log 2>&1 || exit $?
  tail -1 gpurun_out/r6c2a/$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['roofline']['kernels']; print('$tag', round(d['ms_per_step'],4), [round(v['launch_ms'],4) for v in k.values()], flush=True)"
}
run prod X=1
run kb10 EKGPU_KBITS=10
run kb12 EKGPU_KBITS=12
run noemit EKGPU_DEBUG_AGG=2
run loadsonly EKGPU_DEBUG_AGG=34
run prod2 X=1
