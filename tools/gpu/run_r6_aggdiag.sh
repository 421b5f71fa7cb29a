#!/bin/bash
# round 6: where k_agg's time goes on C2 (diagnostic knobs of GroupDesc.pad: 2 no emission, 34 loads only, 32 no LDS atomics)
cd "$(dirname "$0")/../.."; mkdir -p gpurun_out/r6diag
run() { tag=$1; cfg=$2; shift; shift
  env "$@" timeout -k 10 200 python bench.py --config $cfg --steps 20 --warmup 3 --no-cpu --no-ingest > gpurun_out/r6diag/$tag.json 2> gpurun_out/r6diag/$tag.err || { tail -3 gpurun_out/r6diag/$tag.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/r6diag/$tag.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$tag', round(d['ms_per_step'],4), round(r.get('device_ms_per_step',0),4), {k[:14]: round(v['launch_ms'],4) for k,v in r.get('kernels',{}).items()}, flush=True)"
}
run base C2 X=1
for kn in 2 34 32; do run dbg$kn C2 EKGPU_DEBUG_AGG=$kn; done
for kb in 10 12; do run kb$kb C2 EKGPU_KBITS=$kb; done
