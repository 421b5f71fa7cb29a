#!/bin/bash
# round 6: k_agg at 5 waves per EU (tuning build, EKGPU_LIB) against the shipped 6, with k_agg<NUL = false> — C2 / C3, 3x
cd "$(dirname "$0")/../.."; mkdir -p gpurun_out/r6w5
L5=$PWD/ekuiper-vioneta_amd/build_v_w5/libekgpu.so
run() { tag=$1; cfg=$2; shift; shift
  env "$@" timeout -k 10 200 python bench.py --config $cfg --steps 20 --warmup 3 --no-cpu --no-ingest > gpurun_out/r6w5/$tag.json 2> gpurun_out/r6w5/$tag.err || { tail -3 gpurun_out/r6w5/$tag.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/r6w5/$tag.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$tag', round(d['ms_per_step'],4), {k[:14]: round(v['launch_ms'],4) for k,v in r.get('kernels',{}).items()}, flush=True)"
}
for i in 1 2 3; do
  run c2_w6_$i C2 X=1
  run c2_w5_$i C2 EKGPU_LIB=$L5
done
run c3_w6 C3 X=1
run c3_w5 C3 EKGPU_LIB=$L5
