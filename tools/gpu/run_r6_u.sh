#!/bin/bash
# round 6: k_agg rows in flight per lane (EK_AGG_U 8 shipped vs 4 / 6 tuning builds via EKGPU_LIB), C2 / C3, twice each
cd "$(dirname "$0")/../.."; mkdir -p gpurun_out/r6u
L4=$PWD/ekuiper-vioneta_amd/build_v_u4/libekgpu.so; L6=$PWD/ekuiper-vioneta_amd/build_v_u6/libekgpu.so
run() { tag=$1; cfg=$2; shift; shift
  env "$@" timeout -k 10 200 python bench.py --config $cfg --steps 20 --warmup 3 --no-cpu --no-ingest > gpurun_out/r6u/$tag.json 2> gpurun_out/r6u/$tag.err || { tail -3 gpurun_out/r6u/$tag.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/r6u/$tag.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$tag', round(d['ms_per_step'],4), round(r.get('device_ms_per_step',0),4), {k[:14]: round(v['launch_ms'],4) for k,v in r.get('kernels',{}).items()}, flush=True)"
}
for i in 1 2; do
  run c2_u8_$i C2 X=1
  run c2_u4_$i C2 EKGPU_LIB=$L4
  run c2_u6_$i C2 EKGPU_LIB=$L6
done
run c3_u8 C3 X=1
run c3_u4 C3 EKGPU_LIB=$L4
run c3_u6 C3 EKGPU_LIB=$L6
