#!/bin/bash
# k_agg waves-per-EU A/B (6 = the shipped build, 5 / 4 = tuning builds via EKGPU_LIB): C2 and C3 -> gpurun_out/r5wpe
cd "$(dirname "$0")/../.."; mkdir -p gpurun_out/r5wpe
for v in base w5 w4; do
  lib=""; [ $v != base ] && lib=$PWD/ekuiper-vioneta_amd/build_v_$v/libekgpu.so
  for c in C2 C3; do
    EKGPU_LIB=$lib timeout -k 10 200 python bench.py --config $c --steps 20 --warmup 3 --no-cpu --no-ingest > gpurun_out/r5wpe/${c}_$v.json 2> gpurun_out/r5wpe/${c}_$v.err || { tail -3 gpurun_out/r5wpe/${c}_$v.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/r5wpe/${c}_$v.json')); r=d['roofline']; print('$c $v', round(d['ms_per_step'],4), {k[:12]: round(v['launch_ms'],4) for k,v in r.get('kernels',{}).items()})"
  done
done
