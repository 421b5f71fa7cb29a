#!/bin/bash
# round 5 C2 study: key-bucket width sweep (k_agg grid / LDS per block), k_part without global stores (knob 8)
cd "$(dirname "$0")/../.."; mkdir -p gpurun_out/c2c
run() { tag=$1; shift
  env "$@" timeout -k 10 150 python bench.py --config C2 --steps 20 --warmup 3 --no-cpu > gpurun_out/c2c/$tag.log 2>&1 || exit $?
  tail -1 gpurun_out/c2c/$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['roofline']['kernels']; print('$tag', round(d['ms_per_step'],4), [round(v['launch_ms'],4) for v in k.values()])"
}
run kb11 EKGPU_VARIANT=1 EKGPU_KBITS=11
run kb10 EKGPU_VARIANT=1 EKGPU_KBITS=10
run kb9 EKGPU_VARIANT=1 EKGPU_KBITS=9
run kb12 EKGPU_VARIANT=1 EKGPU_KBITS=12
run part_nostore EKGPU_VARIANT=1 EKGPU_DEBUG_AGG=8
