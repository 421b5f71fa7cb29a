#!/bin/bash
# round 6 C2 A/B: fused sorted pass, key-bucket width (kbits 10 / 11 / 12), nullable-key parity tests
cd "$(dirname "$0")/../.."; mkdir -p gpurun_out/r6c2ab
true
true
run() { tag=$1; cfg=${CFG:-C2}; shift
  env "$@" timeout -k 10 150 python bench.py --config $cfg --steps 20 --warmup 3 --no-cpu --no-ingest > gpurun_out/r6c2ab/$tag.json 2> gpurun_out/r6c2ab/$tag.err || { tail -3 gpurun_out/r6c2ab/$tag.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/r6c2ab/$tag.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$tag', round(d['ms_per_step'],4), round(r['device_ms_per_step'],4), {k[:14]: round(v['launch_ms'],4) for k,v in r.get('kernels',{}).items()}, d['config'].get('fused_sorted_batches_last_step'), flush=True)"
}
run base X=1
run fused EKGPU_FUSED=1
run kb10 EKGPU_KBITS=10
run kb12 EKGPU_KBITS=12
run base2 X=1
run fused2 EKGPU_FUSED=1
CFG=C3 run c3 X=1
for ch in 1 4 8 16; do CFG=C3 run c3ch$ch EKGPU_FIN_RING_CHUNKS=$ch; done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for c in C4a C5; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6c2ab/tr_$c -o run -- python3 bench.py --config $c --steps 5 --warmup 1 --no-cpu --no-ingest > gpurun_out/r6c2ab/tr_$c.log 2>&1 || { echo "$c trace failed"; exit 1; }
done
echo traces done
