#!/bin/bash
# round 6: k_finalize_ring prefetch depth A/B (EK_RING_AHEAD 3 shipped vs 8 in build_v_ahead8), C3 parity with the variant
cd "$(dirname "$0")/../.."; mkdir -p gpurun_out/r6ring
V=$PWD/ekuiper-vioneta_amd/build_v_ahead8/libekgpu.so
EKGPU_LIB=$V timeout -k 10 400 python -u -m pytest tests/test_fullsize_parity_gpu.py -k "c3" tests/test_hopping_gap.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6ring/tests.log 2>&1
rc=$?; tail -3 gpurun_out/r6ring/tests.log; [ $rc -eq 0 ] || exit $rc
run() { tag=$1; cfg=$2; shift; shift
  env "$@" timeout -k 10 200 python bench.py --config $cfg --steps 20 --warmup 3 --no-cpu --no-ingest > gpurun_out/r6ring/$tag.json 2> gpurun_out/r6ring/$tag.err || { tail -3 gpurun_out/r6ring/$tag.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/r6ring/$tag.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$tag', round(d['ms_per_step'],4), round(r.get('device_ms_per_step',0),4), {k[:14]: round(v['launch_ms'],4) for k,v in r.get('kernels',{}).items()}, flush=True)"
}
run base C3 X=1
run ahead8 C3 EKGPU_LIB=$V
run ahead8_ch4 C3 EKGPU_LIB=$V EKGPU_FIN_RING_CHUNKS=4
run base_ch4 C3 EKGPU_FIN_RING_CHUNKS=4
run base_ch1 C3 EKGPU_FIN_RING_CHUNKS=1
run base2 C3 X=1
run ahead8_2 C3 EKGPU_LIB=$V
