#!/bin/bash
# round 6: nontemporal staging stores / loads (EKGPU_VARIANT bits 1 / 2) on C2 / C3, nontemporal event-buffer append
# (EKGPU_EB_NT) on C5 / C4a — A/B, each twice; then the pane-mode suites with the knobs on (parity must not change)
cd "$(dirname "$0")/../.."; mkdir -p gpurun_out/r6nt
run() { tag=$1; cfg=$2; shift; shift
  env "$@" timeout -k 10 200 python bench.py --config $cfg --steps 20 --warmup 3 --no-cpu --no-ingest > gpurun_out/r6nt/$tag.json 2> gpurun_out/r6nt/$tag.err || { tail -3 gpurun_out/r6nt/$tag.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/r6nt/$tag.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$tag', round(d['ms_per_step'],4), round(r.get('device_ms_per_step',0),4), {k[:14]: round(v['launch_ms'],4) for k,v in r.get('kernels',{}).items()}, flush=True)"
}
for i in 1 2; do
  run c2_base$i C2 X=1
  run c2_ntst$i C2 EKGPU_VARIANT=2
  run c2_ntld$i C2 EKGPU_VARIANT=4
  run c2_ntboth$i C2 EKGPU_VARIANT=6
done
run c3_base C3 X=1
run c3_ntboth C3 EKGPU_VARIANT=6
for i in 1 2; do
  run c5_base$i C5 X=1
  run c5_ebnt$i C5 EKGPU_EB_NT=1
done
run c4a_base C4a X=1
run c4a_ebnt C4a EKGPU_EB_NT=1
EKGPU_VARIANT=6 EKGPU_EB_NT=1 timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py tests/test_fused_gpu.py tests/test_state_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r6nt/tests.log 2>&1
rc=$?; tail -2 gpurun_out/r6nt/tests.log; exit $rc
