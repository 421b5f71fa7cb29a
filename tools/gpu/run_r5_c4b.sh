#!/bin/bash
# round 5 C4a quick: km_msd tests + C4a bench (msd / radix) + C4a kernel stats
cd "$(dirname "$0")/../.."; mkdir -p gpurun_out/c4b
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_keymajor_gpu.py -k "msd or c4a" -x -q --timeout 300 --timeout-method thread > gpurun_out/c4b/tests.log 2>&1
rc=$?; tail -2 gpurun_out/c4b/tests.log; [ $rc -eq 0 ] || exit $rc
run() { tag=$1; cfg=$2; shift 2
  env "$@" timeout -k 10 200 python bench.py --config $cfg --steps 10 --warmup 2 --no-cpu > gpurun_out/c4b/$tag.log 2>&1 || exit $?
  tail -1 gpurun_out/c4b/$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['roofline']['kernels']; print('$tag', round(d['ms_per_step'],4), [round(v['launch_ms'],4) for v in k.values()])"
}
run c4a_msd C4a X=1
run c4a_radix C4a EKGPU_KM_MSD=0
timeout -k 10 -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c4b/trace -o run -- python3 bench.py --config C4a --steps 5 --warmup 1 --no-cpu --no-ingest > gpurun_out/c4b/trace.log 2>&1 || exit $?
grep -E "k_kmsd_fix|k_grp_scatter|k_grp_hist|k_msd_plan|k_km_gather|k_km_keys|rocprim" $(ls gpurun_out/c4b/trace/*kernel_stats.csv | head -1) | cut -c1-60,200-260
