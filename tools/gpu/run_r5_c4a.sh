#!/bin/bash
# round 5 C4a: the key-major span sort by MSD partition (km_msd) — key-major / range / full-size parity, then the
# C4a and C5 benches with km_msd on and off, and the C4a kernel trace
cd "$(dirname "$0")/../.."; mkdir -p gpurun_out/c4a
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_keymajor_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/c4a/tests_km.log 2>&1
rc=$?; tail -3 gpurun_out/c4a/tests_km.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_range_gpu.py tests/test_fullsize_parity_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/c4a/tests_range.log 2>&1
rc=$?; tail -3 gpurun_out/c4a/tests_range.log; [ $rc -eq 0 ] || exit $rc
run() { tag=$1; cfg=$2; shift 2
  env "$@" timeout -k 10 200 python bench.py --config $cfg --steps 10 --warmup 2 --no-cpu > gpurun_out/c4a/$tag.log 2>&1 || exit $?
  tail -1 gpurun_out/c4a/$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['roofline']['kernels']; print('$tag', round(d['ms_per_step'],4), [round(v['launch_ms'],4) for v in k.values()])"
}
run c4a_msd C4a X=1
run c4a_radix C4a EKGPU_KM_MSD=0
run c4a_msd2 C4a X=1
run c5 C5 X=1
timeout -k 10 -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c4a/trace -o run -- python3 bench.py --config C4a --steps 5 --warmup 1 --no-cpu --no-ingest > gpurun_out/c4a/trace.log 2>&1 || exit $?
head -25 $(ls gpurun_out/c4a/trace/*kernel_stats.csv | head -1) | cut -c1-150
