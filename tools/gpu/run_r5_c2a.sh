#!/bin/bash
# round 5 C2 study: HBM ceilings (mb_stream), k_agg XCD-order A/B (EKGPU_VARIANT=1), FETCH per kernel for both
cd "$(dirname "$0")/../.."; mkdir -p gpurun_out/c2a
export TMPDIR=/tmp
timeout -k 10 60 ./tools/mb_stream > gpurun_out/c2a/mb_stream.txt 2>&1 || exit $?
cat gpurun_out/c2a/mb_stream.txt
for i in 1 2; do
  for v in 0 1; do
    EKGPU_VARIANT=$v timeout -k 10 150 python bench.py --config C2 --steps 20 --warmup 3 --no-cpu > gpurun_out/c2a/ab_${v}_$i.log 2>&1 || exit $?
    tail -1 gpurun_out/c2a/ab_${v}_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('v$v', round(d['ms_per_step'],4), {k: round(x,4) for k,x in r['phase_ms_per_step'].items()})"
  done
done
for v in 0 1; do
  EKGPU_VARIANT=$v timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/c2a/pmc_v$v/f -o run -- python3 bench.py --config C2 --steps 1 --warmup 1 --no-cpu --no-ingest > gpurun_out/c2a/pmc_v$v.log 2>&1 || exit $?
  python3 tools/pmc_kernels.py gpurun_out/c2a/pmc_v$v
done
