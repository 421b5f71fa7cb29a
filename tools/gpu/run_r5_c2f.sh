#!/bin/bash
# round 5 C2: SQ counters of k_part / k_agg (issue vs parked cycles, LDS), bench line with the stats totals fixed
cd "$(dirname "$0")/../.."; mkdir -p gpurun_out/c2f
export TMPDIR=/tmp
timeout -k 10 200 python bench.py --config C2 --steps 20 --warmup 3 --no-cpu > gpurun_out/c2f/C2.log 2>&1 || exit $?
tail -1 gpurun_out/c2f/C2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['roofline']['kernels']; print('C2', round(d['ms_per_step'],4), d['roofline']['device_ms_per_step'], {n: round(v['launch_ms'],4) for n, v in k.items()})"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d gpurun_out/c2f/sq -o run -- python3 bench.py --config C2 --steps 1 --warmup 1 --no-cpu --no-ingest > gpurun_out/c2f/sq.log 2>&1 || exit $?
python3 tools/pmc_kernels.py gpurun_out/c2f/sq
