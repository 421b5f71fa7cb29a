#!/bin/bash
# round 5: asynchronous pushes — parity (async test + engine suite), then every config's bench line and a C2 trace
cd "$(dirname "$0")/../.."; mkdir -p gpurun_out/c2e
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_async_gpu.py tests/test_engine_gpu.py tests/test_state_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/c2e/tests.log 2>&1
rc=$?; tail -5 gpurun_out/c2e/tests.log; [ $rc -eq 0 ] || exit $rc
for c in C2 C3 C4a C4b C5; do
  timeout -k 10 200 python bench.py --config $c --steps 20 --warmup 3 --no-cpu > gpurun_out/c2e/$c.log 2>&1 || exit $?
  tail -1 gpurun_out/c2e/$c.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['roofline']['kernels']; print('$c', round(d['ms_per_step'],4), {n: round(v['launch_ms'],4) for n, v in k.items()})"
done
timeout -k 10 -s KILL 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c2e/trace -o run -- python3 bench.py --config C2 --steps 5 --warmup 2 --no-cpu --no-ingest > gpurun_out/c2e/trace.log 2>&1 || exit $?
python3 tools/trace_gaps.py $(ls gpurun_out/c2e/trace/*kernel_trace.csv | head -1)
