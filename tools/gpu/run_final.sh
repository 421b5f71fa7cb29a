#!/bin/bash
# GPU: the whole -m gpu suite (one pytest process) and the default bench line
cd "$(dirname "$0")/../.."; mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_full.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_full.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/bench_default.log 2>&1 || exit 1
grep '"metric"' gpurun_out/bench_default.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('default', d['config']['workload'][:40], round(d['ms_per_step'],3), 'ms', round(d['roofline']['frac'],3))"
timeout -k 10 300 python -u bench.py --config C5 --steps 10 --no-cpu > gpurun_out/bench_c5.log 2>&1 || exit 1
grep '"metric"' gpurun_out/bench_c5.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('C5', round(d['ms_per_step'],3), 'ms', round(d['roofline']['frac'],3))"
