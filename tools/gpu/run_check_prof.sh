#!/bin/bash
# GPU parity suite + smoke + default bench line, then per-config bench lines under rocprofv3 kernel stats.
cd "$(dirname "$0")/../.."; mkdir -p gpurun_out/cp
export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 300 python bench.py > gpurun_out/cp/bench_default.json 2> gpurun_out/cp/bench_default.err
rc=$?; echo "bench rc=$rc"; cut -c1-300 gpurun_out/cp/bench_default.json; [ $rc -eq 0 ] || exit $rc
for c in ${CONFIGS:-C3 C4a C4b C5}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/cp/$c.prof -o run -- python3 bench.py --config $c --steps 5 --warmup 1 --no-cpu --no-ingest > gpurun_out/cp/$c.json 2> gpurun_out/cp/$c.err || { echo "$c failed"; tail -3 gpurun_out/cp/$c.err; exit 1; }
  f=$(find gpurun_out/cp/$c.prof -name '*kernel_stats.csv' | head -1); echo "== $c"; cut -c1-200 gpurun_out/cp/$c.json | head -1
  head -10 "$f" | cut -d, -f1-4 | cut -c1-150
done
