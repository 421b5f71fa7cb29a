#!/bin/bash
# Development loop on the GPU: selected parity tests, then bench lines of the given configs (no CPU baseline).
cd "$(dirname "$0")/../.."; mkdir -p gpurun_out/dev
export TMPDIR=/tmp
TESTS="${TESTS:-tests/test_keymajor_gpu.py tests/test_ungrouped_gpu.py tests/test_engine_gpu.py}"
if [ -n "$TESTS" ] && [ "$TESTS" != "none" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/dev/pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/dev/pytest.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
fi
for c in ${CONFIGS:-C3 C4b C5 C2}; do
  timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 2 --no-cpu --no-ingest > gpurun_out/dev/$c.json 2> gpurun_out/dev/$c.err || { echo "$c failed"; tail -5 gpurun_out/dev/$c.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/dev/$c.json')); r=d['roofline']; print('$c', round(d['ms_per_step'],3), 'ms', round(r['frac'],4), {k: round(v['launch_ms']*v['launches_per_step'],3) for k,v in r.get('kernels',{}).items()})"
done
