#!/bin/bash
# key-major tests, C4a with the staged (KM_EMIT=1) and direct (KM_EMIT=0) write pass, C1 ingest line
cd "$(dirname "$0")/../.."; mkdir -p gpurun_out/dev
timeout -k 10 600 python -u -m pytest tests/test_keymajor_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/dev/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/dev/pytest.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
for e in 1 0; do
  EKGPU_KM_EMIT=$e timeout -k 10 300 python bench.py --config C4a --steps 10 --warmup 2 --no-cpu --no-ingest > gpurun_out/dev/C4a_$e.json 2> gpurun_out/dev/C4a_$e.err || { echo "C4a $e failed"; tail -5 gpurun_out/dev/C4a_$e.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/dev/C4a_$e.json')); r=d['roofline']; print('C4a emit=$e', round(d['ms_per_step'],3), 'ms', {k: round(v['launch_ms']*v['launches_per_step'],3) for k,v in r['kernels'].items()})"
done
timeout -k 10 300 python bench.py --config C1 --steps 10 --warmup 2 > gpurun_out/dev/C1.json 2> gpurun_out/dev/C1.err || { echo "C1 failed"; tail -5 gpurun_out/dev/C1.err; exit 1; }
cut -c1-900 gpurun_out/dev/C1.json
