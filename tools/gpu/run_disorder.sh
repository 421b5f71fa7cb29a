#!/bin/bash
# Out-of-order C2 (bench.py --disorder 50): parity tests of the unsorted paths, bench line, rocprofv3 kernel stats.
cd "$(dirname "$0")/../.."; mkdir -p gpurun_out/dis
export TMPDIR=/tmp
TESTS="${TESTS:-tests/test_late_tolerance_gpu.py tests/test_engine_gpu.py}"
timeout -k 10 700 python -u -m pytest $TESTS tests/test_fullsize_parity_gpu.py -k "disordered or not fullsize" -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/dis/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "disordered x|passed|failed|Error" gpurun_out/dis/pytest.log | cut -c1-250 | tail -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --disorder 50 --no-cpu --no-ingest > gpurun_out/dis/C2_dis.json 2> gpurun_out/dis/C2_dis.err || { echo "bench failed"; tail -5 gpurun_out/dis/C2_dis.err; exit 1; }
cut -c1-300 gpurun_out/dis/C2_dis.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/dis/prof -o run -- python3 bench.py --disorder 50 --no-cpu --no-ingest --steps 5 --warmup 1 > gpurun_out/dis/prof.log 2>&1 || { echo "prof failed"; tail -5 gpurun_out/dis/prof.log; exit 1; }
f=$(find gpurun_out/dis/prof -name '*kernel_stats.csv' | head -1); head -8 "$f" | cut -d, -f1-4 | cut -c1-150
