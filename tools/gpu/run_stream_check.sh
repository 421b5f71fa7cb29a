#!/bin/bash
# GPU: streaming-path parity (pane-mode tests + full-size C2/C3) then a short C2 bench and its kernel trace
cd "$(dirname "$0")/../.."; mkdir -p gpurun_out/prof_s
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py "tests/test_fullsize_parity_gpu.py::test_c2_full_parity" "tests/test_fullsize_parity_gpu.py::test_c3_shard_full_parity" -m gpu -x -v -s --timeout 200 --timeout-method thread > gpurun_out/pytest_stream.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|Error|error|^C[23]" gpurun_out/pytest_stream.log | tail -30; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu > gpurun_out/bench_stream.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_stream.log | cut -c1-900; [ $rc -eq 0 ] || exit $rc
EKGPU_STREAM=0 timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu > gpurun_out/bench_nostream.log 2>&1
rc=$?; echo "bench(no stream) rc=$rc"; grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_nostream.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_s -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/prof_s.log 2>&1
echo "prof rc=$?"
