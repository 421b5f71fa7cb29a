#!/bin/bash
# round 4: processing-time features (FILTER, delayed / send-twice sliding) + small-window kernel: parity tests,
# the C4b bench line, its kernel profile and SQ counters of k_small_win
cd "$(dirname "$0")/../.."; mkdir -p gpurun_out/pmc_sw
timeout -k 10 700 python -u -m pytest tests/test_processing_gpu.py tests/test_range_gpu.py tests/test_state_window_gpu.py \
  tests/test_first_row_gpu.py tests/test_determinism_gpu.py tests/test_state_gpu.py tests/test_engine_gpu.py \
  "tests/test_fullsize_parity_gpu.py::test_c4b_count_full_parity" \
  -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4_b_tests.log 2>&1
rc=$?; tail -15 gpurun_out/r4_b_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config C4b --steps 10 --warmup 2 --no-cpu > gpurun_out/r4_c4b.json 2> gpurun_out/r4_c4b.err
rc=$?; cut -c1-300 gpurun_out/r4_c4b.json; [ $rc -eq 0 ] || { tail -5 gpurun_out/r4_c4b.err; exit $rc; }
bash tools/gpu/prof.sh C4b 5 || exit 1
export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY" \
           "SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d gpurun_out/pmc_sw/p$i -o run -- python3 bench.py --config C4b --steps 1 --warmup 1 --no-cpu > gpurun_out/pmc_sw/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
