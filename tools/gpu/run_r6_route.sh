#!/bin/bash
# round 6: the key-hash router — unit test, then a 2-rank gloo rehearsal of the routed N-rank bench on one GPU
cd "$(dirname "$0")/../.."; mkdir -p gpurun_out/r6route
timeout -k 10 300 python -u -m pytest tests/test_route_gpu.py tests/test_sharding_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r6route/tests.log 2>&1
rc=$?; tail -2 gpurun_out/r6route/tests.log; [ $rc -eq 0 ] || exit $rc
for cfg in C2 C4a C5; do
  EKGPU_DIST_BACKEND=gloo EKGPU_BENCH_ONE_DEVICE=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --config $cfg --steps 3 --warmup 1 --no-cpu --events 20000000 \
    > gpurun_out/r6route/$cfg.log 2>&1 || { tail -20 gpurun_out/r6route/$cfg.log; exit 1; }
  tail -1 gpurun_out/r6route/$cfg.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$cfg', round(d['ms_per_step'],3), d['config'].get('routing',{}).get('partition_ms_per_step'), d['config'].get('routing',{}).get('exchange_ms_per_step'), d['config']['windows_emitted'], d['config']['rows_per_step_rank0'])"
done
