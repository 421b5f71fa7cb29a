#!/bin/bash
# The N-rank shard-mode bench path rehearsed on ONE GPU (gloo over the device tensors, both ranks on cuda:0):
# the device router, the trigger / count exchanges and the JSON line, at reduced sizes. Usage: run_rehearse_ranks.sh
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
for cfg in "C2 4000000" "C3 2000000" "C4a 1000000" "C4b 4000000" "C5 4000000"; do
    set -- $cfg
    EKGPU_BENCH_ONE_DEVICE=1 EKGPU_DIST_BACKEND=gloo timeout -k 10 240 python -m torch.distributed.run --nnodes=1 \
        --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --config $1 --events $2 \
        --steps 3 --warmup 1 --no-cpu --no-ingest > gpurun_out/rehearse_$1.txt 2>&1 || { echo "rehearsal $1 failed"; exit 1; }
    grep '"metric"' gpurun_out/rehearse_$1.txt | cut -c1-160
done
