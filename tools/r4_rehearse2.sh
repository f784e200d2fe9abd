#!/bin/bash
# Rehearsal of bench.py's 2-rank path on the one-GPU box: both ranks on device
# 0, gloo for the barriers and reductions (RCCL refuses two ranks on one
# device).  Checks the in-place segments, the max-over-ranks timing and the
# per-rank shard of cfg4; the numbers are not a scaling measurement.
set -e
mkdir -p gpurun_out/r4_rehearse
BENCH_SHARE_DEVICE=1 BENCH_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --config cfg4 \
  --steps 5 --warmup 2 --no-cpu --no-e2e > gpurun_out/r4_rehearse/cfg4_n2.json 2> gpurun_out/r4_rehearse/cfg4_n2.err
tail -c 1500 gpurun_out/r4_rehearse/cfg4_n2.json
