#!/bin/bash
# phase clock of the 32-record burst kernel (knobs library), registered mbufs
set -e
O=gpurun_out/r4_phase; mkdir -p $O
for k in 1 2; do
LD_LIBRARY_PATH=exp/knobs BURST_MODE=1 timeout -k 10 90 ./tools/burst_bench 32 > $O/phase_$k.jsonl 2> $O/phase.err
done
echo phase done
