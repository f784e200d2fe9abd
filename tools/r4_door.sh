#!/bin/bash
# doorbell path: parity tests, then burst latency with and without the door
set -e
O=gpurun_out/r4_door; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_zerocopy_gpu.py -k "door or self_staging" > $O/tests.log 2>&1
echo tests done
for t in "door=64" ""; do
  BURST_TUNING=$t BURST_MODE=1 timeout -k 10 120 ./tools/burst_bench 32 256 > $O/burst_$t.jsonl 2> $O/burst_$t.err
done
echo burst done
