#!/bin/bash
# in-order completion retirement: process-path tests on the product and the variants library, burst latency
set -e
O=gpurun_out/r4_order; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_zerocopy_gpu.py tests/test_kmock_driver_gpu.py tests/test_fstack_run.py tests/test_integration.py > $O/tests.log 2>&1
echo tests done
ESPGPU_VARIANTS=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_zerocopy_gpu.py > $O/tests_var.log 2>&1
echo tests var done
for t in "door=64" ""; do
  BURST_TUNING=$t BURST_MODE=1 timeout -k 10 120 ./tools/burst_bench 32 256 > $O/burst_$t.jsonl 2> $O/burst_$t.err
done
echo burst done
