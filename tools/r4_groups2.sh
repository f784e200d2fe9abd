#!/bin/bash
# planner draw groups: parity (GCM / config / fuzz / ETA tests), then same-box A/B against the previous commit
set -e
O=gpurun_out/r4_groups2; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_configs_gpu.py tests/test_fuzz_gpu.py tests/test_gcm_gpu.py tests/test_eta_gpu.py tests/test_edges_gpu.py > $O/tests.log 2>&1
echo tests done
for c in cfg4 cfg2 cfg3; do
  bash tools/lib_ab.sh $c $PWD/abl/prev/libespgpu.so $PWD/f-stack_amd/libespgpu.so > $O/ab_$c.txt 2>&1
  echo ab $c done
done
