#!/bin/bash
# Round 4: planner tile (records per thread of plan_count / plan_scatter:
# 4 = product, abl/pt8, abl/pt16), same box, alternating, in place; parity of
# pt16 on the planner tests first.
set -e
mkdir -p gpurun_out/r4_pt
ESPGPU_LIB=abl/pt16/libespgpu.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_configs_gpu.py tests/test_eta_gpu.py > gpurun_out/r4_pt/tests.log 2>&1
tail -1 gpurun_out/r4_pt/tests.log
for CFG in ${CFGS:-cfg4 cfg2}; do
  for k in 1 2 3; do
    for L in f-stack_amd/libespgpu.so abl/pt8/libespgpu.so abl/pt16/libespgpu.so; do
      echo -n "$CFG $L "
      ESPGPU_LIB=$L timeout -k 10 180 python bench.py --config $CFG --steps 20 --warmup 10 --no-cpu --no-e2e \
        --no-encrypt-leg --no-packed-leg --no-inplace-leg 2>/dev/null | python -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['ms_per_step'], d['roofline']['kernel_ms'])"
    done
  done
done | tee gpurun_out/r4_pt/ab.txt
