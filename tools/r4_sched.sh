#!/bin/bash
# Round 4: the compiler's scheduling strategies (abl/ilp = max-ilp,
# abl/memcl = max-memory-clause) vs the product build, same box, alternating,
# in-place headline kernel_ms; quick parity of each first.
set -e
mkdir -p gpurun_out/r4_sched
for L in abl/ilp/libespgpu.so abl/memcl/libespgpu.so; do
  ESPGPU_LIB=$L timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gcm_gpu.py tests/test_eta_gpu.py > gpurun_out/r4_sched/tests_$(basename $(dirname $L)).log 2>&1
  echo "$L $(tail -1 gpurun_out/r4_sched/tests_$(basename $(dirname $L)).log)"
done
for CFG in ${CFGS:-cfg1 cfg3}; do
  for k in 1 2 3; do
    for L in f-stack_amd/libespgpu.so abl/ilp/libespgpu.so abl/memcl/libespgpu.so; do
      echo -n "$CFG $L "
      ESPGPU_LIB=$L timeout -k 10 180 python bench.py --config $CFG --steps 20 --warmup 10 --no-cpu --no-e2e \
        --no-encrypt-leg --no-packed-leg --no-inplace-leg 2>/dev/null | python -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['ms_per_step'], d['roofline']['kernel_ms'])"
    done
  done
done | tee gpurun_out/r4_sched/ab.txt
