#!/bin/bash
# Round 4: final multiply from LDS (GCM_FMUL_LDS, abl/fmul) vs the product
# library, same box, alternating; in-place headline kernel_ms.  GCM parity of
# the variant first.
set -e
mkdir -p gpurun_out/r4_fmul
ESPGPU_LIB=abl/fmul/libespgpu.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gcm_gpu.py tests/test_configs_gpu.py > gpurun_out/r4_fmul/tests.log 2>&1
tail -1 gpurun_out/r4_fmul/tests.log
for CFG in ${CFGS:-cfg4 cfg2 cfg1}; do
  for k in 1 2 3; do
    for L in f-stack_amd/libespgpu.so abl/fmul/libespgpu.so; do
      echo -n "$CFG $L "
      ESPGPU_LIB=$L timeout -k 10 180 python bench.py --config $CFG --steps 20 --warmup 10 --no-cpu --no-e2e \
        --no-encrypt-leg --no-packed-leg --no-inplace-leg 2>/dev/null | python -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['ms_per_step'], d['roofline']['kernel_ms'])"
    done
  done
done | tee gpurun_out/r4_fmul/ab.txt
