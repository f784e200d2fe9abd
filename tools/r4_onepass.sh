#!/bin/bash
# Round 4: in-place GCM decrypt in one pass with rollback (GCM_INPLACE_ONEPASS)
# vs the two-pass MODE 2 (abl/old = the code before), same box, alternating.
set -e
mkdir -p gpurun_out/r4_onepass
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu ${TESTS:-tests} \
  > gpurun_out/r4_onepass/tests.log 2>&1
tail -1 gpurun_out/r4_onepass/tests.log
for CFG in ${CFGS:-cfg1 cfg4 cfg2}; do
  for k in 1 2 3; do
    for L in f-stack_amd/libespgpu.so abl/old/libespgpu.so; do
      echo -n "$CFG $L "
      ESPGPU_LIB=$L timeout -k 10 180 python bench.py --config $CFG --steps 20 --warmup 10 --no-cpu --no-e2e \
        --no-encrypt-leg --no-packed-leg 2>/dev/null | python -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['ms_per_step'], d['roofline']['kernel_ms'], d['inplace']['kernel_ms'], d['inplace']['status_ok'])"
    done
  done
done | tee gpurun_out/r4_onepass/ab.txt
