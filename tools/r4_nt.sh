#!/bin/bash
# Round 4: nontemporal hints on the GCM record loads (abl/nt1) and stores
# (abl/nt2) vs the product, same box, alternating; cfg1 in place (headline)
# and out of place.
set -e
mkdir -p gpurun_out/r4_nt
for MODE in "" "--out-of-place"; do
  for k in 1 2 3; do
    for L in f-stack_amd/libespgpu.so abl/nt1/libespgpu.so abl/nt2/libespgpu.so; do
      echo -n "cfg1 ${MODE:-inplace} $L "
      ESPGPU_LIB=$L timeout -k 10 180 python bench.py --config cfg1 $MODE --steps 20 --warmup 10 --no-cpu --no-e2e \
        --no-encrypt-leg --no-packed-leg --no-inplace-leg 2>/dev/null | python -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['ms_per_step'], d['roofline']['kernel_ms'])"
    done
  done
done | tee gpurun_out/r4_nt/ab.txt
