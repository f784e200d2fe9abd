#!/bin/bash
# Same-box A/B of engine builds on cfg1 with an out-of-place buffer padded by
# 40 bytes per record (room for the GCM_OUTALIGN layout probe, which puts
# record k's plaintext at out + k*1536 + 128).
#   bash tools/outalign_ab.sh <lib1> <lib2> ... (run on the GPU box)
set -e
B="python bench.py --config cfg1 --out-pad 40 --steps 20 --warmup 10 --no-inplace-leg --no-cpu --no-e2e --no-encrypt-leg --no-packed-leg"
for k in 1 2 3; do
  for L in "$@"; do
    echo -n "$L "
    ESPGPU_LIB=$L timeout -k 10 120 $B 2>/dev/null | python -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['ms_per_step'], d['roofline']['kernel_ms'])"
  done
done
