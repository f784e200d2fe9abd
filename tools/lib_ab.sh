#!/bin/bash
# Same-box A/B/C of engine builds on one bench configuration: alternating runs,
# ms_per_step of each.   bash tools/lib_ab.sh <cfg> <lib1> <lib2> ... (run on the GPU box)
set -e
CFG=$1; shift
B="python bench.py --config $CFG --steps 20 --warmup 10 --no-inplace-leg --no-cpu --no-e2e --no-encrypt-leg --no-packed-leg"
for k in 1 2 3; do
  for L in "$@"; do
    echo -n "$L "
    ESPGPU_LIB=$L timeout -k 10 120 $B 2>/dev/null | python -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['ms_per_step'], d['roofline']['kernel_ms'])"
  done
done
