#!/bin/bash
# Same-box A/B of set_tuning values on one bench configuration: alternating
# runs, ms_per_step and kernel ms of each.
#   bash tools/tuning_ab.sh <cfg> <key=value> <key=value> ... (run on the GPU box)
set -e
CFG=$1; shift
B="python bench.py --config $CFG --steps 20 --warmup 10 --no-inplace-leg --no-cpu --no-e2e --no-encrypt-leg --no-packed-leg"
for k in 1 2 3; do
  for T in "$@"; do
    echo -n "$T "
    timeout -k 10 120 $B --tuning $T 2>/dev/null | python -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['ms_per_step'], d['roofline']['kernel_ms'])"
  done
done
