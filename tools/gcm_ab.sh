#!/bin/bash
# Same-box A/B of the committed engine (exp/head) against the working tree on
# one bench configuration: alternating runs, ms_per_step of each.
#   bash tools/gcm_ab.sh <cfg> [extra bench args]
set -e
CFG=${1:-cfg1}; shift || true
B="python bench.py --config $CFG --steps 20 --warmup 10 --no-inplace-leg --no-cpu --no-e2e $*"
run() { echo -n "$1 "; shift; timeout -k 10 120 "$@" 2>/dev/null | python -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['ms_per_step'])"; }
for k in 1 2 3; do
  run head env ESPGPU_LIB=exp/head/f-stack_amd/libespgpu.so $B
  run new $B
done
