#!/bin/bash
# Kernel-time breakdown with the measurement knobs (libespgpu_knobs.so):
#   bash tools/knob_sweep.sh <cfg> <gcm_opts|eta_opts> <value> [<value> ...]
# prints "<value> <ms_per_step>" per setting (0 = the unmodified kernel).
set -e
CFG=$1; KEY=$2; shift 2
for v in "$@"; do
  echo -n "$KEY=$v "
  ESPGPU_LIB=f-stack_amd/libespgpu_knobs.so timeout -k 10 120 python bench.py --config $CFG --steps 20 --warmup 10 \
    --no-inplace-leg --no-cpu --no-e2e --tuning $KEY=$v 2>/dev/null |
    python -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['ms_per_step'])"
done
