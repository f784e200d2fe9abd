#!/bin/bash
# Same-box A/B of set_tuning settings on one bench configuration (run on the
# GPU box): alternating runs, ms_per_step and kernel_ms of each.
#   bash tools/knob_ab.sh <cfg> "<key=v[,key=v]>" "<key=v>" ... [-- extra bench args]
set -e
CFG=$1; shift
SETS=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do SETS+=("$1"); shift; done
[ "${1:-}" = "--" ] && shift
B="python bench.py --config $CFG --steps 20 --warmup 10 --no-cpu --no-e2e $*"
for k in 1 2 3; do
  for S in "${SETS[@]}"; do
    T=""; for kv in ${S//,/ }; do T="$T --tuning $kv"; done
    echo -n "$S "
    timeout -k 10 150 $B $T 2>/dev/null | python -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['ms_per_step'], d['roofline']['kernel_ms'], d.get('inplace',{}).get('kernel_ms'), d.get('encrypt',{}).get('kernel_ms'))"
  done
done
