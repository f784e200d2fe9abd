#!/bin/bash
# Same-box A/B of engine builds on the 32- and 256-record burst latency
# (run on the GPU box):  bash tools/burst_ab.sh <dir with libespgpu.so> ...
for k in 1 2; do
  for D in "$@"; do
    echo -n "$D "
    LD_LIBRARY_PATH=$D BURST_MODE=1 timeout -k 10 90 ./tools/burst_bench ${BURSTS:-32 256} | python3 -c "
import sys,json
for l in sys.stdin:
  d=json.loads(l)
  if 'burst' in d: print(d['burst'],'x%d'%d['xfer'],d['latency_us_median'],'fs %.2fM'%(d['fstack_records_per_s']/1e6),end='  ')
print()"
  done
done
