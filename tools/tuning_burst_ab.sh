#!/bin/bash
# Same-box A/B of set_tuning settings on the 32- and 256-record bursts of
# tools/burst_bench (registered memory; run on the GPU box):
#   bash tools/tuning_burst_ab.sh "stage_fused=1" "stage_fused=0" ...
for k in 1 2; do
  for T in "$@"; do
    echo -n "$T "
    BURST_TUNING=$T BURST_MODE=1 timeout -k 10 90 ./tools/burst_bench ${BURSTS:-32 256} | python3 -c "
import sys,json
for l in sys.stdin:
  d=json.loads(l); print(d['burst'],'x%d'%d['xfer'],d['latency_us_median'],'fs %.2fM'%(d['fstack_records_per_s']/1e6),end='  ')
print()"
  done
done
