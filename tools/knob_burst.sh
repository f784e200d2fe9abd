for o in 0 2 4 6 32 64 96 102 1 103; do
  echo -n "opts=$o "
  LD_LIBRARY_PATH=exp/knobs BURST_TUNING=gcm_opts=$o BURST_MODE=1 timeout -k 10 60 ./tools/burst_bench 32 | python3 -c "
import sys,json
for l in sys.stdin:
  d=json.loads(l); print('xfer',d['xfer'],'lat',d['latency_us_median'],end='  ')
print()"
done
