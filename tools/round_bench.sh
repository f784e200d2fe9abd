set -e
mkdir -p gpurun_out
bash tools/profile.sh r2g_cfg3 --config cfg3 > gpurun_out/prof_r2g_cfg3.log 2>&1
for c in cfg1 cfg0 cfg2 cfg3 cfg4; do
  timeout -k 10 300 python bench.py --config $c > gpurun_out/bench_$c.json 2> gpurun_out/bench_$c.err
  echo "$c done"
done
