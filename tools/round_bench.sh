# Round-end evidence on one GPU box: rocprofv3 summaries for the GCM configs,
# then one bench line per configuration (CPU baseline included).
#   bash tools/round_bench.sh <tag>      (run ON the GPU box, under gpurun)
set -e
TAG=${1:?tag}
mkdir -p gpurun_out
for c in cfg1 cfg2 cfg4 cfg0; do
  bash tools/profile.sh ${TAG}_$c --config $c > gpurun_out/prof_${TAG}_$c.log 2>&1
  echo "profile $c done"
done
for c in cfg1 cfg0 cfg2 cfg3 cfg4; do
  timeout -k 10 300 python bench.py --config $c > gpurun_out/bench_${TAG}_$c.json 2> gpurun_out/bench_${TAG}_$c.err
  echo "bench $c done"
done
