# Round-end evidence on one GPU box: rocprofv3 summaries for every config
# (summarised on the box, so the bench lines below read the fresh pmc_*.json),
# then one bench line per configuration (CPU baseline included).
#   bash tools/round_bench.sh <tag>      (run ON the GPU box, under gpurun)
# The summaries come back under gpurun_out/profiles/ (copy them to profiles/).
set -e
TAG=${1:?tag}
mkdir -p gpurun_out/profiles
prof() {   # <name> <cfg> [--inplace]
  bash tools/profile.sh ${TAG}_$1 --config $2 $3 > gpurun_out/prof_${TAG}_$1.log 2>&1
  python tools/prof_summary.py gpurun_out/prof_${TAG}_$1 ${TAG}_$1 $2 $3 > gpurun_out/sum_${TAG}_$1.log 2>&1
  echo "profile $1 done"
}
prof cfg1 cfg1
prof cfg2 cfg2
prof cfg3 cfg3
prof cfg4 cfg4
prof cfg0 cfg0
prof cfg1_inplace cfg1 --inplace
cp profiles/${TAG}_*.json profiles/pmc_*.json gpurun_out/profiles/
for c in cfg1 cfg0 cfg2 cfg3 cfg4; do
  timeout -k 10 300 python bench.py --config $c > gpurun_out/bench_${TAG}_$c.json 2> gpurun_out/bench_${TAG}_$c.err
  echo "bench $c done"
done
