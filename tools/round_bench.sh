# Round-end evidence on one GPU box: rocprofv3 summaries for every config
# (summarised on the box, so the bench lines below read the fresh pmc_*.json),
# then one bench line per configuration (CPU baseline included).
#   bash tools/round_bench.sh <tag>      (run ON the GPU box, under gpurun)
# The summaries come back under gpurun_out/profiles/ (copy them to profiles/).
set -e
TAG=${1:?tag}
mkdir -p gpurun_out/profiles
prof() {   # <name> <cfg> [--out-of-place]
  bash tools/profile.sh ${TAG}_$1 --config $2 $3 > gpurun_out/prof_${TAG}_$1.log 2>&1
  python tools/prof_summary.py gpurun_out/prof_${TAG}_$1 ${TAG}_$1 $2 $3 > gpurun_out/sum_${TAG}_$1.log 2>&1
  echo "profile $1 done"
}
# PROFS / BENCHES select a subset (a call has at most 20 minutes)
for p in ${PROFS-cfg1 cfg2 cfg3 cfg4 cfg0 cfg1_oop}; do
  case $p in
    cfg1_oop) prof cfg1_oop cfg1 --out-of-place ;;
    *) prof $p $p ;;
  esac
done
cp profiles/${TAG}_*.json profiles/pmc_*.json gpurun_out/profiles/ 2>/dev/null || true
for c in ${BENCHES-cfg1 cfg0 cfg2 cfg3 cfg4}; do
  timeout -k 10 300 python bench.py --config $c > gpurun_out/bench_${TAG}_$c.json 2> gpurun_out/bench_${TAG}_$c.err
  echo "bench $c done"
done
