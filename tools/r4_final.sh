#!/bin/bash
# Round-4 final evidence on one box, in parts (a call has at most 20 minutes):
#   bash tools/r4_final.sh suite      GPU suite + smoke
#   PROFS="cfg1 cfg1_inplace" bash tools/r4_final.sh prof    rocprofv3 summaries (tools/round_bench.sh)
#   BENCHES="cfg1 cfg0 ..." bash tools/r4_final.sh bench     bench lines (reads the pmc_*.json in profiles/)
set -e
mkdir -p gpurun_out
case ${1:?part} in
  suite)
    timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/r4_final_suite.log 2>&1
    echo suite done
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4_final_smoke.log 2>&1
    echo smoke done ;;
  prof)
    BENCHES="" bash tools/round_bench.sh ${TAG:-r4}
    for d in gpurun_out/prof_${TAG:-r4}_*/; do d=${d%/}; cp $d/trace/run_kernel_stats.csv gpurun_out/profiles/$(basename $d | sed 's/^prof_//')_kernel_stats.csv; done ;;
  bench)
    PROFS="" bash tools/round_bench.sh ${TAG:-r4} ;;
esac
