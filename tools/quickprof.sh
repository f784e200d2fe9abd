#!/bin/bash
# Kernel-level A/B evidence for one configuration (run ON the GPU box):
#   bash tools/quickprof.sh <tag> [bench.py args]
# kernel trace + stats, then FETCH_SIZE, WRITE_SIZE and the SQ instruction /
# wait counters in separate --pmc passes (profile.sh's counter set, fewer
# launches); summarised by tools/prof_summary.py into gpurun_out/.
set -euo pipefail
TAG=${1:?tag}; shift || true
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
BENCH=(python3 "$ROOT/bench.py" --steps 10 --warmup 5 --no-cpu --no-e2e --no-inplace-leg --no-encrypt-leg --no-packed-leg "$@")
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- "${BENCH[@]}" > "$OUT/trace.log" 2>&1
timeout -k 10 240 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o run --output-format csv -- "${BENCH[@]}" > "$OUT/pmc_fetch.log" 2>&1
timeout -k 10 240 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d "$OUT/pmc_write" -o run --output-format csv -- "${BENCH[@]}" > "$OUT/pmc_write.log" 2>&1
timeout -k 10 240 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE -d "$OUT/pmc_sq" -o run --output-format csv -- "${BENCH[@]}" > "$OUT/pmc_sq.log" 2>&1
timeout -k 10 240 rocprofv3 --kernel-trace --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU -d "$OUT/pmc_sq2" -o run --output-format csv -- "${BENCH[@]}" > "$OUT/pmc_sq2.log" 2>&1
timeout -k 10 240 rocprofv3 --kernel-trace --pmc SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_SMEM -d "$OUT/pmc_sq3" -o run --output-format csv -- "${BENCH[@]}" > "$OUT/pmc_sq3.log" 2>&1
echo "quickprof $TAG done"
