#!/bin/bash
# Planner kernel durations per engine build (run ON the GPU box):
#   bash tools/plan_prof.sh "cfg4 cfg2" name=lib ...
# rocprofv3 --kernel-trace --stats of a short bench run per (config, build);
# prints each build's average plan_* and main-kernel durations (us).
set -euo pipefail
CFGS=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd /tmp && export TMPDIR=/tmp
for cfg in $CFGS; do
  for cand in "$@"; do
    name=${cand%%=*}; lib=${cand#*=}
    [[ $lib = /* ]] || lib=$ROOT/$lib
    out=$ROOT/gpurun_out/pp_${name}_$cfg
    ESPGPU_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out" -o run --output-format csv -- \
      python3 "$ROOT/bench.py" --config "$cfg" --steps 20 --warmup 5 --no-cpu --no-e2e --no-inplace-leg \
      --no-encrypt-leg --no-packed-leg > "$out.log" 2>&1
    python3 - "$out" "$name" "$cfg" <<'PY'
import csv, glob, sys
out, name, cfg = sys.argv[1:4]
f = glob.glob(out + "/**/*kernel_stats.csv", recursive=True)[0]
row = []
for r in csv.DictReader(open(f)):
    n = r["Name"]
    k = next((x for x in ("plan_count", "plan_scan", "plan_emit", "plan_scatter", "gcm_kernel", "eta_kernel") if x in n), None)
    if k:
        row.append("%s %.1f" % (k if "kernel" not in k else n.split("(")[0].split("::")[-1][:28], float(r["AverageNs"]) / 1e3))
print("%-5s %-6s %s" % (cfg, name, "  ".join(row)))
PY
  done
done
