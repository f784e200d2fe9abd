#!/bin/bash
# Same-box A/B of engine builds and tuning knobs (run ON the GPU box): every
# candidate runs once per round on every config, candidates alternating, so
# box drift hits all of them alike.  One JSON line per run on stdout and in
# $OUT (default gpurun_out/ab.jsonl).
#
#   bash tools/ab.sh [-r ROUNDS] [-c "cfg1 cfg4"] [-o OUT] [-x "bench args"] [-e] CAND...
# (-e: also the encrypt leg; its kernel time is summarised as enc_ms)
#
# CAND = name=LIB[@key=val,key=val][%bench-arg]: LIB a libespgpu.so (e.g. abl/<name>/libespgpu.so
# from tools/variant.sh, or f-stack_amd/libespgpu.so), the optional @ list set_tuning
# knobs, the optional % one extra bench.py argument for this candidate.  Default bench args: in-place headline only (no side legs, no CPU).
# Replaces round 4's one-off tools/r4_*.sh A/B scripts.
set -euo pipefail
ROUNDS=3; CFGS="cfg1"; OUT=gpurun_out/ab.jsonl; XARGS=""; ENC=--no-encrypt-leg
while getopts "r:c:o:x:e" o; do
  case $o in r) ROUNDS=$OPTARG ;; c) CFGS=$OPTARG ;; o) OUT=$OPTARG ;; x) XARGS=$OPTARG ;; e) ENC="" ;; *) exit 2 ;; esac
done
shift $((OPTIND - 1))
[ $# -ge 1 ] || { echo "usage: tools/ab.sh [-r N] [-c cfgs] [-o out] [-x args] name=lib[@k=v,...] ..." >&2; exit 2; }
mkdir -p "$(dirname "$OUT")"
B=(python bench.py --steps 20 --warmup 10 --no-inplace-leg --no-cpu --no-e2e $ENC --no-packed-leg)
for r in $(seq 1 "$ROUNDS"); do
  for cfg in $CFGS; do
    for cand in "$@"; do
      name=${cand%%=*}; rest=${cand#*=}; carg=""
      [[ $rest == *%* ]] && { carg=${rest#*%}; rest=${rest%%%*}; }
      lib=${rest%%@*}; knobs=""
      [[ $rest == *@* ]] && knobs=${rest#*@}
      targs=()
      if [ -n "$knobs" ]; then IFS=, read -ra kv <<< "$knobs"; for k in "${kv[@]}"; do targs+=(--tuning "$k"); done; fi
      line=$(ESPGPU_LIB=$lib timeout -k 10 180 "${B[@]}" --config "$cfg" "${targs[@]}" $XARGS $carg 2>/dev/null | tail -1)
      python3 - "$name" "$cfg" "$r" "$knobs" "$line" <<'EOF' | tee -a "$OUT"
import json, sys
name, cfg, rnd, knobs, line = sys.argv[1:6]
d = json.loads(line)
print(json.dumps({"cand": name, "config": cfg, "round": int(rnd), "knobs": knobs,
                  "ms_per_step": d["ms_per_step"], "kernel_ms": d["roofline"]["kernel_ms"],
                  "value": d["value"], "frac": d["roofline"]["frac"],
                  "enc_ms": d.get("encrypt", {}).get("kernel_ms")}))
EOF
    done
  done
done
python3 - "$OUT" <<'EOF'
import collections, json, sys
runs = collections.defaultdict(list)
enc = collections.defaultdict(list)
for ln in open(sys.argv[1]):
    d = json.loads(ln)
    runs[(d["config"], d["cand"])].append(d["kernel_ms"])
    if d.get("enc_ms"):
        enc[(d["config"], d["cand"])].append(d["enc_ms"])
for (cfg, cand), v in sorted(runs.items()):
    v.sort()
    e = sorted(enc.get((cfg, cand), []))
    tail = "  enc_ms min %.4f median %.4f" % (e[0], e[len(e) // 2]) if e else ""
    print("%-6s %-14s kernel_ms min %.4f median %.4f  (%d runs)%s" % (cfg, cand, v[0], v[len(v) // 2], len(v), tail))
EOF
