#!/bin/bash
# concurrent ETA design (eta_fused 4, variants library): parity, then same-box cfg3 A/B against the default
set -e
O=gpurun_out/r4_etac; mkdir -p $O
ESPGPU_VARIANTS=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_eta_gpu.py -k "variants or knob" > $O/tests.log 2>&1
echo tests done
V=$PWD/f-stack_amd/libespgpu_variants.so
B="python bench.py --config cfg3 --steps 20 --warmup 10 --no-inplace-leg --no-cpu --no-e2e --no-encrypt-leg --no-packed-leg"
for k in 1 2 3; do
  for t in eta_fused=2 eta_fused=4; do
    echo -n "$t "
    ESPGPU_LIB=$V timeout -k 10 120 $B --tuning $t 2>/dev/null | python -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['ms_per_step'], d['roofline']['kernel_ms'])"
  done
done > $O/ab_cfg3.txt 2>&1
echo ab done
cd /tmp && export TMPDIR=/tmp
ESPGPU_LIB=$V timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/kt -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config cfg3 --steps 10 --warmup 5 --no-inplace-leg --no-cpu --no-e2e --no-encrypt-leg --no-packed-leg --tuning eta_fused=4 > $GRAFT_REPO_ROOT/$O/kt.log 2>&1
echo kt done
