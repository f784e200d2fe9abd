#!/bin/bash
# Round 4 timing probe: cfg3 in place through the one-pass lane = record
# MODE 0 kernel (abl/etaprobe, no rollback: all bench records are valid) vs
# the product's two-pass MODE 2, same box, alternating.
set -e
mkdir -p gpurun_out/r4_etaprobe
for k in 1 2 3; do
  for L in f-stack_amd/libespgpu.so abl/etaprobe/libespgpu.so; do
    echo -n "cfg3 $L "
    ESPGPU_LIB=$L timeout -k 10 180 python bench.py --config cfg3 --steps 20 --warmup 10 --no-cpu --no-e2e \
      --no-encrypt-leg --no-packed-leg --no-inplace-leg 2>/dev/null | python -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['ms_per_step'], d['roofline']['kernel_ms'])"
  done
done | tee gpurun_out/r4_etaprobe/ab.txt
# parity of the variants library's MODE 0 (its tail hash words now read before its stores)
ESPGPU_VARIANTS=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_eta_gpu.py tests/test_trailer.py > gpurun_out/r4_etaprobe/variants_eta.log 2>&1
tail -1 gpurun_out/r4_etaprobe/variants_eta.log
