#!/bin/bash
# output ring A/B: LDS write probe, GCM parity with the ring library, same-box cfg1/cfg4 A/B
set -e
O=gpurun_out/r4_ring; mkdir -p $O
timeout -k 10 60 ./tools/ldsalign > $O/ldsalign.jsonl 2>&1
ESPGPU_LIB=$PWD/abl/ring/libespgpu.so timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gcm_gpu.py tests/test_configs_gpu.py > $O/tests.log 2>&1
echo tests done
bash tools/lib_ab.sh cfg1 $PWD/abl/base/libespgpu.so $PWD/abl/ring/libespgpu.so > $O/ab_cfg1.txt 2>&1
echo ab cfg1 done
bash tools/lib_ab.sh cfg4 $PWD/abl/base/libespgpu.so $PWD/abl/ring/libespgpu.so > $O/ab_cfg4.txt 2>&1
echo ab cfg4 done
