#!/bin/bash
# ETA decrypt pass record mapping by ballot/readlane (ETA_LANE_MAP): parity, then same-box cfg3 A/B
set -e
O=gpurun_out/r4_lanemap; mkdir -p $O
ESPGPU_LIB=$PWD/abl/lanemap/libespgpu.so timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_eta_gpu.py tests/test_configs_gpu.py tests/test_fuzz_gpu.py tests/test_trailer.py > $O/tests.log 2>&1
echo tests done
bash tools/lib_ab.sh cfg3 $PWD/f-stack_amd/libespgpu.so $PWD/abl/lanemap/libespgpu.so > $O/ab_cfg3.txt 2>&1
echo ab done
