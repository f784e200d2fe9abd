#!/bin/bash
# multi-chunk GCM tickets (GCM_GROUP): GCM parity on grp4, same-box A/B on the planner configs
set -e
O=gpurun_out/r4_group; mkdir -p $O
ESPGPU_LIB=$PWD/abl/grp8/libespgpu.so timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_configs_gpu.py tests/test_fuzz_gpu.py tests/test_gcm_gpu.py > $O/tests_grp8.log 2>&1
echo tests done
bash tools/lib_ab.sh cfg4 $PWD/f-stack_amd/libespgpu.so $PWD/abl/grp4/libespgpu.so $PWD/abl/grp8/libespgpu.so > $O/ab_cfg4.txt 2>&1
echo ab cfg4 done
bash tools/lib_ab.sh cfg2 $PWD/f-stack_amd/libespgpu.so $PWD/abl/grp4/libespgpu.so $PWD/abl/grp8/libespgpu.so > $O/ab_cfg2.txt 2>&1
echo ab cfg2 done
