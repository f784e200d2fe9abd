#!/bin/bash
# planner scan / lazy T-table / small GCM grid for ETA-only contexts / partial tail loads:
# ETA tests first (serialized kernels), then the GPU suite, same-box A/B on the planner configs, kernel trace
set -e
O=gpurun_out/r4_plan; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_eta_gpu.py > $O/eta_first.log 2>&1
echo eta done
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/gpu_suite.log 2>&1
echo suite done
bash tools/lib_ab.sh cfg3 $PWD/abl/base/libespgpu.so $PWD/f-stack_amd/libespgpu.so $PWD/abl/etashfl/libespgpu.so > $O/ab_cfg3_shfl.txt 2>&1
echo ab shfl done
for c in cfg4 cfg2; do
  bash tools/lib_ab.sh $c $PWD/abl/base/libespgpu.so $PWD/f-stack_amd/libespgpu.so > $O/ab_$c.txt 2>&1
  echo ab $c done
done
cd /tmp && export TMPDIR=/tmp
for c in cfg3 cfg4; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/kt_$c -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config $c --steps 10 --warmup 5 --no-inplace-leg --no-cpu --no-e2e --no-encrypt-leg --no-packed-leg > $GRAFT_REPO_ROOT/$O/kt_$c.log 2>&1
  echo kt $c done
done
