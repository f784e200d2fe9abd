#!/bin/bash
# bisect the ETA variants-decrypt failure: one library per run, serialized kernels; stop at a fault
O=gpurun_out/r4_bisect; mkdir -p $O
for n in base nplan ngrid ngcm cur; do
  L=$PWD/abl/$n/libespgpu.so; [ $n = cur ] && L=$PWD/f-stack_amd/libespgpu.so
  AMD_SERIALIZE_KERNEL=3 ESPGPU_LIB=$L timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_eta_gpu.py > $O/$n.log 2>&1
  rc=$?
  echo "$n rc=$rc $(tail -1 $O/$n.log)"
  if grep -q "illegal memory\|Memory access fault" $O/$n.log || [ $rc -ge 124 ]; then echo "fault/timeout at $n: stop"; exit 1; fi
done
exit 0
