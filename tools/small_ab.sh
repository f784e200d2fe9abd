# Same-box A/B of the committed engine (exp/head) against the working tree on
# small caller-grouped GCM batches (tools/gcm_timing.py kernel time) and on
# the opencrypto burst path (tools/burst_bench, built against each library).
set -e
for n in ${SIZES:-32 256 2048 8192 16000 24000 32000 40000 65536}; do
  for L in exp/head/f-stack_amd/libespgpu.so f-stack_amd/libespgpu.so; do
    echo -n "$L "; ESPGPU_LIB=$L timeout -k 10 120 python tools/gcm_timing.py --records $n --reps 200 2>/dev/null | tail -1
  done
done
if [ -x tools/burst_bench_head ]; then
  for k in 1 2; do
    echo "head"; timeout -k 10 120 ./tools/burst_bench_head 32 256 2048
    echo "new"; timeout -k 10 120 ./tools/burst_bench 32 256 2048
  done
fi
