# bitsliced ctr pass: parity subset, bench lines per gcm_bs mode, kernel trace of each mode
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_edges_gpu.py tests/test_gcm_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "bs" > gpurun_out/bs_tests.log 2>&1
echo "tests rc=$?"
for t in ${MODES-1 2}; do
  timeout -k 10 120 python bench.py --no-cpu --no-e2e --no-inplace-leg --no-encrypt-leg --tuning gcm_bs=$t > gpurun_out/bs_bench_$t.json 2> gpurun_out/bs_bench_$t.err; echo "bench $t rc=$?"
done
cd /tmp && export TMPDIR=/tmp
for t in ${MODES-1 2}; do
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/bsprof$t -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 5 --no-cpu --no-e2e --no-inplace-leg --no-encrypt-leg --tuning gcm_bs=$t > $GRAFT_REPO_ROOT/gpurun_out/bsprof$t.log 2>&1; echo "prof $t rc=$?"
done
