# full GPU suite, then the opencrypto burst bench (all modes)
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputest_r3b.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/gputest_r3b.log; exit 1; }
tail -2 gpurun_out/gputest_r3b.log
timeout -k 10 240 ./tools/burst_bench > gpurun_out/burst_r3b.jsonl 2> gpurun_out/burst_r3b.err
