# one iteration of the bitsliced ctr pass work: parity subset, then knob timing
timeout -k 10 300 python -u -m pytest tests/test_edges_gpu.py tests/test_gcm_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "bs" > gpurun_out/bs_tests.log 2>&1 || { echo TESTS FAILED; exit 1; }
bash tools/bs_knobs.sh
