#!/bin/bash
# Round 4: bench with the in-place verify-first headline (one-pass GCM), quick
# lines for cfg1 (both modes) and cfg3, then the GPU suite.
set -e
mkdir -p gpurun_out/r4_ih
timeout -k 10 300 python bench.py --config cfg1 --no-cpu --no-e2e > gpurun_out/r4_ih/cfg1.json 2> gpurun_out/r4_ih/cfg1.err
echo cfg1 done
timeout -k 10 300 python bench.py --config cfg1 --out-of-place --no-cpu --no-e2e > gpurun_out/r4_ih/cfg1_oop.json 2> gpurun_out/r4_ih/cfg1_oop.err
echo cfg1 oop done
timeout -k 10 300 python bench.py --config cfg3 --no-cpu --no-e2e > gpurun_out/r4_ih/cfg3.json 2> gpurun_out/r4_ih/cfg3.err
echo cfg3 done
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/r4_ih/suite.log 2>&1
tail -1 gpurun_out/r4_ih/suite.log
