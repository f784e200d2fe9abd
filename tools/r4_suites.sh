#!/bin/bash
# Round 4: default GPU suite + smoke, then the suite on the variants library.
set -e
mkdir -p gpurun_out/r4_suites
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/r4_suites/default.log 2>&1
tail -1 gpurun_out/r4_suites/default.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4_suites/smoke.log 2>&1
tail -1 gpurun_out/r4_suites/smoke.log
ESPGPU_VARIANTS=1 timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/r4_suites/variants.log 2>&1
tail -1 gpurun_out/r4_suites/variants.log
