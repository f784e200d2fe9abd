#!/bin/bash
# round-4 session-3 baseline on one box: LDS alignment probe, GPU suite, cfg1/cfg3/cfg4 bench lines
set -e
O=gpurun_out/r4s3_base; mkdir -p $O
timeout -k 10 60 ./tools/ldsalign > $O/ldsalign.jsonl 2>&1
echo probe done
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/gpu_suite.log 2>&1
echo suite done
for c in cfg1 cfg3 cfg4; do
  timeout -k 10 300 python bench.py --config $c --no-cpu > $O/bench_$c.json 2> $O/bench_$c.err
  echo bench $c done
done
