#!/bin/bash
# round-4 baseline on one box: cfg1 bench line, burst latency, burst kernel trace
set -e
O=gpurun_out/r4_base; mkdir -p $O
timeout -k 10 300 python bench.py --config cfg1 > $O/bench_cfg1.json 2> $O/bench_cfg1.err
echo bench done
BURST_MODE=1 timeout -k 10 120 ./tools/burst_bench 32 256 > $O/burst.jsonl 2> $O/burst.err
echo burst done
cd /tmp && export TMPDIR=/tmp
BURST_MODE=1 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/kt -o run --output-format csv -- $GRAFT_REPO_ROOT/tools/burst_bench 32 > $GRAFT_REPO_ROOT/$O/kt.log 2>&1
echo kt done
