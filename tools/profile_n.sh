#!/bin/bash
# Kernel-trace stats of the bench workload at a given stream count: tools/profile_n.sh <tag> <streams>
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- \
    python3 $R/bench.py --streams-per-gpu $2 --steps 10 --warmup 2 --no-cpu-baseline --no-verify --no-md5 --no-e2e > $OUT/stats.log 2>&1
