#!/bin/bash
# Kernel-trace statistics of the bench workload (rocprofv3 --kernel-trace --stats, CSV), on
# the GPU box. Counters are collected separately by tools/pmc.sh (never in the same run).
# Usage: tools/profile.sh <tag> [bench args]  -> gpurun_out/<tag>/stats/*kernel_stats.csv, bench line
# in stats.log. Default bench args: one run in flight (--inflight 1), so the per-kernel averages
# are isolated launches, as the bench line's roofline uses.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-prof}
shift || true
EXTRA=${@:---inflight 1}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- \
    python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --no-md5 $EXTRA > $OUT/stats.log 2>&1
