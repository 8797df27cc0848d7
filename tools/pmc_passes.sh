#!/bin/bash
# Extra PMC passes (one rocprofv3 run per pass, counters only, no tracing domains) over the
# bench workload: tools/pmc_passes.sh <tag> <streams> "<pass1 counters>" ["<pass2>" ...]
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; N=$2; shift 2
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for P in "$@"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d $OUT/p$i -o run -- \
      python3 $R/bench.py --streams-per-gpu $N --steps 3 --warmup 1 --no-cpu-baseline --no-verify --no-md5 --no-e2e > $OUT/p$i.log 2>&1 || exit 1
done
echo done > $OUT/status.txt
