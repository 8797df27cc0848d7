#!/bin/bash
# Round-3 measurement set (GPU box): the default bench line, then rocprofv3 kernel-trace
# statistics of the same workload with one run in flight (isolated launches, what the
# roofline uses) and with three (the headline's overlap). Usage: tools/r3_profile.sh <tag>
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r3prof}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R && timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/serial -o run -- \
    python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --no-md5 --inflight 1 > $O/serial.log 2>&1 || exit $?
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/inflight3 -o run -- \
    python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --no-md5 > $O/inflight3.log 2>&1
