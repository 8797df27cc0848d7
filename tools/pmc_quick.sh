#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=$R/gpurun_out/$1; mkdir -p $O
ARGS="--steps 3 --warmup 1 --no-cpu-baseline --no-verify --no-md5 --no-e2e --inflight 1"
(cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_WAVE_CYCLES --kernel-trace --output-format csv -d $O/p1 -o run -- python3 $R/bench.py $ARGS) > $O/p1.log 2>&1
