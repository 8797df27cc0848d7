#!/bin/bash
# Collect PMC counters for the bench workload in separate rocprofv3 passes (counters are
# never combined with tracing domains), plus the FETCH_SIZE/WRITE_SIZE calibration of
# tools/calib_pmc.hip. Usage: tools/pmc.sh <tag>   (on the GPU box)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-pmc}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
ARGS="--steps 3 --warmup 1 --no-cpu-baseline --no-verify --no-md5 --no-e2e --inflight 1"
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_WAVE_CYCLES"
P2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES"
P3="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VMEM SQ_WAVES"
i=0
for P in "$P1" "$P2" "$P3" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $OUT/p$i -o run -- python3 $R/bench.py $ARGS > $OUT/p$i.log 2>&1
done
for P in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $OUT/calib_$P -o run -- $R/tools/_build/calib_pmc > $OUT/calib_$P.log 2>&1
done
echo done >> $OUT/status.txt
