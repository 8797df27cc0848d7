#!/bin/bash
# PMC A/B of the previous build (tools/_build/libzflac_hip_prev.so) vs the in-tree one on the bench
# workload. Usage (GPU box): TAG=<dir> PMC="<counters>" bash tools/pmc_ab.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-icache}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
ARGS="--steps 3 --warmup 1 --no-cpu-baseline --no-verify --no-md5 --no-e2e"
P="${PMC:-SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_BUSY_CYCLES SQ_INSTS_VALU}"
ZFLAC_HIP_LIB=$R/tools/_build/libzflac_hip_prev.so timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d $OUT/prev -o run -- python3 $R/bench.py $ARGS > $OUT/prev.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d $OUT/new -o run -- python3 $R/bench.py $ARGS > $OUT/new.log 2>&1 || exit 1
echo done > $OUT/status.txt
