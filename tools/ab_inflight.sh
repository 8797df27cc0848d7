#!/bin/bash
# Same-box A/B of library builds (ZFLAC_HIP_LIB) x shard runs in flight, twice each.
# Usage: tools/ab_inflight.sh "<lib> <lib> ..." "<inflight> <inflight> ..." [tag]
set -e
LIBS=${1:-"zflac_amd/libzflac_hip.so"}
NS=${2:-"1 2 3"}
TAG=${3:-abinf}
mkdir -p gpurun_out/$TAG
for i in 1 2; do
for L in $LIBS; do
for N in $NS; do
  n=$(basename $L .so)
  ZFLAC_HIP_LIB=$L timeout -k 10 200 python bench.py --no-e2e --no-cpu-baseline --no-md5 --no-verify --steps 40 --inflight $N \
    > gpurun_out/$TAG/${n}_inf${N}_$i.json 2> gpurun_out/$TAG/${n}_inf${N}_$i.err
done; done; done
