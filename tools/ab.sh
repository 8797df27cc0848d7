#!/bin/bash
# Same-box bench A/B of library builds (ZFLAC_HIP_LIB), alternating, R rounds.
# Usage: tools/ab.sh <tag> <rounds> <lib.so>... (bench args via AB_ARGS)
TAG=$1; R=$2; shift 2
O=gpurun_out/$TAG
mkdir -p $O
for i in $(seq 1 $R); do
for L in "$@"; do
  n=$(basename $L .so)
  ZFLAC_HIP_LIB=$L timeout -k 10 200 python bench.py --no-e2e --no-cpu-baseline --no-md5 --steps 30 ${AB_ARGS} \
      > $O/${n}_$i.json 2> $O/${n}_$i.err || exit $?
done; done
