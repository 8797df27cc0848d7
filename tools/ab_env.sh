#!/bin/bash
# Same-box A/B of (library, environment) variants at one in-flight depth, alternating, twice.
# Usage: tools/ab_env.sh <tag> <inflight> "<lib>|<VAR=val,...>" ...
set -e
TAG=$1; N=$2; shift 2
mkdir -p gpurun_out/$TAG
for i in 1 2; do
  k=0
  for V in "$@"; do
    k=$((k+1))
    L=${V%%|*}; E=${V#*|}
    env $(echo $E | tr ',' ' ') ZFLAC_HIP_LIB=$L timeout -k 10 200 python bench.py --no-e2e --no-cpu-baseline --no-md5 \
      --no-verify --steps 40 --inflight $N > gpurun_out/$TAG/v${k}_$i.json 2> gpurun_out/$TAG/v${k}_$i.err
    echo "v$k $V" > gpurun_out/$TAG/v${k}.name
  done
done
