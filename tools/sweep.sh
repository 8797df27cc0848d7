#!/bin/bash
# Decode-kernel time vs. number of streams (waves) on one GPU: tools/sweep.sh <tag> [counts...]
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-sweep}; shift
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
for n in ${@:-256 512 1024 1250 2048}; do
  timeout -k 10 120 python3 $R/bench.py --streams-per-gpu $n --steps 10 --warmup 2 --no-cpu-baseline --no-verify > $OUT/n$n.json 2> $OUT/n$n.err || exit 1
  python3 -c "import json,sys; d=json.load(open('$OUT/n$n.json')); print($n, d['stages_ms'], d['roofline']['frac'])" >> $OUT/summary.txt
done
