#!/bin/bash
# Runs in flight A/B on the current build: bench with --inflight 2..5, twice each, alternating.
O=gpurun_out/$1; mkdir -p $O
for i in 1 2; do for n in 3 4 5 2; do
  timeout -k 10 200 python bench.py --no-e2e --no-cpu-baseline --no-md5 --steps 30 --inflight $n > $O/inf${n}_$i.json 2> $O/inf${n}_$i.err || exit $?
done; done
