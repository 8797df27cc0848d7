#!/bin/bash
# Timing probe of C2, C3 and the C5 shard (tools/probe.py, -DZFLAC_PROBE build) and the op-issue
# microbenchmark. Usage: tools/r3_probe.sh <tag>
O=gpurun_out/$1; mkdir -p $O
for c in c2 c3 1250; do
  ZFLAC_HIP_LIB=tools/_build/lib_probe.so timeout -k 10 300 python tools/probe.py $c > $O/probe_$c.json 2> $O/probe_$c.err || exit $?
done
timeout -k 10 120 tools/_build/ubench_ops > $O/ubench_ops.json 2> $O/ubench_ops.err
