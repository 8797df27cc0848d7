#!/bin/bash
# Timing probe (tools/probe.py, -DZFLAC_PROBE build) of bench_configs rows. Usage: tools/r3_probe_rows.sh <tag> <row>...
O=gpurun_out/$1; shift; mkdir -p $O
i=0
for r in "$@"; do
  i=$((i+1))
  ZFLAC_HIP_LIB=tools/_build/lib_probe.so timeout -k 10 300 python tools/probe.py "row:$r" > $O/probe_$i.json 2> $O/probe_$i.err || exit $?
done
