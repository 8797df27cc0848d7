#!/bin/bash
# Per-config rows (tools/bench_configs.py, every row, the library's own walk choice) into
# gpurun_out/<tag>/configs.json. Usage: tools/r3_configs.sh <tag> [extra args]
TAG=${1:-r3cfg}; shift
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 900 python tools/bench_configs.py --steps 5 --out $O/configs.json "$@" > $O/configs.log 2>&1
