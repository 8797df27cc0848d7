#!/bin/bash
# GPU tests, smoke and a default bench run into gpurun_out/<tag> (on the GPU box).
# Usage: tools/gpu_check.sh <tag> [bench args...]
TAG=${1:-check}; shift
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gputest.txt 2>&1 || exit $?
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit $?
timeout -k 10 400 python bench.py "$@" > $O/bench.json 2> $O/bench.err
