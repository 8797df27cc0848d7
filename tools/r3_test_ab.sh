#!/bin/bash
# GPU tests of the current build, then a same-box bench A/B against a saved build.
# Usage: tools/r3_test_ab.sh <tag> <old.so> [rounds]
TAG=$1; OLD=$2; R=${3:-3}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gputest.txt 2>&1 || exit $?
bash tools/ab.sh $TAG $R $OLD zflac_amd/libzflac_hip.so
