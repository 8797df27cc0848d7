#!/bin/bash
# GPU tests, config rows (tools/bench_configs.py --rows ROWS) and a bench A/B against a saved
# build. Usage: tools/r3_rows_ab.sh <tag> <old.so> "<rows>" [rounds]
TAG=$1; OLD=$2; ROWS=$3; R=${4:-2}
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gputest.txt 2>&1 || exit $?
timeout -k 10 400 python tools/bench_configs.py --rows "$ROWS" --steps 5 --out $O/rows_new.json > $O/rows_new.log 2>&1 || exit $?
ZFLAC_HIP_LIB=$OLD timeout -k 10 400 python tools/bench_configs.py --rows "$ROWS" --steps 5 --out $O/rows_old.json > $O/rows_old.log 2>&1 || exit $?
bash tools/ab.sh $TAG $R $OLD zflac_amd/libzflac_hip.so
