#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
O=gpurun_out/$1; mkdir -p $O
QUIET="--no-cpu-baseline --no-e2e --no-md5"
for cfg in "4 4" "4 8" "6 8" "8 8" "8 12" "4 4"; do
  set -- $cfg
  GPU_MAX_HW_QUEUES=$2 timeout -k 10 200 python bench.py $QUIET --steps 30 --inflight $1 > $O/i$1_q$2.json 2> $O/i$1_q$2.err || exit $?
  echo "$cfg $(python -c "import json;d=json.loads(open('$O/i$1_q$2.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'])")"
done
