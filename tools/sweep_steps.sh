#!/bin/bash
# bench.py step-count / scheduling sweep on one box: sweep_steps.sh <tag> "<steps> <sched>"...
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
O=gpurun_out/$1; shift; mkdir -p $O
QUIET="--no-cpu-baseline --no-e2e --no-md5"
for cfg in "$@"; do
  set -- $cfg
  n="s$1_$2"
  timeout -k 10 200 python bench.py $QUIET --steps $1 --sched $2 > $O/$n.json 2> $O/$n.err || exit $?
  echo "$n $(python -c "import json;d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'])")"
done
