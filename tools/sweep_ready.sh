#!/bin/bash
# bench.py runs-in-flight sweep with ready-order scheduling: sweep_ready.sh <tag> <inflight>...
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
O=gpurun_out/$1; shift; mkdir -p $O
QUIET="--no-cpu-baseline --no-e2e --no-md5"
for n in "$@"; do
  timeout -k 10 200 python bench.py $QUIET --steps 20 --sched ready --inflight $n > $O/i$n.json 2> $O/i$n.err || exit $?
  echo "i$n $(python -c "import json;d=json.loads(open('$O/i$n.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'])")"
done
