#!/bin/bash
# Same-box A/B of two library builds: alternating short bench runs (quiet legs off).
# usage: tools/ab_lib.sh <out-subdir> <libA> <libB> [reps]
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
O=gpurun_out/$1; mkdir -p $O
A=$2; B=$3; N=${4:-3}
QUIET="--no-cpu-baseline --no-e2e --no-md5"
for i in $(seq 1 $N); do
  for v in A B; do
    L=$A; [ $v = B ] && L=$B
    ZFLAC_HIP_LIB=$L timeout -k 10 200 python bench.py $QUIET --steps 20 > $O/${v}_$i.json 2> $O/${v}_$i.err || exit $?
    echo "$v $i $(python -c "import json;d=json.loads(open('$O/${v}_$i.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['stages_ms'])")"
  done
done
