#!/bin/bash
# decode+MD5 leg sweep: md5_sweep2.sh <tag> "<inflight run_streams runs hubs>"...
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
O=gpurun_out/$1; shift; mkdir -p $O
for cfg in "$@"; do
  set -- $cfg
  n="i$1_rs$2_r$3_h$4"
  GPU_MAX_HW_QUEUES=$(( $2 + $4 )) timeout -k 10 300 python bench.py --md5-only --md5-steps 96 --warmup 12 --md5-inflight $1 \
      --md5-run-streams $2 --md5-runs $3 --md5-hub-streams $4 > $O/$n.json 2> $O/$n.err || exit $?
  echo "$n $(python -c "import json;d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1]);print(d.get('decode_plus_md5_msps_rank0'), d.get('all_match'), d.get('md5_ms'))")"
done
