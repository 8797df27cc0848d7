#!/bin/bash
# Decode+MD5 leg sweep over hash workgroup shapes / hub settings: md5_sweep.sh <tag> "<W runs hubs>"...
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
O=gpurun_out/$1; shift; mkdir -p $O
for cfg in "$@"; do
  set -- $cfg
  n="w$1_r$2_h$3"
  ZFLAC_MD5_WG_WAVES=$1 GPU_MAX_HW_QUEUES=${MD5Q:-7} timeout -k 10 300 python bench.py --md5-only --md5-steps 96 --warmup 12 \
      --md5-runs $2 --md5-hub-streams $3 > $O/$n.json 2> $O/$n.err || exit $?
  echo "$n $(python -c "import json;d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1]);print(d.get('decode_plus_md5_msps_rank0'), d.get('all_match'), d.get('md5_ms'))")"
done
