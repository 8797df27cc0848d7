#!/bin/bash
# decode+MD5 leg at several timed run counts on one box: md5_steps_sweep.sh <tag> <runs>...
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
O=gpurun_out/$1; shift; mkdir -p $O
for n in "$@"; do
  GPU_MAX_HW_QUEUES=7 timeout -k 10 300 python bench.py --md5-only --md5-steps $n --warmup 12 > $O/m$n.json 2> $O/m$n.err || exit $?
  echo "m$n $(python -c "import json;d=json.loads(open('$O/m$n.json').read().strip().splitlines()[-1]);m=d.get('device_md5',d);print(m['decode_plus_md5_msps_rank0'],m['ms_per_step'],m['all_match'])")"
done
