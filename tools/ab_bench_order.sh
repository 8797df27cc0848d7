#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/abb; mkdir -p $O
for i in 1 2 3; do for b in bench_prev bench; do
  timeout -k 10 200 python $b.py --steps 20 --warmup 5 --no-cpu-baseline --no-e2e --no-md5 > $O/${b}_$i.json 2> $O/${b}_$i.err || exit 1
  echo "$b $i $(python -c "import json;d=json.loads(open('$O/${b}_$i.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['roofline']['kernel_ms'],d['ms_per_step_serial'])")"
done; done
