#!/bin/bash
# rocprofv3 kernel statistics of the C2 / C3 / C4 config rows (tools/bench_configs.py).
# Usage: tools/r3_profile_rows.sh <tag>
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for r in "C2 mono" "C3 stereo" "C4 stereo"; do
  n=$(echo $r | cut -c1-2)
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$n -o run -- \
      python3 $R/tools/bench_configs.py --rows "$r" --steps 5 --out $O/$n.json > $O/$n.log 2>&1 || exit $?
done
