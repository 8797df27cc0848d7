#!/bin/bash
# Round-3 measurement set of the current build (GPU box): PMC passes and their summary (so the
# bench line's roofline.traffic is filled from the same build), GPU tests, smoke, the default
# bench line, rocprof kernel stats (serial / three in flight), every config row.
# Usage: tools/r3_final.sh <tag>
TAG=${1:-r3final}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG; mkdir -p $O
cd $R
bash tools/pmc.sh ${TAG}_pmc || exit $?
python3 tools/pmc_summary.py gpurun_out/${TAG}_pmc --json $O/pmc_summary.json > $O/pmc_summary.log 2>&1 || exit $?
cp $O/pmc_summary.json profiles/pmc_current.json
bash tools/gpu_check.sh $TAG || exit $?
bash tools/r3_profile.sh ${TAG}_prof || exit $?
bash tools/r3_configs.sh ${TAG}_cfg
