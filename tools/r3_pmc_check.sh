#!/bin/bash
# PMC passes + summary of the current build (into profiles/pmc_current.json on the box and
# gpurun_out/<tag>/pmc_summary.json), then GPU tests, smoke and the default bench line.
TAG=${1:-r3pc}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG; mkdir -p $O
cd $R
bash tools/pmc.sh ${TAG}_pmc || exit $?
python3 tools/pmc_summary.py gpurun_out/${TAG}_pmc --json $O/pmc_summary.json > $O/pmc_summary.log 2>&1 || exit $?
cp $O/pmc_summary.json profiles/pmc_current.json
bash tools/gpu_check.sh $TAG
