#!/bin/bash
# PMC passes of the bench workload (tools/pmc.sh) and the per-config rows (tools/r3_configs.sh)
# on the current build. Usage: tools/r3_pmc_configs.sh <tag>
TAG=${1:-r3pc}
bash tools/pmc.sh ${TAG}_pmc || exit $?
bash tools/r3_configs.sh ${TAG}_cfg
