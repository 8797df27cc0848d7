set -o pipefail
bash tools/gpu_check.sh r3a || exit $?
bash tools/r3_profile.sh r3a_prof
