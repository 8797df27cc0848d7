bash tools/r3_pmc_check.sh v39 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/v39_prof/serial -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --no-md5 --inflight 1 > $GRAFT_REPO_ROOT/gpurun_out/v39_prof_serial.log 2>&1
