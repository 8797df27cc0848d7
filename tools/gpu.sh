#!/bin/bash
# The one GPU-box runner for every measurement this repository commits under profiles/.
# Each step has its own time limit; steps are chained so the first failure ends the call.
# Output goes to gpurun_out/<tag>/ (merged back by gpurun); copy what is judged to profiles/.
#
#   tools/gpu.sh check   <tag> [bench args]   GPU tests, smoke(), one default bench line
#   tools/gpu.sh tests   <tag> [pytest -k]    GPU tests only
#   tools/gpu.sh bench   <tag> [bench args]   one bench line
#   tools/gpu.sh profile <tag> [bench args]   rocprofv3 --kernel-trace --stats of the bench
#                                             workload: serial (one run in flight, the isolated
#                                             launches the roofline uses) and the bench's default
#                                             runs in flight (four; round-4 profiles: three)
#   tools/gpu.sh md5leg  <tag> <name> [args]  the decode+MD5 leg alone (MD5Q hardware queues, default 8 =
#                                             bench's 5 run + 3 md5 hub streams)
#   tools/gpu.sh md5trace <tag>               rocprofv3 kernel trace of the decode+MD5 leg alone
#   tools/gpu.sh pmc     <tag>                PMC passes (one rocprofv3 run per pass, counters only)
#                                             + FETCH/WRITE calibration + summary (pmc_summary.json,
#                                             also copied to profiles/pmc_current.json on the box)
#   tools/gpu.sh configs <tag> [bench_configs args]   per-config / per-format rows (configs.json)
#   tools/gpu.sh rowprof <tag> <row substring>...     rocprofv3 kernel stats of bench_configs rows
#   tools/gpu.sh ab      <tag> <rounds> <lib.so>...   same-box bench A/B of library builds
#                                                     (ZFLAC_HIP_LIB, alternating; AB_ARGS = bench args)
#   tools/gpu.sh probe   <tag> <c2|c3|1250|row:...>... timing probe (-DZFLAC_PROBE build in
#                                                     tools/_build/lib_probe.so)
#   tools/gpu.sh final   <tag>                pmc, check, profile, configs: the round's measurement set
#
# Libraries are built beforehand on the CPU host (python -c "import __graft_entry__ as g; g.build()"),
# never inside a GPU call.
R=${GRAFT_REPO_ROOT:-$(pwd)}
CMD=$1; TAG=$2; shift 2
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
QUIET="--no-cpu-baseline --no-e2e --no-md5"

prof() {  # prof <outdir> <cmd...>: rocprofv3 kernel statistics of one command
  local d=$1; shift
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
      -d $d -o run -- "$@")
}

case $CMD in
  tests)
    timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${1:+-k "$1"} \
        > $O/gputest.txt 2>&1
    ;;
  bench)
    timeout -k 10 600 python bench.py "$@" > $O/bench.json 2> $O/bench.err
    ;;
  check)
    timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
        > $O/gputest.txt 2>&1 || exit $?
    timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit $?
    timeout -k 10 600 python bench.py "$@" > $O/bench.json 2> $O/bench.err
    ;;
  profile)
    prof $O/serial python3 $R/bench.py --steps 20 --warmup 3 $QUIET --inflight 1 "$@" > $O/serial.log 2>&1 || exit $?
    prof $O/inflight python3 $R/bench.py --steps 20 --warmup 3 $QUIET "$@" > $O/inflight.log 2>&1
    ;;
  md5leg)  # md5leg <tag> <name> [bench args]: the decode+MD5 leg alone
    NAME=$1; shift
    GPU_MAX_HW_QUEUES=${MD5Q:-8} timeout -k 10 300 python bench.py --md5-only --md5-steps 48 --warmup 12 "$@" \
        > $O/$NAME.json 2> $O/$NAME.err
    ;;
  md5trace)
    export GPU_MAX_HW_QUEUES=${MD5Q:-8}  # as the bench's decode+MD5 child runs (set before rocprofv3, not via env)
    prof $O/md5leg python3 $R/bench.py --md5-only --md5-steps 36 --warmup 12 "$@" > $O/md5leg.log 2>&1
    ;;
  pmc)
    ARGS="--steps 3 --warmup 1 --no-cpu-baseline --no-verify --no-md5 --no-e2e --inflight 1"
    P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_WAVE_CYCLES"
    P2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES"
    P3="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VMEM SQ_WAVES"
    i=0
    for P in "$P1" "$P2" "$P3" "FETCH_SIZE" "WRITE_SIZE"; do
      i=$((i+1))
      (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $O/pmc/p$i \
          -o run -- python3 $R/bench.py $ARGS) > $O/pmc_p$i.log 2>&1 || exit $?
    done
    for P in FETCH_SIZE WRITE_SIZE; do
      (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 60 rocprofv3 --pmc $P --output-format csv \
          -d $O/pmc/calib_$P -o run -- $R/tools/_build/calib_pmc) > $O/pmc_calib_$P.log 2>&1 || exit $?
    done
    python3 tools/pmc_summary.py $O/pmc --json $O/pmc_summary.json > $O/pmc_summary.log 2>&1 || exit $?
    cp $O/pmc_summary.json profiles/pmc_current.json
    ;;
  configs)
    timeout -k 10 1100 python tools/bench_configs.py --steps 5 --out $O/configs.json "$@" > $O/configs.log 2>&1
    ;;
  rowprof)
    for r in "$@"; do
      n=$(echo "$r" | tr -c 'A-Za-z0-9\n' '_')
      prof $O/$n python3 $R/tools/bench_configs.py --rows "$r" --steps 5 --out $O/$n.json > $O/$n.log 2>&1 || exit $?
    done
    ;;
  ab)
    ROUNDS=$1; shift
    for i in $(seq 1 $ROUNDS); do
      for L in "$@"; do
        n=$(basename $L .so)
        ZFLAC_HIP_LIB=$L timeout -k 10 200 python bench.py $QUIET --steps 30 ${AB_ARGS} \
            > $O/${n}_$i.json 2> $O/${n}_$i.err || exit $?
      done
    done
    python3 tools/ab_summary.py $O $O/summary.json > $O/summary.txt 2>&1
    ;;
  probe)
    for c in "$@"; do
      n=$(echo "$c" | tr -c 'A-Za-z0-9\n' '_')
      ZFLAC_HIP_LIB=tools/_build/lib_probe.so timeout -k 10 300 python tools/probe.py "$c" > $O/probe_$n.json \
          2> $O/probe_$n.err || exit $?
    done
    ;;
  final)
    bash tools/gpu.sh pmc $TAG || exit $?
    bash tools/gpu.sh check $TAG || exit $?
    bash tools/gpu.sh profile $TAG || exit $?
    bash tools/gpu.sh configs $TAG
    ;;
  *)
    echo "usage: tools/gpu.sh {check|tests|bench|profile|md5trace|pmc|configs|rowprof|ab|probe|final} <tag> ..." >&2
    exit 2
    ;;
esac
