#!/bin/bash
# Per-kernel SQ counters of two library builds (one rocprofv3 pass each, one run in flight).
# usage: tools/pmc_ab.sh <out-subdir> <libA> <libB>
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=$R/gpurun_out/$1; mkdir -p $O
ARGS="--steps 3 --warmup 1 --no-cpu-baseline --no-verify --no-md5 --no-e2e --inflight 1"
for v in A B; do
  L=$2; [ $v = B ] && L=$3
  case $L in /*) ;; *) L=$R/$L;; esac
  (cd /tmp && export TMPDIR=/tmp ZFLAC_HIP_LIB=$L && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_WAVE_CYCLES --kernel-trace --output-format csv -d $O/$v -o run -- python3 $R/bench.py $ARGS) > $O/$v.log 2>&1 || exit $?
done
python3 - "$O" <<'PY'
import csv, glob, sys, collections
o = sys.argv[1]
for v in "AB":
    f = glob.glob(f"{o}/{v}/**/*counter_collection.csv", recursive=True)
    if not f:
        print(v, "no counter csv"); continue
    acc = collections.defaultdict(lambda: collections.Counter()); n = collections.Counter()
    for r in csv.DictReader(open(f[0])):
        k = r["Kernel_Name"].split("(")[0][:60]
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        n[(k, r["Counter_Name"])] += 1
    for k, c in sorted(acc.items(), key=lambda x: -x[1]["SQ_INSTS_VALU"])[:6]:
        d = n[(k, "SQ_INSTS_VALU")] or 1
        print(v, k, {m: round(x / d / 1e6, 3) for m, x in c.items()})
PY
