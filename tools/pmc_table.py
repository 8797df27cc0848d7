"""Print per-dispatch PMC counters of one kernel from `tools/gpu.sh pmc` output dirs.
Usage: python tools/pmc_table.py <kernel substring> gpurun_out/<tag> [gpurun_out/<tag2> ...]"""
import csv, glob, os, sys
from collections import defaultdict

kern = sys.argv[1]
cols = {}
for d in sys.argv[2:]:
    acc = defaultdict(float)
    disp = defaultdict(set)
    for f in glob.glob(os.path.join(d, "p*", "*counter_collection.csv")):
        for row in csv.DictReader(open(f)):
            if kern not in row["Kernel_Name"]:
                continue
            acc[row["Counter_Name"]] += float(row["Counter_Value"])
            disp[row["Counter_Name"]].add(row["Dispatch_Id"])
    cols[d] = {c: v / len(disp[c]) for c, v in acc.items()}
names = sorted({c for v in cols.values() for c in v})
print("%-40s" % "counter" + "".join("%18s" % os.path.basename(d) for d in cols))
for c in names:
    print("%-40s" % c + "".join("%18.4g" % cols[d].get(c, float("nan")) for d in cols))
