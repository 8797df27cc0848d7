"""Summarise a same-box A/B (`tools/gpu.sh ab` output dir) into one JSON: per library, each run's
value / ms_per_step / serial step / isolated stage times. Usage: ab_summary.py <dir> <out.json> [note]"""
import glob
import json
import os
import sys

d, out = sys.argv[1], sys.argv[2]
note = sys.argv[3] if len(sys.argv) > 3 else ""
rows = {}
for f in sorted(glob.glob(os.path.join(d, "*.json"))):
    lib, run = os.path.basename(f)[:-5].rsplit("_", 1)
    if not run.isdigit():  # not a bench line (config rows of the same call)
        continue
    j = json.load(open(f))
    rows.setdefault(lib, []).append({"run": int(run), "value": j["value"], "ms_per_step": j["ms_per_step"],
                                     "ms_per_step_serial": j.get("ms_per_step_serial"), "stages_ms": j["stages_ms"],
                                     "bit_exact": j["bit_exact"], "lib_sha256": j.get("lib_sha256")})
gt = os.path.join(d, "gputest.txt")
res = {"source": d, "note": note, "libs": rows}
if os.path.exists(gt):
    res["gputest"] = open(gt).read().strip().splitlines()[-1]
json.dump(res, open(out, "w"), indent=1)
print(json.dumps({k: [r["value"] for r in v] for k, v in rows.items()}))
