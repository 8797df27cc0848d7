"""Summarise a `tools/gpu.sh pmc` run: per-kernel PMC counters per dispatch, FETCH/WRITE calibration
factors from tools/calib_pmc.hip, and the corrected HBM traffic of the decode kernel.

Usage: python tools/pmc_summary.py gpurun_out/<tag> [--json out.json]
FETCH_SIZE / WRITE_SIZE are in KiB per dispatch (rocprofv3).
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
from collections import defaultdict


def load(path):
    """{kernel: {counter: [values per dispatch]}} from every counter_collection.csv under path."""
    acc = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        per = defaultdict(float)
        names = {}
        for row in csv.DictReader(open(f)):
            key = (row["Dispatch_Id"], row["Counter_Name"])
            per[key] += float(row["Counter_Value"])  # sum over dimensions (XCDs / SEs)
            names[row["Dispatch_Id"]] = row["Kernel_Name"]
        for (d, c), v in per.items():
            acc[names[d]][c].append(v)
    return acc


def short(name):
    return name.split("(")[0].replace("void ", "")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--json")
    ap.add_argument("--lib", help="library the counters were taken on (default: the in-tree build)")
    ap.add_argument("--store-pattern", choices=["runs", "private"], default="runs",
                    help="store pattern of the decode kernel: staged 128-B runs (16-bit stereo) or per-lane")
    a = ap.parse_args()
    calib = load(os.path.join(a.dir, "calib_FETCH_SIZE"))
    calib_w = load(os.path.join(a.dir, "calib_WRITE_SIZE"))
    nbytes = 5242880000.0  # tools/calib_pmc.hip: LANE_BYTES * LANES
    f_read = w_write = w_runs = None
    for k, v in calib.items():
        if "k_read_private" in k:
            f_read = nbytes / (sum(v["FETCH_SIZE"]) / len(v["FETCH_SIZE"]) * 1024)
    for k, v in calib_w.items():
        if "k_write_private" in k:
            w_write = nbytes / (sum(v["WRITE_SIZE"]) / len(v["WRITE_SIZE"]) * 1024)
        if "k_write_runs" in k:
            w_runs = nbytes / (sum(v["WRITE_SIZE"]) / len(v["WRITE_SIZE"]) * 1024)
    lib = a.lib or os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "zflac_amd",
                                "libzflac_hip.so")
    import hashlib

    out = {"calibration": {"fetch_factor_private_16B": f_read, "write_factor_private_16B": w_write,
                           "write_factor_runs_128B": w_runs},
           "lib_sha256": hashlib.sha256(open(lib, "rb").read()).hexdigest(), "_source": a.dir, "kernels": {}}
    # the source fingerprint embedded in the measured library itself (builds are not
    # bit-reproducible; bench.py matches the library it loads against this)
    import sys

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from zflac_amd import build as zbuild

    bid = zbuild.lib_build_id(lib)
    out["src_sha256"] = bid[4:] if bid else None
    runs = [d for d in sorted(glob.glob(os.path.join(a.dir, "p*"))) if os.path.isdir(d)]
    merged = defaultdict(dict)
    for d in runs:
        for k, cs in load(d).items():
            for c, vals in cs.items():
                merged[short(k)][c] = sum(vals) / len(vals)
    for k, cs in merged.items():
        row = dict(cs)
        if "FETCH_SIZE" in cs and f_read:
            row["hbm_read_bytes"] = cs["FETCH_SIZE"] * 1024 * f_read
        wf = w_runs if a.store_pattern == "runs" else w_write
        if "WRITE_SIZE" in cs and wf:
            row["hbm_write_bytes"] = cs["WRITE_SIZE"] * 1024 * wf
        if "hbm_read_bytes" in row and "hbm_write_bytes" in row:
            row["hbm_traffic_bytes"] = row["hbm_read_bytes"] + row["hbm_write_bytes"]
        w = cs.get("SQ_WAVES")
        if w:
            for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR",
                      "SQ_INSTS_BRANCH", "SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_ACTIVE_INST_ANY"):
                if c in cs:
                    row[c + "_per_wave"] = cs[c] / w
        out["kernels"][k] = row
    txt = json.dumps(out, indent=1, sort_keys=True)
    print(txt)
    if a.json:
        with open(a.json, "w") as f:
            f.write(txt + "\n")


if __name__ == "__main__":
    main()
