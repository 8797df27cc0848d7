"""Concurrency of kernels in a rocprofv3 kernel trace (`tools/gpu.sh md5trace`, `profile`):
per kernel name, count, mean duration, and how many dispatches of it run at once on
average and at most (time-weighted over the span from its first start to its last end);
plus the queues the dispatches used. Usage: python tools/trace_overlap.py <dir with
*kernel_trace.csv> [--json out.json] [--kernel substring]"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
from collections import defaultdict


def load(path):
    rows = []
    for f in glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
            rows.append({"name": name.split("(")[0],
                         "start": int(r["Start_Timestamp"]), "end": int(r["End_Timestamp"]),
                         "queue": r.get("Queue_Id"), "stream": r.get("Stream_Id")})
    return rows


def concurrency(iv):
    """Time-weighted mean and max number of overlapping [start, end) intervals."""
    ev = sorted([(s, 1) for s, _ in iv] + [(e, -1) for _, e in iv])
    cur = mx = 0
    acc = 0.0
    last = ev[0][0] if ev else 0
    for t, d in ev:
        acc += cur * (t - last)
        last = t
        cur += d
        mx = max(mx, cur)
    span = (ev[-1][0] - ev[0][0]) if ev else 0
    return (acc / span if span else 0.0), mx, span


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--json")
    ap.add_argument("--kernel", default="")
    a = ap.parse_args()
    rows = load(a.dir)
    by = defaultdict(list)
    for r in rows:
        if a.kernel in r["name"]:
            by[r["name"]].append(r)
    out = {"source": a.dir, "dispatches": len(rows), "kernels": {}}
    for name, rs in sorted(by.items(), key=lambda kv: -sum(r["end"] - r["start"] for r in kv[1])):
        mean_c, max_c, span = concurrency([(r["start"], r["end"]) for r in rs])
        out["kernels"][name] = {
            "count": len(rs), "mean_us": round(sum(r["end"] - r["start"] for r in rs) / len(rs) / 1e3, 2),
            "span_ms": round(span / 1e6, 3), "mean_concurrent": round(mean_c, 2), "max_concurrent": max_c,
            "queues": len({r["queue"] for r in rs}), "streams": len({r["stream"] for r in rs})}
    allc, allm, span = concurrency([(r["start"], r["end"]) for r in rows])
    out["all"] = {"mean_concurrent": round(allc, 2), "max_concurrent": allm, "span_ms": round(span / 1e6, 3),
                  "queues": len({r["queue"] for r in rows})}
    txt = json.dumps(out, indent=1)
    print(txt)
    if a.json:
        with open(a.json, "w") as f:
            f.write(txt + "\n")


if __name__ == "__main__":
    main()
