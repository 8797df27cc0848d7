"""Per-config throughput on one GPU beside the CPU oracle (BASELINE.md's table).

For each BASELINE.json config that runs on one GPU (C2 mono fixed-2, C3 mid/side LPC-8,
C4 24-bit LPC-32 with wasted bits: one long stream each; C3 also as a 1250-stream batch
is bench.py's workload) this decodes the stream with the HIP path, inputs resident in HBM,
and reports:
  * gpu_msps: channel-samples / wall time of one device-resident run (scan..verify);
  * kernel times (scan+compact, walk, decode) from the library's HIP events;
  * cpu_1t_msps: the oracle's ReleaseFast-like build on one host thread, same stream
    (zflac decodes one stream on one thread), MD5 included;
  * bit_exact: every run's PCM hashes to the STREAMINFO MD5, and equals the oracle.
Usage (GPU box): python tools/bench_configs.py [--frames N] [--out file.json]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

import oracle  # noqa: E402  (CPU baseline and checker only)
import synth  # noqa: E402
import zflac_amd  # noqa: E402


def run_config(name, cfg, steps, cpu_seconds):
    t0 = time.perf_counter()
    st = synth.generate(**cfg)
    gen_s = time.perf_counter() - t0
    b = zflac_amd.Batch([st.flac], timing=True)
    for _ in range(2):
        b.run()
    walls, tms = [], []
    for _ in range(steps):
        t = time.perf_counter()
        b.run()
        walls.append(time.perf_counter() - t)
        tms.append(b.timings())
    d = b.read(0, verify_md5=True)  # raises InvalidChecksum on a mismatch
    ref = oracle.decode(st.flac, "fast")
    exact = ref.error == "OK" and np.array_equal(d.samples.values, ref.samples)
    n = d.samples.values.size
    b.close()
    # CPU: the oracle, one thread, whole stream decodes for ~cpu_seconds
    reps, t_cpu = 0, 0.0
    while t_cpu < cpu_seconds or reps == 0:
        t = time.perf_counter()
        err, ns = oracle.decode_count_only(st.flac)
        t_cpu += time.perf_counter() - t
        reps += 1
        assert err == 0 and ns == n
    wall = float(np.median(walls))
    return {
        "config": name, "channel_samples": int(n), "compressed_bytes": len(st.flac),
        "bytes_per_sample_alg": round((len(st.flac) + d.samples.values.nbytes) / n, 3),
        "gpu_msps": round(n / wall / 1e6, 1), "gpu_wall_ms": round(wall * 1e3, 3),
        "scan_ms": round(float(np.mean([t.scan_ms for t in tms])), 4),
        "walk_ms": round(float(np.mean([t.walk_ms for t in tms])), 4),
        "decode_ms": round(float(np.mean([t.decode_ms for t in tms])), 4),
        "decode_kernel_msps": round(n / (float(np.mean([t.decode_ms + t.walk_ms for t in tms])) * 1e-3) / 1e6, 1),
        "cpu_1t_msps": round(n * reps / t_cpu / 1e6, 1), "cpu_sample": f"{reps} whole-stream decodes, 1 thread",
        "gpu_over_cpu_1t": round((n / wall) / (n * reps / t_cpu), 1),
        "bit_exact": bool(exact), "gen_seconds": round(gen_s, 2),
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=4096, help="frames per stream (block 4096)")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--cpu-seconds", type=float, default=3.0)
    ap.add_argument("--out")
    a = ap.parse_args()
    cfgs = {
        "C2 mono 16-bit fixed-2 k=4": synth.config_c2(n_frames=a.frames),
        "C3 stereo mid/side 16-bit LPC-8": synth.config_c3(n_frames=a.frames),
        "C4 stereo 24-bit LPC-32 shift 15, 4 wasted bits": synth.config_c4(n_frames=a.frames),
    }
    rows = []
    for name, cfg in cfgs.items():
        r = run_config(name, cfg, a.steps, a.cpu_seconds)
        print(json.dumps(r), flush=True)
        rows.append(r)
    if a.out:
        with open(a.out, "w") as f:
            json.dump({"frames_per_stream": a.frames, "rows": rows}, f, indent=1)
    if not all(r["bit_exact"] for r in rows):
        sys.exit(1)


if __name__ == "__main__":
    main()
