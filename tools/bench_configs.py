"""Per-config throughput on one GPU beside the CPU oracle (BASELINE.md's table, SURVEY.md
8(d) sizes), plus the format rows of SURVEY.md 8(f)4 and the repair paths.

For each row one stream (a seeded segment repeated to the row's frame count with
synth.tile_flac: every frame is decoded and the STREAMINFO MD5 covers the whole output):
  * device_msps: channel-samples / wall time of one device-resident zflac_hip_batch_run
    (inputs in HBM, scan .. verify), and its kernel times (HIP events);
  * e2e_msps: the drop-in decode(): zflac_hip_open + zflac_hip_read (upload, device
    decode, copy back overlapped with the host STREAMINFO MD5), best of 2;
  * oracle_1t_msps: the oracle's ReleaseFast-like build on one host thread (zflac decodes
    one stream on one thread), MD5 included, timed on the segment and scaled by the repeats;
  * bit_exact: decode() verified the whole-stream MD5 and the segment equals the oracle.
Usage (GPU box): python tools/bench_configs.py [--rows a,b] [--out file.json]
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

B = 4096
SAT = 32768  # frames of the format rows
ROWS = {
    # name: (flacgen config of one segment, segment frames, total frames, unknown total or
    # "bad_crc8")
    "C2 mono 16-bit fixed-2 k=4": (synth.config_c2(), 1024, 65536, False),
    "C3 stereo M/S 16-bit LPC-8": (synth.config_c3(), 1024, 65536, False),
    "C4 stereo 24-bit LPC-32 shift 15 wasted 4": (synth.config_c4(), 512, 65536, False),
    # format rows at a saturating size: 32,768 frames (512-1,024 decode waves)
    "verbatim stereo 16-bit": (dict(channels=2, bps=16, predictor=0, stereo_mode=1, block_size=B), 256, SAT, False),
    "constant-heavy stereo 16-bit": (dict(channels=2, bps=16, stereo_mode=1, silence_every=1, block_size=B), 256, SAT,
                                     False),
    "mono 8-bit LPC-4": (dict(channels=1, bps=8, order=4, precision=7, block_size=B, noise_lsb=1.0, tone_amp=0.3), 256,
                         SAT, False),
    "stereo 12-bit M/S LPC-8": (dict(channels=2, bps=12, stereo_mode=10, order=8, block_size=B, noise_lsb=4.0), 256,
                                SAT, False),
    "stereo 20-bit M/S LPC-12": (dict(channels=2, bps=20, stereo_mode=10, order=12, precision=14, block_size=B,
                                      noise_lsb=16.0), 256, SAT, False),
    "stereo 32-bit LPC-8": (dict(channels=2, bps=32, stereo_mode=1, order=8, precision=15, block_size=B, tone_amp=0.2,
                                 noise_lsb=1e6), 256, SAT, False),
    "6-channel 24-bit LPC-10": (dict(channels=6, bps=24, order=10, precision=14, block_size=B, noise_lsb=64.0), 128,
                                SAT, False),
    "C3, 2600 frames (a ~4-minute track)": (synth.config_c3(), 2600, 2600, False),
    "C3, total unknown (parallel pass since round 6)": (synth.config_c3(), 256, 4096, True),
    "C3, planted false syncs (repair path)": (dict(channels=2, bps=16, stereo_mode=1, order=8, block_size=B,
                                                   plant_sync_every=2), 256, 4096, False),
    # every header's CRC-8 byte wrong (zflac ignores it): the indexer drops every header and
    # the sequential planner finds the frames through its batched probes
    "C3, every header CRC-8 wrong (batched probes)": (synth.config_c3(), 4096, 4096, "bad_crc8"),
}


def run_row(name, cfg, seg, frames, unknown, steps, walk=None):
    st = synth.generate(**dict(cfg, n_samples=B * seg, seed=cfg.get("seed", 7)))
    reps = max(1, frames // seg)
    if unknown == "bad_crc8":  # one generated stream, every header CRC-8 flipped
        b = bytearray(st.flac)
        for off in st.frame_offsets:
            b[synth.header_crc8_index(st.flac, int(off))] ^= 0x5A
        data, reps = bytes(b), 1
    else:
        data = synth.tile_flac(st, reps, unknown_total=unknown)
    n = st.pcm.size * reps
    # device-resident batch runs
    b = zflac_amd.Batch([data], timing=True, walk=walk)
    for _ in range(2):
        b.run()
    walls, tms = [], []
    for _ in range(steps):
        t = time.perf_counter()
        b.run()
        walls.append(time.perf_counter() - t)
        tms.append(b.timings())
    b.close()
    # decode() end to end (raises InvalidChecksum unless the whole output is bit-exact)
    best, tm = None, {}
    for _ in range(2):
        cur = {}
        t0 = time.perf_counter()
        d = zflac_amd.decode(data, timings=cur)
        w = time.perf_counter() - t0
        if best is None or w < best:
            best, tm = w, cur
        assert d.samples.values.size == n
    seg_ref = oracle.decode(st.flac, "fast")
    exact = seg_ref.error == "OK" and np.array_equal(d.samples.values[: seg_ref.samples.size], seg_ref.samples)
    del d
    # oracle, one thread, on the segment
    reps_cpu, t_cpu = 0, 0.0
    while t_cpu < 1.0 or reps_cpu == 0:
        t = time.perf_counter()
        err, ns = oracle.decode_count_only(st.flac, "fast")
        t_cpu += time.perf_counter() - t
        reps_cpu += 1
        assert err == 0
    cpu_msps = st.pcm.size * reps_cpu / t_cpu / 1e6
    wall = float(np.median(walls))
    mean = lambda f: round(float(np.mean([f(t) for t in tms])), 4)  # noqa: E731
    # algorithmic bytes: compressed frame bytes read + PCM bytes written
    out_bytes = n * (1 if cfg["bps"] <= 8 else 2 if cfg["bps"] <= 16 else 4)
    alg = (len(data) - int(st.frame_offsets[0])) + out_bytes
    dec_ms = mean(lambda t: t.decode_ms)
    # a launch that decoded nothing of the row (every frame left to the sequential planner)
    # gives no roofline figure: a fraction above 1 of HBM is not a measurement
    dec_frac = round(alg / (dec_ms * 1e-3) / 8e12, 4) if dec_ms else None
    if dec_frac is not None and dec_frac > 1.0:
        dec_frac = None
    return {
        "row": name, "walk": walk or "auto", "frames": seg * reps, "channel_samples": int(n), "compressed_bytes": len(data),
        "device_msps": round(n / wall / 1e6, 1), "device_wall_ms": round(wall * 1e3, 3),
        "scan_ms": mean(lambda t: t.scan_ms), "walk_ms": mean(lambda t: t.walk_ms),
        "decode_ms": mean(lambda t: t.decode_ms), "verify_ms": mean(lambda t: t.verify_ms),
        "e2e_msps": round(n / best / 1e6, 1), "e2e_ms": round(best * 1e3, 1),
        "e2e_breakdown_ms": {k: round(tm[k], 2) for k in ("upload_ms", "run_wall_ms", "read_ms", "host_md5_ms")},
        "oracle_1t_msps": round(cpu_msps, 1), "device_over_oracle_1t": round(n / wall / 1e6 / cpu_msps, 1),
        "e2e_over_oracle_1t": round(n / best / 1e6 / cpu_msps, 2), "bit_exact": bool(exact),
        "alg_bytes": int(alg), "decode_kernel_frac_of_8TBs": dec_frac,
        "device_run_frac_of_8TBs": round(alg / wall / 8e12, 4),
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", help="comma-separated substrings of row names (default: all)")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--out")
    ap.add_argument("--walk", default="auto", help="auto, lane, wave, or both (each row twice)")
    a = ap.parse_args()
    sel = [r for r in ROWS if not a.rows or any(x in r for x in a.rows.split(","))]
    rows = []
    for name in sel:
        cfg, seg, frames, unknown = ROWS[name]
        for w in (["lane", "wave"] if a.walk == "both" else [None if a.walk == "auto" else a.walk]):
            r = run_row(name, cfg, seg, frames, unknown, a.steps, w)
            print(json.dumps(r), flush=True)
            rows.append(r)
    if a.out:
        import zflac_amd

        with open(a.out, "w") as f:  # the loaded library's embedded build id (zflac_hip_build_id)
            json.dump({"build_id": zflac_amd.build_id(), "lib": zflac_amd.lib_path, "rows": rows}, f, indent=1)
    if not all(r["bit_exact"] for r in rows):
        sys.exit(1)


if __name__ == "__main__":
    main()
