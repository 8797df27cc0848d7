"""Benchmark: device-resident FLAC decode of the C5 per-GPU shard.

Workload (BASELINE.json configs[4], per-GPU share; its codec parameters are configs[2]):
1250 independent stereo 16-bit mid/side streams per GPU, 32 frames x 4096 samples each,
LPC order 8 (synthetic, seeded per global stream index). One "step" = one call of
zflac_hip_batch_run over the rank's whole shard: frame-sync scan, candidate compaction,
subframe decode (Rice, LPC rollback, decorrelation, PCM pack-out) and chain verification,
inputs already in HBM, outputs left in HBM. N GPUs = N ranks with disjoint shards (weak
scaling, no collective in the data path; torch.distributed only for the timing barrier
and the max over ranks).

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

STREAMS_PER_GPU = 1250
FRAMES_PER_STREAM = 32
BLOCK = 4096
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md, HBM3E peak
# PMC summary of the current k_decode build (tools/pmc.sh + tools/pmc_summary.py; FETCH_SIZE /
# WRITE_SIZE corrected by the factors tools/calib_pmc.hip measures for this access pattern)
PMC_SUMMARY = os.path.join(ROOT, "profiles", "pmc_current.json")


def pmc_traffic(kernel: str):
    """Corrected HBM bytes per launch of `kernel` from the committed PMC summary, or None."""
    try:
        with open(PMC_SUMMARY) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    row = d.get("kernels", {}).get(kernel)
    if not row or "hbm_traffic_bytes" not in row:
        return None
    return {"bytes": int(row["hbm_traffic_bytes"]), "read": int(row["hbm_read_bytes"]),
            "write": int(row["hbm_write_bytes"]), "source": os.path.relpath(d.get("_source", PMC_SUMMARY), ROOT)}


def parse_args():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--streams-per-gpu", type=int, default=STREAMS_PER_GPU)
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline sample budget")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--no-md5", action="store_true", help="skip the device-MD5 leg")
    return ap.parse_args()


def make_shard(rank: int, world: int, n_streams: int):
    import synth
    from zflac_amd.shard import shard_range

    cfgs = [synth.config_c5(g, n_frames=FRAMES_PER_STREAM) for g in shard_range(rank, world, n_streams)]
    out = [None] * n_streams
    workers = min(16, os.cpu_count() or 1)

    def work(k):
        for i in range(k, n_streams, workers):
            st = synth.generate(**cfgs[i])
            out[i] = st.flac  # keep only the compressed bytes; MD5 lives in STREAMINFO
    ts = [threading.Thread(target=work, args=(k,)) for k in range(workers)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    return out


def cpu_baseline(streams, seconds: float):
    """The oracle (C restatement of zflac decode, ReleaseFast-like build) on host cores,
    independent streams in parallel; bounded sample."""
    import oracle

    oracle.decode_count_only(streams[0])  # load
    threads = min(16, os.cpu_count() or 1)
    counts = [0] * threads
    stop = time.perf_counter() + seconds
    t0 = time.perf_counter()

    def work(k):
        i = k
        n = 0
        while time.perf_counter() < stop:
            err, ns = oracle.decode_count_only(streams[i % len(streams)])
            assert err == 0
            n += ns
            i += threads
        counts[k] = n
    ts = [threading.Thread(target=work, args=(k,)) for k in range(threads)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    dt = time.perf_counter() - t0
    total = sum(counts)
    return {"value": total / dt / 1e6, "unit": "Msamples/s", "cores": threads, "kind": "port",
            "sample": f"oracle/zflac_oracle.c (-O3 -march=x86-64-v4, Debug checks off) decoding C5 shard streams "
                      f"round-robin on {threads} threads for {dt:.1f} s ({total / 1e6:.0f} M samples, MD5 incl.)"}


def verify(batch, streams, n_check_oracle=4):
    """Bit-exactness gate: every stream's PCM must hash to its STREAMINFO MD5 (checked
    inside read), and a sample must equal the oracle."""
    import oracle

    errs = []
    lock = threading.Lock()
    workers = min(16, os.cpu_count() or 1)

    def work(k):
        for i in range(k, len(streams), workers):
            try:
                batch.read(i, verify_md5=True)
            except Exception as e:  # noqa: BLE001
                with lock:
                    errs.append((i, repr(e)))
    ts = [threading.Thread(target=work, args=(k,)) for k in range(workers)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    for i in range(0, len(streams), max(1, len(streams) // n_check_oracle)):
        d = batch.read(i, verify_md5=False)
        if not np.array_equal(d.samples.values, oracle.decode(streams[i], "fast").samples):
            errs.append((i, "differs from oracle"))
    return errs


def main():
    args = parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as tdist

        torch.cuda.set_device(local_rank)
        tdist.init_process_group("nccl")
        dist = tdist

    import zflac_amd

    t_gen = time.perf_counter()
    streams = make_shard(rank, world, args.streams_per_gpu)
    t_gen = time.perf_counter() - t_gen
    batch = zflac_amd.Batch(streams, device=local_rank, timing=True)

    def barrier_sync():
        if dist is not None:
            import torch

            dist.barrier()
            torch.cuda.synchronize()

    for _ in range(args.warmup):
        batch.run()
    barrier_sync()
    t0 = time.perf_counter()
    dec_ms = []
    walk_ms = []
    scan_ms = []
    ver_ms = []
    for _ in range(args.steps):
        batch.run()
        t = batch.timings()
        dec_ms.append(t.decode_ms)
        walk_ms.append(t.walk_ms)
        scan_ms.append(t.scan_ms)
        ver_ms.append(t.verify_ms)
    barrier_sync()
    elapsed = time.perf_counter() - t0
    tm = batch.timings()
    samples_rank = tm.samples
    in_bytes, out_bytes = tm.input_bytes, tm.output_bytes

    errs = [] if args.no_verify else verify(batch, streams)
    from zflac_amd.shard import aggregate

    tot = aggregate(dist, "cuda" if dist is not None else None, elapsed, samples_rank, in_bytes, out_bytes, len(errs))
    elapsed = tot.elapsed_s
    samples_all, in_all, out_all = tot.samples, tot.input_bytes, tot.output_bytes
    ok = tot.errors == 0

    # decode() also checks the STREAMINFO MD5 (src/zflac.zig:267-280): the same shard with
    # the batched device MD5 (k_md5) after each decode, reported beside the headline
    md5 = None
    if not args.no_md5:
        batch.close()
        mb = zflac_amd.Batch(streams, device=local_rank, timing=True, device_md5=True)
        md5_ms, tot_ms = [], []
        for k in range(3):
            mb.run()
            if k:
                md5_ms.append(mb.timings().md5_ms)
                tot_ms.append(mb.timings().total_ms)
        md5_ok = all(mb.info(i)[0] == 0 and mb.md5(i) is not None for i in range(len(streams)))
        mb.close()
        m_avg = float(np.mean(md5_ms))
        md5 = {"kernel": "k_md5", "md5_ms": round(m_avg, 4), "all_match": md5_ok,
               "decode_plus_md5_msps_rank0": round(samples_rank / ((elapsed / args.steps) + m_avg * 1e-3) / 1e6, 1),
               "hashed_bytes_rank0": int(out_bytes),
               "note": "one lane per stream (MD5 is a serial chain per stream); not in `value`"}
        ok = ok and md5_ok
        batch = None

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(streams, args.cpu_seconds)

    if rank == 0:
        ms_step = elapsed / args.steps * 1e3
        value = samples_all * args.steps / elapsed / 1e6
        dec_avg = float(np.mean(dec_ms))
        alg_bytes = in_bytes + out_bytes  # per decode launch (this rank)
        achieved = alg_bytes / (dec_avg * 1e-3) / 1e9
        pmc = pmc_traffic("zflac::k_decode<1, 2>")
        traffic = pmc["bytes"] if pmc else None
        line = {
            "metric": "Msamples/s decoded (bit-exact) + achieved HBM GB/s, 4096-blk stereo",
            "value": round(value, 1),
            "unit": "Msamples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int32",
            "data": "synthetic (seeded flacgen streams, per-stream seeds)",
            "config": {"workload": "C5 shard: %d stereo 16-bit mid/side FLAC streams/GPU x %d frames x %d samples,"
                                   " LPC order 8, partition order 4" % (args.streams_per_gpu, FRAMES_PER_STREAM,
                                                                       BLOCK),
                       "streams_total": args.streams_per_gpu * world, "parallelism": f"stream-shard x{world}"},
            "hbm_gbs_step": round((in_all + out_all) * args.steps / elapsed / 1e9, 1),
            "bit_exact": ok,
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                         "kernel": "k_decode<1, 2>", "kernel_ms": round(dec_avg, 4),
                         "alg_bytes_per_launch": int(alg_bytes)},
            "stages_ms": {"scan+compact": round(float(np.mean(scan_ms)), 4),
                          "walk": round(float(np.mean(walk_ms)), 4), "decode": round(dec_avg, 4),
                          "verify": round(float(np.mean(ver_ms)), 4)},
            "traffic_detail": pmc,
            "device_md5": md5,
            "cpu_baseline": cpu,
            "gen_seconds": round(t_gen, 2),
        }
        if cpu:
            line["gpu_over_cpu"] = round(value / cpu["value"], 1)
        print(json.dumps(line), flush=True)
        if errs:
            print("BIT-EXACTNESS FAILURES:", errs[:10], file=sys.stderr)
    if batch is not None:
        batch.close()
    if dist is not None:
        dist.destroy_process_group()
    if not ok:
        sys.exit(1)


if __name__ == "__main__":
    main()
