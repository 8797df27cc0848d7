"""Benchmark: device-resident FLAC decode of the C5 per-GPU shard, plus the drop-in
decode() measured end to end.

Workload (BASELINE.json configs[4], per-GPU share; its codec parameters are configs[2]):
1250 independent stereo 16-bit mid/side streams per GPU, 32 frames x 4096 samples each,
LPC order 8 (synthetic, seeded per global stream index). One "step" = one batch run
(zflac_hip_batch_submit + _wait) over the rank's whole shard: frame-sync scan, candidate
compaction, subframe decode (Rice, LPC rollback, decorrelation, PCM pack-out) and chain
verification, inputs already in HBM, outputs left in HBM. Four runs are kept in flight
(--inflight 4, each with its own buffers; bench.py sets ZFLAC_RUN_STREAMS to --inflight so
each run has a run stream of its own), so one run's scan and walk overlap another's decode;
`ms_per_step_serial` is the same shard one run at a time; that serial leg runs before the
warm-up and the timed steps (the device ramps its clock up from idle over ~10-20 ms of load;
`pre_timed_runs` in the JSON line) and gives the isolated kernel times from its second half.
N GPUs = N ranks with disjoint shards (weak
scaling, no collective in the data path; torch.distributed only for the timing barrier
and the max over ranks).

`python bench.py --gpus N` with N > 1 and no WORLD_SIZE in the environment launches the N
ranks itself (one child process per GPU, RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set
before any HIP call); under torchrun WORLD_SIZE must equal --gpus. `--dry-run` runs the
launcher, sharding and aggregation on CPU over gloo without touching a GPU (tests).

Bit-exactness gate: every stream of every in-flight batch is compared with the oracle's
decode of it, and every stream's PCM hashes to its STREAMINFO MD5.

Beside the headline: decode + STREAMINFO MD5 as zflac's decode() does it (the device MD5
pipelined behind each run, several batches in flight), and (rank 0, N = 1 only) the CPU oracle on
the host's cores (decode alone, and decode + MD5 as zflac's decode() does, all cores and
one thread) and the drop-in decode() end to end (host bytes -> samples in host memory,
STREAMINFO MD5 verified) on long single streams, with its breakdown.

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import socket
import subprocess
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
METRIC = "Msamples/s decoded (bit-exact) + achieved HBM GB/s, 4096-blk stereo"
# PMC summary of the current k_decode build (tools/gpu.sh pmc; FETCH_SIZE /
# WRITE_SIZE corrected by the factors tools/calib_pmc.hip measures for this access pattern)
PMC_SUMMARY = os.path.join(ROOT, "profiles", "pmc_current.json")


def pmc_traffic(prefix: str, lib_sha: str | None, src_sha: str | None = None):
    """Corrected HBM bytes per step of the kernels named `prefix`* (the per-order-bucket
    k_decode launches, timed together) from the committed PMC summary, or None; `bytes` only
    when the summary was taken on the library build being timed: the same .so (sha256), or a
    build of the same sources, flags and defines (the fingerprint each build embeds, read from
    the library this process loaded: zflac_hip_build_id; hipcc output is not bit-reproducible,
    so a rebuild of unchanged sources has another .so hash)."""
    try:
        with open(PMC_SUMMARY) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    rows = [r for k, r in d.get("kernels", {}).items() if k.startswith(prefix) and "hbm_traffic_bytes" in r]
    if not rows:
        return None
    rd = sum(r["hbm_read_bytes"] for r in rows)
    wr = sum(r["hbm_write_bytes"] for r in rows)
    same_lib = lib_sha is not None and d.get("lib_sha256") == lib_sha
    same_src = src_sha is not None and d.get("src_sha256") == src_sha
    same = same_lib or same_src
    return {"bytes": int(rd + wr) if same else None, "read": int(rd), "write": int(wr), "kernels": len(rows),
            "same_build": same, "match": "lib" if same_lib else ("sources" if same_src else None),
            "lib_sha256": d.get("lib_sha256"), "src_sha256": d.get("src_sha256"),
            "source": os.path.relpath(d.get("_source", PMC_SUMMARY), ROOT)}


def progress(msg: str) -> None:
    """One line per phase on stderr (long runs keep writing, so a watchdog sees progress)."""
    print(f"bench [{time.strftime('%H:%M:%S')}] rank {os.environ.get('RANK', '0')}: {msg}", file=sys.stderr, flush=True)


def parse_args():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None, help="ranks (one per GPU); default WORLD_SIZE or 1")
    ap.add_argument("--steps", type=int, default=100,
                    help="timed steps; 100 by default so that the four-run pipeline's fill and drain "
                         "(about one step) are amortized (20 steps: ~4 %% lower, profiles/r5_steps_sweep.json)")
    ap.add_argument("--inflight", type=int, default=4,
                    help="shard runs overlapped on the device (1 = serial), on as many run streams")
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--streams-per-gpu", type=int, default=STREAMS_PER_GPU)
    ap.add_argument("--cpu-seconds", type=float, default=8.0, help="CPU baseline sample budget (all cores)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--no-md5", action="store_true", help="skip the device-MD5 leg")
    ap.add_argument("--md5-inflight", type=int, default=24, help="batches in flight in the decode+MD5 leg")
    ap.add_argument("--md5-steps", type=int, default=384,
                    help="timed runs of the decode+MD5 leg (its last hashes, ~8 ms each, end the timed region: "
                         "at 384 runs, ~280 ms, fill and drain are under 5 %%; 96 runs read 5-10 %% lower, "
                         "profiles/r5_md5_steps_sweep.json)")
    ap.add_argument("--md5-run-streams", type=int, default=5,
                    help="decode+MD5 leg: the library's run streams (ZFLAC_RUN_STREAMS)")
    ap.add_argument("--md5-hub-streams", type=int, default=3,
                    help="decode+MD5 leg: md5 hub streams (ZFLAC_HUB_STREAMS), each launch hashing --md5-runs runs")
    ap.add_argument("--md5-runs", type=int, default=8, help="decode+MD5 leg: runs per md5 hub launch (ZFLAC_MD5_RUNS)")
    # (64 of 256 CUs with three hub streams: 467-474k vs 435-463k shared, two same-box sweeps,
    # profiles/r6_md5_hub_cus.json)
    ap.add_argument("--md5-hub-cus", type=int, default=64,
                    help="decode+MD5 leg: CUs of the md5 hub's own (ZFLAC_HUB_CUS; 0 = hub and runs share every CU)")
    ap.add_argument("--md5-hw-queues", type=int, default=None,
                    help="GPU_MAX_HW_QUEUES of the decode+MD5 leg's process (default: run + hub streams)")
    ap.add_argument("--timed-events", choices=["on", "off"], default="off",
                    help="HIP timing events (5 per run) in the timed steps too (on: stages_ms_overlapped); "
                         "the serial leg always records them. Off by default since round 6: same box, "
                         "alternating, 700-710k vs 673-695k Msamples/s with them on (profiles/r6_events_ab.json)")
    ap.add_argument("--sched", choices=["rr", "ready"], default="rr",
                    help="headline runs in flight: round robin, or whichever batch finished first")
    ap.add_argument("--md5-leg-child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--md5-only", action="store_true",
                    help="only the decode+MD5 leg, in this process (kernel traces: set GPU_MAX_HW_QUEUES outside)")
    ap.add_argument("--no-e2e", action="store_true", help="skip the single-stream decode() legs")
    ap.add_argument("--e2e-frames", type=int, default=65536, help="frames of the long single stream")
    ap.add_argument("--backend", choices=["nccl", "gloo"], default=None)
    ap.add_argument("--same-device", action="store_true", help="every rank on GPU 0 (multi-process test)")
    ap.add_argument("--dry-run", action="store_true", help="CPU only: launcher, shards, aggregation")
    return ap.parse_args()


# ------------------------------------------------------------------------ launcher
def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch(n: int) -> int:
    """Spawn n ranks of this script (the parent never touches a GPU) and wait for them."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rcs = [p.wait() for p in procs]
    return next((rc for rc in rcs if rc), 0)


# ------------------------------------------------------------------------ workload
def make_shard(rank: int, world: int, n_streams: int):
    import synth
    from zflac_amd.shard import shard_range

    cfgs = [synth.config_c5(g, n_frames=FRAMES_PER_STREAM) for g in shard_range(rank, world, n_streams)]
    out = [None] * n_streams
    workers = host_threads(world)

    def work(k):
        for i in range(k, n_streams, workers):
            out[i] = synth.generate(**cfgs[i]).flac  # MD5 lives in STREAMINFO
    ts = [threading.Thread(target=work, args=(k,)) for k in range(workers)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    return out


def host_cores() -> tuple[int, str]:
    """CPUs this job may use: the affinity set, capped by a cgroup CPU quota if any."""
    n = len(os.sched_getaffinity(0))
    note = f"sched_getaffinity {n}"
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) // int(p)))
            note += f", cgroup quota {quota}"
            n = min(n, quota)
    except (OSError, ValueError):
        pass
    return n, note


def host_threads(world: int) -> int:
    """Host threads per rank for generation and verification: the job's cores split over the
    ranks of this node (8 ranks on a 16-core allowance would otherwise run 128 threads)."""
    return max(1, min(16, host_cores()[0] // max(1, world)))


def _oracle_rate(streams, seconds: float, threads: int, md5: bool):
    import oracle

    counts = [0] * threads
    stop = time.perf_counter() + seconds
    t0 = time.perf_counter()

    def work(k):
        i, n = k, 0
        while time.perf_counter() < stop:
            err, ns = oracle.decode_count_only(streams[i % len(streams)], "fast", md5=md5)
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
    return sum(counts) / dt / 1e6, sum(counts), dt


def cpu_baseline(streams, seconds: float):
    """The oracle (C restatement of zflac decode, ReleaseFast-like build) on the host:
    bounded samples of the shard's streams. `value` is the decode alone on every core
    (like-for-like with the device headline, which excludes MD5); decode + MD5 (what
    zflac's decode() does) on every core and on one thread are reported beside it."""
    import oracle

    oracle.decode_count_only(streams[0])  # load
    cores, note = host_cores()
    v_dec, n_dec, t_dec = _oracle_rate(streams, seconds, cores, md5=False)
    v_md5, _, _ = _oracle_rate(streams, seconds / 2, cores, md5=True)
    v_1t, _, _ = _oracle_rate(streams[:1], 3.0, 1, md5=True)
    v_1t_dec, _, _ = _oracle_rate(streams[:1], 2.0, 1, md5=False)
    return {"value": round(v_dec, 1), "unit": "Msamples/s", "cores": cores, "kind": "port",
            "sample": f"oracle/zflac_oracle.c (-O3 -march=x86-64-v4, Debug checks off), decode only (MD5 "
                      f"skipped), C5 shard streams round-robin on {cores} threads ({note}) for {t_dec:.1f} s "
                      f"({n_dec / 1e6:.0f} M samples)",
            "value_with_md5": round(v_md5, 1), "value_1thread_with_md5": round(v_1t, 1),
            "value_1thread": round(v_1t_dec, 1)}


def verify(batches, streams):
    """Bit-exactness gate: every stream of every batch must hash to its STREAMINFO MD5
    (checked inside read) and equal the oracle's decode of the same bytes (the oracle runs
    once per stream, on the host's cores). Returns (failures, streams compared)."""
    import oracle

    errs = []
    lock = threading.Lock()
    workers = host_threads(int(os.environ.get("WORLD_SIZE", "1")))
    compared = [0] * workers

    def work(k):
        for i in range(k, len(streams), workers):
            ref = oracle.decode(streams[i], "fast")
            for bi, b in enumerate(batches):
                try:
                    d = b.read(i, verify_md5=True)
                    ok = ref.error == "OK" and np.array_equal(d.samples.values, ref.samples)
                    if not ok:
                        with lock:
                            errs.append((bi, i, "differs from oracle"))
                except Exception as e:  # noqa: BLE001
                    with lock:
                        errs.append((bi, i, repr(e)))
            compared[k] += 1
    ts = [threading.Thread(target=work, args=(k,)) for k in range(workers)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    return errs, sum(compared)


def e2e_leg(name: str, cfg: dict, seg_frames: int, frames: int, oracle_full: bool):
    """decode() end to end on one stream: zflac_hip_open (plan, H2D, device decode) +
    zflac_hip_read (D2H overlapped with the host STREAMINFO MD5), best of 2, with the
    oracle's one-thread decode() of the same stream beside it."""
    import oracle
    import synth
    import zflac_amd

    st = synth.generate(**dict(cfg, n_samples=BLOCK * seg_frames))
    reps = max(1, frames // seg_frames)
    data = synth.tile_flac(st, reps) if reps > 1 else st.flac
    n = st.pcm.size * reps
    best = None
    for _ in range(2):
        tm = {}
        t0 = time.perf_counter()
        d = zflac_amd.decode(data, timings=tm)  # raises InvalidChecksum unless bit-exact
        wall = time.perf_counter() - t0
        assert d.samples.values.size == n
        if best is None or wall < best[0]:
            best = (wall, tm)
        del d
    wall, tm = best
    if oracle_full:
        t0 = time.perf_counter()
        err, ns = oracle.decode_count_only(data, "fast")
        cpu_s = time.perf_counter() - t0
        cpu_note = "whole stream"
    else:  # bounded: the repeated segment, scaled (same frames, same work per frame)
        t0 = time.perf_counter()
        err, ns = oracle.decode_count_only(st.flac, "fast")
        cpu_s = (time.perf_counter() - t0) * reps
        cpu_note = f"one {seg_frames}-frame segment x {reps}"
    assert err == 0
    out_bytes = n * (2 if cfg["bps"] <= 16 else 4)
    return {"stream": name, "frames": seg_frames * reps, "channel_samples": int(n), "input_bytes": len(data),
            "output_bytes": int(out_bytes), "wall_ms": round(wall * 1e3, 1),
            "msps": round(n / wall / 1e6, 1),
            "breakdown_ms": {"plan": round(tm["plan_ms"], 2), "upload_h2d": round(tm["upload_ms"], 2),
                             "device_run": round(tm["run_wall_ms"], 2), "kernels": round(tm["total_ms"], 3),
                             "read_d2h_with_md5": round(tm["read_ms"], 2), "host_md5": round(tm["host_md5_ms"], 2)},
            "oracle_1thread_ms": round(cpu_s * 1e3, 1), "oracle_1thread_msps": round(n / cpu_s / 1e6, 1),
            "oracle_sample": cpu_note, "speedup_vs_oracle_1thread": round(cpu_s / wall, 2),
            "md5_bound_msps": round(n / (tm["host_md5_ms"] * 1e-3) / 1e6, 1) if tm["host_md5_ms"] else None}


def run_ready_order(batches, k: int, on_done=None) -> None:
    """k runs over `batches`, one run in flight per batch: every batch is submitted, then
    whichever batch's run has finished (zflac_hip_batch_ready) is collected and resubmitted
    until k runs have been submitted, then the rest drain. Round robin instead waits for the
    oldest run while younger ones may already be done (head-of-line blocking: with the
    decode+MD5 leg's ~9 ms hashes, a slow batch idled the others)."""
    pending = [False] * len(batches)
    submitted = 0
    for j, b in enumerate(batches):
        if submitted == k:
            break
        b.submit()
        pending[j] = True
        submitted += 1
    while any(pending):
        for j, b in enumerate(batches):
            if pending[j] and b.ready():
                b.wait()
                pending[j] = False
                if on_done is not None:
                    on_done(j)
                if submitted < k:
                    b.submit()
                    pending[j] = True
                    submitted += 1


def md5_leg(args, streams, device: int, barrier=lambda: None):
    """decode + STREAMINFO MD5 of every stream of the shard: batches created with
    ZFLAC_FLAG_DEVICE_MD5; each run's certified streams go to the device's md5 hub, which
    hashes several runs per k_md5_coop launch on streams of its own (a serial chain per
    stream, ~7-9 ms for this shard) while other batches' runs decode on the run streams.
    `md5_inflight` batches in completion order (run_ready_order), `md5_steps` timed runs."""
    for k, v in (("ZFLAC_RUN_STREAMS", args.md5_run_streams), ("ZFLAC_HUB_STREAMS", args.md5_hub_streams),
                 ("ZFLAC_MD5_RUNS", args.md5_runs), ("ZFLAC_HUB_CUS", args.md5_hub_cus)):
        os.environ.setdefault(k, str(v))  # read by the library when it creates the device's streams
    import zflac_amd

    n_steps = args.md5_steps
    k_md5 = max(1, min(args.md5_inflight, n_steps))
    mbs = [zflac_amd.Batch(streams, device=device, timing=True, device_md5=True) for _ in range(k_md5)]
    rec = []

    def steps(k):
        run_ready_order(mbs, k, lambda j: rec.append(mbs[j].timings().md5_ms))

    steps(max(args.warmup, k_md5))
    rec.clear()
    barrier()
    t1 = time.perf_counter()
    steps(n_steps)
    barrier()
    el = time.perf_counter() - t1
    samples = mbs[0].timings().samples
    out_bytes = mbs[0].timings().output_bytes
    ok = all(mb.info(i)[0] == 0 and mb.md5(i) == s[26:42] for mb in mbs for i, s in enumerate(streams))
    for mb in mbs:
        mb.close()
    return {"kernel": "k_md5_coop", "md5_ms": round(float(np.mean(rec)), 4), "all_match": ok, "inflight": k_md5,
            "steps": n_steps, "gpu_max_hw_queues": os.environ.get("GPU_MAX_HW_QUEUES"),
            "run_streams": os.environ.get("ZFLAC_RUN_STREAMS"), "hub_streams": os.environ.get("ZFLAC_HUB_STREAMS"),
            "runs_per_hub_launch": os.environ.get("ZFLAC_MD5_RUNS"), "hub_cus": os.environ.get("ZFLAC_HUB_CUS"),
            "decode_plus_md5_msps_rank0": round(samples * n_steps / el / 1e6, 1),
            "ms_per_step": round(el / n_steps * 1e3, 4),
            "hashed_bytes_rank0": int(out_bytes),
            "note": "decode + STREAMINFO MD5 of every stream (one lane per stream, the wave's loads through LDS); "
                    "md5_ms = one md5 hub launch (several runs) while overlapped; not in `value`"}


def start_md5_child(args):
    """Start the process that will run md5_leg (same rank, same shard) with GPU_MAX_HW_QUEUES
    set, so the headline's process keeps the runtime's defaults. Started before this process
    touches the GPU (no fork / exec from a process with a GPU context). It does not generate
    anything: it blocks on its stdin until md5_leg_in_child sends it this rank's shard. Started
    by rank 0 only: world + 1 processes in all, each with host_threads(world) host threads."""
    cmd = [sys.executable, os.path.abspath(__file__), "--md5-leg-child", "--steps", str(args.steps), "--warmup",
           str(args.warmup), "--streams-per-gpu", str(args.streams_per_gpu), "--md5-inflight", str(args.md5_inflight),
           "--md5-steps", str(args.md5_steps), "--md5-run-streams", str(args.md5_run_streams),
           "--md5-hub-streams", str(args.md5_hub_streams), "--md5-runs", str(args.md5_runs),
           "--md5-hub-cus", str(args.md5_hub_cus)]
    if args.same_device:
        cmd.append("--same-device")
    if args.dry_run:
        cmd.append("--dry-run")
    q = args.md5_hw_queues or args.md5_run_streams + args.md5_hub_streams  # one hardware queue per stream
    env = dict(os.environ, GPU_MAX_HW_QUEUES=str(q), ZFLAC_RUN_STREAMS=str(args.md5_run_streams),
               ZFLAC_HUB_STREAMS=str(args.md5_hub_streams), ZFLAC_MD5_RUNS=str(args.md5_runs),
               ZFLAC_HUB_CUS=str(args.md5_hub_cus))
    return subprocess.Popen(cmd, env=env, stdin=subprocess.PIPE, stdout=subprocess.PIPE)


def write_shard(f, streams) -> None:
    """The shard as bytes: stream count, each length (u64 little-endian), then the streams."""
    f.write(np.array([len(streams)] + [len(s) for s in streams], dtype="<u8").tobytes())
    for s in streams:
        f.write(s)
    f.flush()


def read_shard(f):
    n = int(np.frombuffer(f.read(8), dtype="<u8")[0])
    lens = np.frombuffer(f.read(8 * n), dtype="<u8") if n else []
    return [f.read(int(x)) for x in lens]


def md5_leg_in_child(proc, streams):
    """Send the child started by start_md5_child this rank's shard and let it run its leg;
    returns its dict (None on failure)."""
    try:
        write_shard(proc.stdin, streams)
        proc.stdin.close()
    except (BrokenPipeError, OSError):
        pass
    out = proc.stdout.read().decode()
    proc.wait()
    if proc.returncode != 0 or not out.strip():
        return None
    return json.loads(out.strip().splitlines()[-1])


# ------------------------------------------------------------------------ main
def main():
    args = parse_args()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus and args.gpus > 1:
        sys.exit(launch(args.gpus))
    world = int(env_world or 1)
    if args.md5_leg_child:  # the decode+MD5 leg of this rank, in its own process (start_md5_child)
        device = 0 if args.same_device else int(os.environ.get("LOCAL_RANK", "0"))
        streams = read_shard(sys.stdin.buffer)  # the parent's shard, not a regenerated one
        if args.dry_run:
            print(json.dumps({"dry_run": True, "streams": len(streams), "pid": os.getpid(),
                              "digest": hashlib.sha256(b"".join(streams)).hexdigest()[:16]}), flush=True)
            return
        print(json.dumps(md5_leg(args, streams, device)), flush=True)
        return
    if args.md5_only:  # the decode+MD5 leg alone, in this process (tools/gpu.sh md5trace)
        rank = int(os.environ.get("RANK", "0"))
        device = 0 if args.same_device else int(os.environ.get("LOCAL_RANK", "0"))
        print(json.dumps(md5_leg(args, make_shard(rank, world, args.streams_per_gpu), device)), flush=True)
        return
    if args.gpus is not None and args.gpus != world:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    device = 0 if args.same_device else local_rank
    backend = args.backend or ("gloo" if (args.dry_run or args.same_device) else "nccl")
    # the decode+MD5 leg (reported for rank 0 only) runs on rank 0 alone: at world 8 that is 9
    # processes on the node instead of 16, the other ranks' GPUs idle meanwhile
    md5_proc = None if (args.no_md5 or rank != 0) else start_md5_child(args)
    # one run stream per run in flight (read by the library when it first uses the device;
    # the HIP default of four hardware queues covers four run streams)
    os.environ.setdefault("ZFLAC_RUN_STREAMS", str(max(1, args.inflight)))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as tdist

        if backend == "nccl":
            torch.cuda.set_device(device)
        tdist.init_process_group(backend, rank=rank, world_size=world)
        dist = tdist
    coll_dev = "cuda" if (dist is not None and backend == "nccl") else None

    def barrier_sync():
        if dist is not None:
            dist.barrier()
            if backend == "nccl":
                import torch

                torch.cuda.synchronize()

    from zflac_amd.shard import aggregate, shard_range

    t_gen = time.perf_counter()
    streams = make_shard(rank, world, args.streams_per_gpu)
    t_gen = time.perf_counter() - t_gen
    progress(f"shard of {len(streams)} streams generated in {t_gen:.1f} s")

    if args.dry_run:  # no GPU: the launch / shard / aggregation path only
        barrier_sync()
        t0 = time.perf_counter()
        samples = sum(int.from_bytes(s[21:26], "big") & ((1 << 36) - 1) for s in streams) * 2
        barrier_sync()
        el = time.perf_counter() - t0
        tot = aggregate(dist, coll_dev, el, samples, sum(len(s) for s in streams), samples * 2, 0)
        digest = hashlib.sha256(b"".join(streams)).hexdigest()[:16]
        child = md5_leg_in_child(md5_proc, streams) if md5_proc is not None else None
        # per rank: this process, its decode+MD5 child (rank 0 only), and the host threads it may use
        rng = shard_range(rank, world, args.streams_per_gpu)
        mine = {"rank": rank, "shard": [rng.start, rng.stop], "pid": os.getpid(), "processes": 1 + (child is not None),
                "host_threads": host_threads(world),
                "child_got_shard": bool(child and child["digest"] == digest and child["streams"] == len(streams))}
        ranks = [None] * world
        if dist is not None:
            dist.all_gather_object(ranks, mine)
        else:
            ranks = [mine]
        if rank == 0:
            print(json.dumps({"metric": METRIC, "dry_run": True, "n_gpus": world, "value": None,
                              "config": {"streams_total": args.streams_per_gpu * world,
                                         "parallelism": f"stream-shard x{world}"},
                              "shards": [r["shard"] for r in ranks], "ranks": ranks,
                              "processes_total": sum(r["processes"] for r in ranks),
                              "host_threads_total": sum(r["host_threads"] for r in ranks),
                              "host_cores": host_cores()[0],
                              "samples_total": tot.samples, "backend": backend, "digest_rank0": digest}), flush=True)
        if dist is not None:
            dist.destroy_process_group()
        return

    import zflac_amd

    # `inflight` runs of the shard overlap on the device: each has its own Batch (HIP stream,
    # input copy, candidate tables, output), and step k+1 is submitted before step k is
    # waited for, so one run's scan and walk execute beside the other's decode. Every step
    # still decodes and verifies the whole shard.
    n_inf = max(1, min(args.inflight, args.steps))  # every batch runs (and is verified)
    timed_ev = args.timed_events == "on" or n_inf == 1  # (one in flight: no serial leg, the timed runs give the times)
    batches = [zflac_amd.Batch(streams, device=device, timing=timed_ev) for _ in range(n_inf)]
    # the serial leg's batch always records its stage events (the isolated kernel times)
    serial_batch = batches[:1] if timed_ev else [zflac_amd.Batch(streams, device=device, timing=True)]
    STAGES = ("scan_ms", "walk_ms", "decode_ms", "verify_ms")

    def run_steps(k, bs, rec=None):
        """k runs over the batches `bs` round robin, len(bs) in flight; per-run HIP-event
        stage times appended to `rec`."""
        pending = [False] * len(bs)

        def done(j):
            bs[j].wait()
            if rec is not None:
                t = bs[j].timings()
                for name in STAGES:
                    rec[name].append(getattr(t, name))

        if args.sched == "ready":
            def rec_done(j):
                if rec is not None:
                    t = bs[j].timings()
                    for name in STAGES:
                        rec[name].append(getattr(t, name))
            run_ready_order(bs, k, rec_done)
            return
        for i in range(k):
            j = i % len(bs)
            if pending[j]:
                done(j)
            bs[j].submit()
            pending[j] = True
        for t in range(len(bs)):  # drain, oldest first
            j = (k + t) % len(bs)
            if pending[j]:
                done(j)

    # The serial leg first: the same shard one run at a time (no overlap), `steps` runs, for
    # the isolated kernel times the roofline uses and the serial step time. It runs before the
    # warm-up and the timed steps because the device leaves idle at a lower clock: after an
    # idle gap, the first ~10 ms of load run slower (tools/warm_test.py,
    # profiles/r5_warm_test.json: 20-step stretches at 0.53 ms/step right after 5 warm-up
    # runs, 0.47-0.49 once the device has been busy ~20 ms, 0.55-0.57 after a 50-500 ms
    # idle gap). The isolated times come from the leg's second half, where the clock has
    # settled (and `ms_per_step_serial` from the same half). The timed steps are unchanged:
    # `warmup` runs, a barrier, `steps` runs.
    serial = None
    rec = None
    if n_inf > 1:
        half = args.steps // 2
        run_steps(half, serial_batch)
        rec = {n: [] for n in STAGES}
        t1 = time.perf_counter()
        run_steps(args.steps - half, serial_batch, rec)
        serial = (time.perf_counter() - t1) / (args.steps - half)
    run_steps(args.warmup, batches)
    progress("warm-up done")
    barrier_sync()
    t0 = time.perf_counter()
    rec_ov = {n: [] for n in STAGES}
    run_steps(args.steps, batches, rec_ov if timed_ev else None)
    barrier_sync()
    elapsed = time.perf_counter() - t0
    tm = batches[0].timings() or serial_batch[0].timings()
    samples_rank = tm.samples
    in_bytes, out_bytes = tm.input_bytes, tm.output_bytes
    if rec is None:
        rec = rec_ov
    scan_ms, walk_ms, dec_ms, ver_ms = (rec[n] for n in STAGES)

    progress(f"timed steps done ({elapsed / args.steps * 1e3:.3f} ms/step)")
    errs = []
    n_compared = 0
    if not args.no_verify:
        errs, n_compared = verify(batches, streams)
    for b in batches[1:]:
        b.close()
    if serial_batch[0] is not batches[0]:
        serial_batch[0].close()
    batch = batches[0]
    tot = aggregate(dist, coll_dev, elapsed, samples_rank, in_bytes, out_bytes, len(errs))
    elapsed = tot.elapsed_s
    samples_all, in_all, out_all = tot.samples, tot.input_bytes, tot.output_bytes
    ok = tot.errors == 0

    # decode() also checks the STREAMINFO MD5 (src/zflac.zig:267-280): the same shard with
    # ZFLAC_FLAG_DEVICE_MD5, in a child process of its own whose GPU_MAX_HW_QUEUES covers
    # one hardware queue per batch in flight (md5_leg)
    md5 = None
    if md5_proc is not None:
        batch.close()
        batch = None
        progress("verification done; decode+MD5 leg")
        md5 = md5_leg_in_child(md5_proc, streams)
        ok = ok and bool(md5 and md5.get("all_match"))

    cpu = None
    e2e = None
    if rank == 0 and world == 1:
        if not args.no_cpu_baseline:
            progress("CPU baseline")
            cpu = cpu_baseline(streams, args.cpu_seconds)
        if not args.no_e2e:
            import synth

            progress("end-to-end decode() legs")
            e2e = [e2e_leg("C3 stereo M/S 16-bit LPC-8, 65536 frames (SURVEY 8d size)", synth.config_c3(),
                           1024, args.e2e_frames, oracle_full=False),
                   e2e_leg("C3, 2600 frames (a ~4-minute track)", synth.config_c3(), 2600, 2600, oracle_full=True)]

    if rank == 0:
        ms_step = elapsed / args.steps * 1e3
        value = samples_all * args.steps / elapsed / 1e6
        dec_avg = float(np.mean(dec_ms))
        alg_bytes = in_bytes + out_bytes  # per decode launch (this rank)
        achieved = alg_bytes / (dec_avg * 1e-3) / 1e9
        lib_sha = hashlib.sha256(open(zflac_amd.lib_path, "rb").read()).hexdigest()
        bid = zflac_amd.build_id()  # embedded by the build: the sources of the loaded library
        src_sha = bid[4:] if bid and bid.startswith("src=") else None
        pmc = pmc_traffic("zflac::k_decode<1, 2", lib_sha, src_sha)
        line = {
            "metric": METRIC,
            "value": round(value, 1),
            "unit": "Msamples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_step, 4),
            "inflight": n_inf,
            "ms_per_step_serial": round(serial * 1e3, 4) if serial else None,
            "pre_timed_runs": {"serial_leg": args.steps if serial else 0, "warmup": args.warmup,
                               "why": "the serial leg (one run at a time, isolated kernel times) runs before the "
                                      "warm-up: the device leaves idle at a lower clock (profiles/r5_warm_test.json)"},
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
            "oracle_compared": f"{n_compared}/{len(streams)} streams x {len(batches)} in-flight batches (rank 0)",
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": pmc["bytes"] if pmc else None,
                         "kernel": "k_decode<1, 2, *> (order-bucket launches, one event pair)", "kernel_ms": round(dec_avg, 4),
                         "kernel_timing": "isolated launches (serial leg, one run in flight)" if serial else "timed steps",
                         "alg_bytes_per_launch": int(alg_bytes)},
            "stages_ms": {"scan+compact": round(float(np.mean(scan_ms)), 4),
                          "walk": round(float(np.mean(walk_ms)), 4), "decode": round(dec_avg, 4),
                          "verify": round(float(np.mean(ver_ms)), 4)},
            "stages_ms_overlapped": {"scan+compact": round(float(np.mean(rec_ov["scan_ms"])), 4),
                                     "walk": round(float(np.mean(rec_ov["walk_ms"])), 4),
                                     "decode": round(float(np.mean(rec_ov["decode_ms"])), 4)}
            if serial and rec_ov["decode_ms"] else None,
            "traffic_detail": pmc,
            "lib_sha256": lib_sha[:16],
            "build_id": bid,
            "device_md5": md5,
            "cpu_baseline": cpu,
            "e2e_decode": e2e,
            "gen_seconds": round(t_gen, 2),
        }
        if cpu:
            line["gpu_over_cpu"] = round(value / cpu["value"], 1)  # decode alone on both sides
            if md5:
                line["gpu_over_cpu_with_md5"] = round(md5["decode_plus_md5_msps_rank0"] / cpu["value_with_md5"], 1)
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
