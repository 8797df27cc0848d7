"""Multi-rank path on CPU: world_size 2 over gloo (127.0.0.1).

The GPU job shards independent streams across ranks (zflac_amd.shard) and only reduces the
timing and counters. Here each rank decodes its shard with the oracle, checks it against
the generator's PCM, and the aggregation must equal the single-process totals.
"""
from __future__ import annotations

import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from tests.util import expected_samples

WORLD = 2
PER_RANK = 3


def _cfg(g):
    import synth

    return synth.config_c5(g, n_frames=2)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank, world, port, out_q):
    import torch
    import torch.distributed as dist

    import oracle
    import synth
    from zflac_amd.shard import aggregate, shard_range

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        idx = list(shard_range(rank, world, PER_RANK))
        samples = in_bytes = out_bytes = errors = 0
        for g in idx:
            st = synth.generate(**_cfg(g))
            r = oracle.decode(st.flac, "checked")
            if r.error != "OK" or not np.array_equal(r.samples, expected_samples(st).ravel()):
                errors += 1
            samples += r.samples.size
            in_bytes += len(st.flac)
            out_bytes += r.samples.nbytes
        elapsed = 0.5 + rank  # distinct per rank: the job time is the max
        tot = aggregate(dist, None, elapsed, samples, in_bytes, out_bytes, errors)
        got = [None] * world
        dist.all_gather_object(got, idx)
        out_q.put((rank, tot, got, samples))
    finally:
        dist.destroy_process_group()


def test_shard_range_partitions_the_job():
    from zflac_amd.shard import shard_range

    seen = [g for r in range(4) for g in shard_range(r, 4, 5)]
    assert seen == list(range(20))
    with pytest.raises(ValueError):
        shard_range(4, 4, 5)


def test_gloo_world2_shards_and_aggregates():
    import oracle

    oracle.build()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, WORLD, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    codes = [p.exitcode for p in procs]
    for p in procs:
        if p.is_alive():
            p.kill()
    assert codes == [0] * WORLD, f"rank exit codes {codes}"
    res = [q.get(timeout=10) for _ in range(WORLD)]
    res.sort(key=lambda t: t[0])
    per_rank_samples = [r[3] for r in res]
    for rank, tot, gathered, _ in res:
        assert tot.errors == 0
        assert tot.elapsed_s == pytest.approx(0.5 + (WORLD - 1))
        assert tot.samples == sum(per_rank_samples)
        flat = [g for part in gathered for g in part]
        assert sorted(flat) == list(range(WORLD * PER_RANK)) and len(set(flat)) == len(flat)

    # single-process reference of the same job
    import synth

    total = 0
    for g in range(WORLD * PER_RANK):
        total += synth.generate(**_cfg(g)).pcm.size
    assert res[0][1].samples == total


def _bench(*extra, timeout=300):
    import json
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, os.path.join(root, "bench.py"), *extra], capture_output=True, text=True,
                       timeout=timeout, env=env, cwd=root)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout  # ONE JSON line, from rank 0
    return json.loads(lines[0])


def test_bench_self_launch_dry_run():
    """`bench.py --gpus 2` launches its two ranks itself (no torchrun): disjoint shards,
    job totals over both ranks, one JSON line. CPU only (gloo, no HIP call)."""
    d = _bench("--gpus", "2", "--dry-run", "--streams-per-gpu", "3", "--steps", "1", "--warmup", "0")
    assert d["dry_run"] and d["n_gpus"] == 2 and d["backend"] == "gloo"
    assert d["config"]["streams_total"] == 6
    assert d["shards"] == [[0, 3], [3, 6]]
    assert d["samples_total"] == 6 * 32 * 4096 * 2


def test_bench_self_launch_dry_run_world8():
    """The driver's 8-GPU shape, rehearsed on the CPU: `bench.py --gpus 8 --dry-run` starts 8
    ranks; rank 0 also starts its decode+MD5 child (the leg is reported for rank 0 only), which
    receives the rank's shard over a pipe (it does not regenerate it); host threads are the
    job's cores split over the ranks."""
    d = _bench("--gpus", "8", "--dry-run", "--streams-per-gpu", "2", "--steps", "1", "--warmup", "0", timeout=600)
    assert d["n_gpus"] == 8 and len(d["ranks"]) == 8
    assert d["shards"] == [[2 * r, 2 * r + 2] for r in range(8)]
    assert d["ranks"][0]["child_got_shard"] and d["ranks"][0]["processes"] == 2
    assert all(r["processes"] == 1 for r in d["ranks"][1:])
    assert d["processes_total"] == 9
    assert d["host_threads_total"] <= max(8, d["host_cores"])
    print("per-rank processes", [r["processes"] for r in d["ranks"]], "host threads",
          [r["host_threads"] for r in d["ranks"]], "cores", d["host_cores"])


def test_bench_world_mismatch_fails():
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--dry-run"],
                       capture_output=True, text=True, timeout=120, env=env, cwd=root)
    assert p.returncode != 0 and "WORLD_SIZE" in p.stderr


@pytest.mark.gpu
def test_bench_two_ranks_two_hip_contexts(gpu_ready):
    """Two ranks launched by bench.py itself, each with its own HIP context on GPU 0 (the
    only GPU of the test box), gloo for the barrier: shards decode bit-exactly and the
    job line covers both ranks."""
    d = _bench("--gpus", "2", "--same-device", "--streams-per-gpu", "16", "--steps", "2", "--warmup", "1",
               "--no-cpu-baseline", "--no-md5", "--no-e2e")
    assert d["n_gpus"] == 2 and d["bit_exact"] is True
    assert d["config"]["streams_total"] == 32 and d["value"] > 0
