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
