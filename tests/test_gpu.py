"""GPU parity tests: the HIP decode path (through the C ABI) against the oracle, the
reference's golden vectors, the committed fixtures and the writer's ground truth.
Bar: bit-exact samples and identical zflac error names."""
import hashlib
import os

import numpy as np
import pytest

import oracle
import synth
import zflac_amd
from zflac_amd import errors

from . import malformed
from .util import GOLDEN, PARITY_CONFIGS, expected_samples, load_fixture_manifest, load_kats, splice_frames

pytestmark = pytest.mark.gpu


def _gpu(data):
    try:
        d = zflac_amd.decode(data)
        return "OK", d
    except errors.ZflacError as e:
        return type(e).__name__, None


def test_native_library_is_the_path(gpu_ready):
    assert os.path.exists(zflac_amd.lib_path)
    assert zflac_amd.device_count() >= 1


@pytest.mark.parametrize("kat", load_kats(), ids=lambda k: k["name"])
def test_kat_basic_zig_gpu(gpu_ready, kat):
    err, d = _gpu(bytes.fromhex(kat["flac_hex"]))
    assert err == "OK"
    assert d.channels == kat["channels"]
    assert getattr(d.samples, kat["sample_kind"]).tolist() == kat["expected"]


def test_golden_fixtures_gpu(gpu_ready):
    for fx in load_fixture_manifest()["fixtures"]:
        data = open(os.path.join(GOLDEN, fx["file"]), "rb").read()
        err, d = _gpu(data)
        assert err == fx["error"], fx["file"]
        assert hashlib.sha256(d.samples.values.tobytes()).hexdigest() == fx["samples_sha256"], fx["file"]


@pytest.mark.parametrize("name", sorted(PARITY_CONFIGS))
def test_parity_configs(gpu_ready, name):
    st = synth.generate(**PARITY_CONFIGS[name])
    r = oracle.decode(st.flac)
    assert r.error == "OK"
    err, d = _gpu(st.flac)
    assert err == "OK", name
    np.testing.assert_array_equal(d.samples.values, r.samples)
    np.testing.assert_array_equal(d.samples.values, expected_samples(st))
    assert (d.channels, d.sample_rate, d.bits_per_sample) == (r.channels, r.sample_rate, r.bits_per_sample)


_CASES = malformed.cases()


@pytest.mark.parametrize("case", sorted(_CASES))
def test_malformed_parity(gpu_ready, case):
    data, _ = _CASES[case]
    r = oracle.decode(data)
    err, d = _gpu(data)
    assert err == r.error, case
    if err == "OK":
        np.testing.assert_array_equal(d.samples.values, r.samples)


@pytest.mark.parametrize("name", ["c3_ms16_lpc8", "ch3_16", "variable_blocking", "mono8_lpc3",
                                  "c4_24bit_lpc32_wasted"])
def test_sequential_path_parity(gpu_ready, name):
    """The host-planned sequential chain (used when the parallel chain is not certified)."""
    st = synth.generate(**PARITY_CONFIGS[name])
    b = zflac_amd.Batch([st.flac], force_slow=True)
    b.run()
    d = b.read(0)
    b.close()
    np.testing.assert_array_equal(d.samples.values, expected_samples(st))


def test_mixed_batch(gpu_ready):
    """One batch, several stream classes (container, channel count) and malformed members."""
    names = sorted(PARITY_CONFIGS)
    streams = [synth.generate(**dict(PARITY_CONFIGS[n], seed=1000 + i)) for i, n in enumerate(names)]
    bad = [_CASES[c][0] for c in ("bad_sync_frame2", "wrong_md5", "residual_method_2", "bad_crc8_frame1")]
    datas = [s.flac for s in streams] + bad
    b = zflac_amd.Batch(datas)
    b.run()
    for i, data in enumerate(datas):
        r = oracle.decode(data)
        try:
            d = b.read(i)
            err = "OK"
        except errors.ZflacError as e:
            err, d = type(e).__name__, None
        assert err == r.error, i
        if d is not None:
            np.testing.assert_array_equal(d.samples.values, r.samples)
    b.close()


def _md5_pre_justify(v: np.ndarray, bps: int) -> bytes:
    """hashlib MD5 of the samples as zflac hashes them (src/zflac.zig:267-277)."""
    js = 16 - bps if 9 <= bps <= 15 else 32 - bps if 17 <= bps <= 31 else 0
    x = v >> js
    if v.dtype == np.int32 and (bps + 7) // 8 == 3:
        b = x.astype("<i4").view(np.uint8).reshape(-1, 4)[:, :3]
        return hashlib.md5(np.ascontiguousarray(b).tobytes()).digest()
    return hashlib.md5(x.astype(v.dtype.newbyteorder("<")).tobytes()).digest()


def _streaminfo_md5(flac: bytes) -> bytes:
    return flac[26:42]  # 'fLaC', block header, then STREAMINFO bytes 18..33


def test_device_md5_every_class(gpu_ready):
    """k_md5 (ZFLAC_FLAG_DEVICE_MD5): every container/depth class (8..32-bit, justify
    undone, 24-bit as 3 bytes), ragged lengths and unaligned stream bases in one batch;
    digests equal hashlib over the oracle's pre-justify bytes and the STREAMINFO MD5;
    a corrupted MD5 turns into InvalidChecksum."""
    names = sorted(PARITY_CONFIGS)
    streams = [synth.generate(**dict(PARITY_CONFIGS[n], seed=2000 + i)) for i, n in enumerate(names)]
    datas = [s.flac for s in streams] + [_CASES["wrong_md5"][0]]
    b = zflac_amd.Batch(datas, device_md5=True, timing=True)
    b.run()
    for i, data in enumerate(datas):
        r = oracle.decode(data)
        rc, _ = b.info(i)
        assert errors.NAMES.get(rc) == r.error, (i, rc, r.error)
        if r.error != "OK":
            continue
        dig = b.md5(i)
        assert dig is not None, i
        assert dig == _streaminfo_md5(data), i
        assert dig == _md5_pre_justify(r.samples, r.bits_per_sample), i
        d = b.read(i)  # device verdict stands in for the host hash
        np.testing.assert_array_equal(d.samples.values, r.samples)
    assert b.timings().md5_ms > 0
    b.close()


@pytest.mark.parametrize("loads", ["coop", "lane"])
@pytest.mark.parametrize("name", ["mono8_lpc3", "c3_ms16_lpc8", "stereo12_ms", "ms20_lpc16_escape",
                                  "c4_24bit_lpc32_wasted", "stereo32", "stereo31_ls_loud"])
def test_device_md5_cooperative_loads(gpu_ready, name, loads):
    """One class per batch (every job in one mode: k_md5_coop, the wave's 64 streams read
    through LDS; ZFLAC_MD5_LANE_LOADS=1 forces k_md5). 70 streams (a second, partial wave
    whose idle lanes only help load) of ragged lengths (lanes leave the unit loop at
    different units); one stream's MD5 corrupted. Digests equal STREAMINFO and hashlib."""
    cfg = PARITY_CONFIGS[name]
    bs = cfg["block_size"]
    datas = [synth.generate(**dict(cfg, seed=4000 + i, n_samples=bs * (1 + (i * 7) % 5) + (i * 13) % 97)).flac
             for i in range(70)]
    bad = bytearray(datas[65])
    bad[30] ^= 0x01  # a STREAMINFO MD5 byte
    datas[65] = bytes(bad)
    if loads == "lane":
        os.environ["ZFLAC_MD5_LANE_LOADS"] = "1"
    try:
        b = zflac_amd.Batch(datas, device_md5=True, timing=True)
    finally:
        os.environ.pop("ZFLAC_MD5_LANE_LOADS", None)
    for _ in range(2):  # the second run reuses the batch (and the md5 hub)
        b.run()
        for i, data in enumerate(datas):
            rc, _ = b.info(i)
            if i == 65:
                assert errors.NAMES.get(rc) == "InvalidChecksum", rc
                continue
            assert rc == 0, (i, rc)
            assert b.md5(i) == _streaminfo_md5(data), i
    r = oracle.decode(datas[3])
    assert b.md5(3) == _md5_pre_justify(r.samples, r.bits_per_sample)
    b.close()


@pytest.mark.parametrize("nohub", [False, True])
def test_device_md5_hub_and_run_stream(gpu_ready, monkeypatch, nohub):
    """Eight batches in flight, collected in completion order: through the md5 hub (several
    runs per k_md5_coop launch, on hub streams), and with ZFLAC_MD5_NOHUB=1 (each run's hash
    on its run stream, right behind its decode). Every digest equals STREAMINFO's, on
    every run, and _ready turns 1 only once the hash has landed."""
    if nohub:
        monkeypatch.setenv("ZFLAC_MD5_NOHUB", "1")
    sts = [synth.generate(**synth.config_c3(n_frames=4, seed=9100 + k)) for k in range(20)]
    datas = [s.flac for s in sts]
    bs = [zflac_amd.Batch(datas, device_md5=True, timing=True) for _ in range(8)]
    for rnd in range(2):
        for b in bs:
            b.submit()
        pending = set(range(len(bs)))
        while pending:
            for j in list(pending):
                if bs[j].ready():
                    bs[j].wait()
                    pending.discard(j)
                    for i, d in enumerate(datas):
                        assert bs[j].info(i)[0] == 0, (rnd, j, i)
                        assert bs[j].md5(i) == _streaminfo_md5(d), (rnd, j, i)
    for b in bs:
        b.close()


@pytest.mark.parametrize("via_ready", [False, True])
def test_md5_hub_failed_launch_does_not_poison_next_run(gpu_ready, monkeypatch, via_ready):
    """A failed md5 hub launch (fault injected with ZFLAC_FAULT_HUB_FLUSH=1) fails that run
    with DeviceError, through _wait or through _ready; the batch's next run succeeds, with every
    digest equal to STREAMINFO's (round-5 advisor finding: the failure flag leaked into the next
    run, whose good results then read as DeviceError)."""
    sts = [synth.generate(**synth.config_c3(n_frames=4, seed=9300 + k)) for k in range(6)]
    datas = [s.flac for s in sts]
    b = zflac_amd.Batch(datas, device_md5=True)
    monkeypatch.setenv("ZFLAC_FAULT_HUB_FLUSH", "1")
    b.submit()
    if via_ready:
        import time

        t0 = time.time()
        with pytest.raises(errors.DeviceError):
            while not b.ready():  # ready() launches the pending hash itself: the flush fails there
                assert time.time() - t0 < 60
                time.sleep(0.001)
        with pytest.raises(errors.DeviceError):
            b.ready()  # still failed, never "finished"
    with pytest.raises(errors.DeviceError):
        b.wait()
    monkeypatch.delenv("ZFLAC_FAULT_HUB_FLUSH")
    for _ in range(2):
        b.run()
        for i, d in enumerate(datas):
            assert b.info(i)[0] == 0, i
            assert b.md5(i) == _streaminfo_md5(d), i
            np.testing.assert_array_equal(b.read(i).samples.values, expected_samples(sts[i]))
    b.close()


def test_device_md5_c5_shard(gpu_ready):
    """C5-shaped members (32 frames, 131072 samples/ch), device MD5 against STREAMINFO."""
    streams = synth.generate_many([synth.config_c5(i) for i in range(130)])
    b = zflac_amd.Batch([s.flac for s in streams], device_md5=True)
    b.run()
    for i, s in enumerate(streams):
        assert b.info(i)[0] == 0, i
        assert b.md5(i) == _streaminfo_md5(s.flac), i
    b.close()


def test_batch_rerun_is_stable(gpu_ready):
    streams = [synth.generate(**synth.config_c5(i, n_frames=8)).flac for i in range(40)]
    b = zflac_amd.Batch(streams, timing=True)
    outs = []
    for _ in range(3):
        b.run()
        outs.append([b.read(i).samples.values.copy() for i in range(len(streams))])
    for i in range(len(streams)):
        np.testing.assert_array_equal(outs[0][i], outs[1][i])
        np.testing.assert_array_equal(outs[0][i], outs[2][i])
    t = b.timings()
    assert t is not None and t.decode_ms > 0
    b.close()


def test_overlapped_batches_submit_wait(gpu_ready):
    """zflac_hip_batch_submit / _wait: three batches in flight at once on their own HIP
    streams (the bench's pipelined mode), a mixed-class batch and a flagged-stream batch
    among them; every result equals the oracle, and the usage errors hold (double submit,
    wait without submit, results between submit and wait, destroy while in flight)."""
    names = sorted(PARITY_CONFIGS)
    mixed = [synth.generate(**dict(PARITY_CONFIGS[n], seed=3000 + i)).flac for i, n in enumerate(names)]
    c5 = [s.flac for s in synth.generate_many([synth.config_c5(i) for i in range(64)])]
    bad = [_CASES[c][0] for c in ("bad_sync_frame2", "wrong_md5", "bad_crc8_frame1")] + c5[:3]
    groups = [c5, mixed, bad]
    bs = [zflac_amd.Batch(g, timing=True) for g in groups]
    for rnd in range(2):
        for b in bs:
            b.submit()
        with pytest.raises(errors.InvalidArgument):
            bs[0].submit()
        assert bs[1].info(0)[0] == errors.InvalidArgument.code
        for b in reversed(bs):
            b.wait()
        with pytest.raises(errors.InvalidArgument):
            bs[2].wait()
        for g, b in zip(groups, bs):
            for i in range(0, len(g), 7 if g is c5 else 1):
                r = oracle.decode(g[i], "fast")
                try:
                    d = b.read(i)
                    err = "OK"
                except errors.ZflacError as e:
                    err, d = type(e).__name__, None
                assert err == r.error, (rnd, i)
                if d is not None:
                    np.testing.assert_array_equal(d.samples.values, r.samples)
    bs[0].submit()
    for b in bs:
        b.close()  # the in-flight one waits for its kernels first


def test_batch_ready_completion_order(gpu_ready):
    """zflac_hip_batch_ready: InvalidArgument without a submitted run; after submit it turns
    true once the run's device work is done (then _wait only produces the results), so a
    caller can collect whichever of several batches finished first (bench.run_ready_order)."""
    import time

    c5 = [s.flac for s in synth.generate_many([synth.config_c5(i, n_frames=8) for i in range(40)])]
    bs = [zflac_amd.Batch(c5[k::2], device_md5=k == 1) for k in range(2)]
    with pytest.raises(errors.InvalidArgument):
        bs[0].ready()
    for rnd in range(3):
        for b in bs:
            b.submit()
        left = set(range(len(bs)))
        t0 = time.time()
        while left:
            for j in list(left):
                if bs[j].ready():
                    bs[j].wait()
                    left.discard(j)
            assert time.time() - t0 < 60
        for k, b in enumerate(bs):
            for i in range(0, len(b), 5):
                np.testing.assert_array_equal(b.read(i).samples.values, oracle.decode(c5[2 * i + k], "fast").samples)
    for b in bs:
        b.close()


def test_c5_shard_md5_property(gpu_ready):
    """Full-shape C5 members (32 frames each) at a reduced stream count: every stream's
    decoded PCM must hash to its STREAMINFO MD5 (checked inside read) and a sample of
    them must equal the oracle."""
    cfgs = [synth.config_c5(i) for i in range(96)]
    streams = synth.generate_many(cfgs)
    b = zflac_amd.Batch([s.flac for s in streams])
    b.run()
    for i, s in enumerate(streams):
        d = b.read(i, verify_md5=True)
        if i % 16 == 0:
            np.testing.assert_array_equal(d.samples.values, oracle.decode(s.flac, "fast").samples)
    b.close()


@pytest.mark.parametrize("cfg", [synth.config_c2(1024), synth.config_c3(1024), synth.config_c4(256)],
                         ids=["c2", "c3", "c4"])
def test_large_single_stream(gpu_ready, cfg):
    """Long single streams: frame-sync scan over ~MBs, MD5 of the whole output."""
    st = synth.generate(**cfg)
    err, d = _gpu(st.flac)  # decode() verifies the STREAMINFO MD5
    assert err == "OK"
    np.testing.assert_array_equal(d.samples.values, expected_samples(st))


def _spliced_order_change():
    """Frames 0-2 LPC order 8, frames 3-5 LPC order 32 (16-bit mid/side): the host predicts
    the order-8 bucket from the first frame, so the order-32 frame groups have no launch of
    their own in the first run and are decoded by the synchronous `rest` launch
    (enqueue_rest in host.cpp); the bucket then joins the batch's launch plan."""
    base = dict(channels=2, bps=16, stereo_mode=10, block_size=4096, n_samples=4096 * 6, partition_order=4)
    a = synth.generate(**dict(base, order=8, precision=12, seed=4100))
    b = synth.generate(**dict(base, order=32, precision=12, seed=4101))
    return splice_frames(a, b, 3)


def test_bucket_misprediction_still_decodes(gpu_ready):
    data = _spliced_order_change()
    r = oracle.decode(data)
    assert r.error == "OK"
    err, d = _gpu(data)
    assert err == "OK"
    np.testing.assert_array_equal(d.samples.values, r.samples)
    # a batch of many such streams: 6 x 70 frames, so several frame groups per bucket
    b = zflac_amd.Batch([data] * 70, timing=True)
    b.run()
    assert b.timings().rest_launches == 1  # the unpredicted order-32 groups
    for i in range(0, 70, 9):
        np.testing.assert_array_equal(b.read(i).samples.values, r.samples)
    b.run()  # learned: the order-32 bucket has its own launch now, no synchronous rest launch
    assert b.timings().rest_launches == 0
    for i in range(0, 70, 9):
        np.testing.assert_array_equal(b.read(i).samples.values, r.samples)
    b.close()


def _with_min_frame(flac: bytes, v: int) -> bytes:
    """STREAMINFO's minimum frame size (24 bits at block offset 4) set to `v` bytes."""
    d = bytearray(flac)
    assert d[:4] == b"fLaC" and (d[4] & 0x7F) == 0
    d[12:15] = v.to_bytes(3, "big")
    return bytes(d)


def test_unknown_total_certified_by_parallel_pass(gpu_ready):
    """STREAMINFO total 0 (unknown): zflac reads frames until fewer than 4 bytes are left
    (src/zflac.zig:343-350) and grows its buffer as it goes. The batch's creation scans the
    stream once and reserves the units its sync candidates claim; k_verify then certifies the
    chain to the end of the stream, so no stream goes to the sequential planner, whatever
    STREAMINFO's frame sizes say. 4 trailing bytes (a frame header zflac reads and rejects) and
    planted false syncs send the stream to the planner: same samples / error as the oracle
    either way."""
    st = synth.generate(**dict(PARITY_CONFIGS["c3_ms16_lpc8"], write_total=0, seed=4400))
    avail = len(st.flac) - st.frames_begin
    planted = synth.generate(channels=2, bps=16, stereo_mode=1, block_size=4096, n_samples=4096 * 5, write_total=0,
                             predictor=3, order=8, plant_sync_every=2, seed=93).flac
    cases = {  # name: (stream, streams the planner finishes of the 3 in the batch)
        "plain": (st.flac, 0),
        "trailing_3_bytes": (st.flac + b"\x00\x01\x02", 0),
        "min_frame_too_large": (_with_min_frame(st.flac, avail // 2), 0),
        "min_frame_unknown": (_with_min_frame(st.flac, 0), 0),
        "trailing_4_bytes": (st.flac + b"\x00\x01\x02\x03", 3),
        "planted_syncs": (planted, 3),
    }
    for name, (data, seq) in cases.items():
        r = oracle.decode(data)
        b = zflac_amd.Batch([data] * 3, timing=True)
        for _ in range(2):  # the second run reuses the reservation and the unit read-back
            b.run()
            assert b.timings().sequential_streams == seq, name
            for i in range(3):
                assert b.error_name(i) == r.error, name
                if r.error == "OK":
                    d = b.read(i)
                    np.testing.assert_array_equal(d.samples.values, r.samples, err_msg=name)
                    assert d.samples.values.size == r.samples.size, name
        b.close()
    assert oracle.decode(st.flac).error == "OK"
    assert oracle.decode(st.flac + b"\x00\x01\x02\x03").error != "OK"


def test_unknown_total_all_formats(gpu_ready):
    """Every parity config written with STREAMINFO total 0, in one batch: samples equal to the
    oracle's, and every stream certified by the parallel pass (k_verify to EOF; the formats,
    channel counts, block sizes and the variable-blocking stream all reserved by the
    creation's pre-scan), none left to the sequential planner."""
    names = sorted(PARITY_CONFIGS)
    sts = [synth.generate(**dict(PARITY_CONFIGS[n], write_total=0, seed=4600 + i)) for i, n in enumerate(names)]
    b = zflac_amd.Batch([st.flac for st in sts], timing=True)
    b.run()
    assert b.timings().sequential_streams == 0
    for i, (n, st) in enumerate(zip(names, sts)):
        r = oracle.decode(st.flac)
        assert b.error_name(i) == r.error, n
        if r.error == "OK":
            np.testing.assert_array_equal(b.read(i).samples.values, r.samples, err_msg=n)
    b.close()


def test_unknown_total_truncations_and_tails(gpu_ready):
    """Total-unknown streams cut at random byte offsets (mid-frame, at frame boundaries, 1-3
    bytes past one) or followed by random tails (garbage, a copy of a frame header, a whole
    frame): one batch, every stream's error name and samples equal to the oracle's, whichever
    of the parallel pass and the planner finished it."""
    rng = np.random.default_rng(4700)
    st = synth.generate(**dict(PARITY_CONFIGS["c3_ms16_lpc8"], write_total=0, seed=4701))
    fo = [int(x) for x in st.frame_offsets] + [len(st.flac)]
    datas = []
    for _ in range(12):  # anywhere in the frame section
        datas.append(st.flac[: int(rng.integers(st.frames_begin + 1, len(st.flac)))])
    for b in fo[1:]:  # at a frame boundary, and 1..3 bytes past it
        datas += [st.flac[:b], st.flac[: b + int(rng.integers(1, 4))]]
    for n in (1, 2, 3, 4, 5, 17, 300):
        datas.append(st.flac + rng.integers(0, 256, n, dtype=np.uint8).tobytes())
    datas.append(st.flac + st.flac[fo[0]: fo[0] + 8])  # a frame header with nothing after it
    datas.append(st.flac + st.flac[fo[1]: fo[2]])  # one more whole frame
    b = zflac_amd.Batch(datas)
    b.run()
    for i, data in enumerate(datas):
        r = oracle.decode(data)
        try:
            d = b.read(i)
            err = "OK"
        except errors.ZflacError as e:
            err, d = type(e).__name__, None
        assert err == r.error, (i, len(data))
        if d is not None:
            np.testing.assert_array_equal(d.samples.values, r.samples)
    b.close()


def test_pipelined_device_md5_overlapped(gpu_ready):
    """ZFLAC_FLAG_DEVICE_MD5 with three batches in flight (submit / wait): the certified
    streams' digests come from the k_md5 enqueued by submit, the sequential ones (a false
    sync, an unknown total, a broken frame) from wait; every digest equals STREAMINFO and
    hashlib over the oracle's samples, and a wrong STREAMINFO MD5 is InvalidChecksum."""
    c5 = [s.flac for s in synth.generate_many([synth.config_c5(i, n_frames=6) for i in range(40)])]
    seq = [synth.generate(**dict(PARITY_CONFIGS["c3_ms16_lpc8"], write_total=0, seed=4200)).flac,
           _CASES["wrong_md5"][0], _CASES["bad_sync_frame2"][0]]
    mixed = [synth.generate(**dict(PARITY_CONFIGS[n], seed=4300 + i)).flac
             for i, n in enumerate(["c4_24bit_lpc32_wasted", "mono8_lpc3", "stereo12_ms", "ch3_16"])]
    groups = [c5, seq + c5[:5], mixed]
    bs = [zflac_amd.Batch(g, device_md5=True, timing=True) for g in groups]
    refs = {}
    for rnd in range(2):
        for b in bs:
            b.submit()
        for b in bs:
            b.wait()
        for g, b in zip(groups, bs):
            for i, data in enumerate(g):
                if data not in refs:
                    refs[data] = oracle.decode(data, "fast")
                r = refs[data]
                rc, _ = b.info(i)
                assert errors.NAMES.get(rc) == r.error, (rnd, i)
                if r.error != "OK":
                    continue
                assert b.md5(i) == _streaminfo_md5(data), (rnd, i)
                assert b.md5(i) == _md5_pre_justify(r.samples, r.bits_per_sample), (rnd, i)
        assert bs[0].timings().md5_ms > 0
    for b in bs:
        b.close()


_WALK_CASES = ["c3_ms16_lpc8", "c4_24bit_lpc32_wasted", "ch3_16", "ch6_24_wasted", "ch8_16_fixed", "stereo32",
               "longcodes24_k16", "longcodes16_k3", "ms20_lpc16_escape", "ls16_fixed_mix", "uncommon_po15",
               "auto_stereo_lpc12", "stereo12_ms", "uncommon_block65535", "lpc32_16bit"]


@pytest.mark.parametrize("walk", ["lane", "wave"])
def test_both_walks_parity(gpu_ready, walk):
    """k_walk (lane per frame) and k_walk_wave (wave per frame, wave-wide Rice scan) give the
    same subframe starts: every parity config with 2+ channels, plus the malformed cases,
    decoded in one batch under each walk, equal to the oracle (errors included)."""
    names = [n for n in _WALK_CASES if n in PARITY_CONFIGS]
    datas = [synth.generate(**dict(PARITY_CONFIGS[n], seed=4500 + i)).flac for i, n in enumerate(names)]
    datas += [_CASES[c][0] for c in sorted(_CASES)]
    b = zflac_amd.Batch(datas, walk=walk)
    b.run()
    for i, data in enumerate(datas):
        r = oracle.decode(data)
        try:
            d = b.read(i)
            err = "OK"
        except errors.ZflacError as e:
            err, d = type(e).__name__, None
        assert err == r.error, (walk, i)
        if d is not None:
            np.testing.assert_array_equal(d.samples.values, r.samples)
    b.close()


@pytest.mark.parametrize("walk", ["lane", "wave"])
def test_both_walks_mutants(gpu_ready, walk):
    """Bit-flip mutants of the C3 / C4 fixtures under each walk: the walk must never read out
    of bounds or hang on garbage, and the frame's error is the oracle's."""
    import random

    rng = random.Random(4600)
    bases = [synth.generate(**dict(PARITY_CONFIGS[n], seed=4601)).flac for n in ("c3_ms16_lpc8", "c4_24bit_lpc32_wasted")]
    datas = []
    for k in range(60):
        d = bytearray(bases[k % 2])
        for _ in range(1 + k % 3):
            p = rng.randrange(60, len(d))
            d[p] ^= 1 << rng.randrange(8)
        datas.append(bytes(d))
    b = zflac_amd.Batch(datas, walk=walk)
    b.run()
    for i, data in enumerate(datas):
        r = oracle.decode(data)
        try:
            d = b.read(i)
            err = "OK"
        except errors.ZflacError as e:
            err, d = type(e).__name__, None
        assert err == r.error, (walk, i)
        if d is not None:
            np.testing.assert_array_equal(d.samples.values, r.samples)
    b.close()


def test_huge_stream_multi_pass_chunk_scan(gpu_ready):
    """One 590 MB stream (C3, 65,536 frames, the SURVEY 8(d) size): 18 Ki scan chunks, i.e.
    five of k_scan_chunks' 4,096-chunk tiles, with the running sums carried from tile to tile;
    decode() verifies the STREAMINFO MD5 of the whole 1 GiB output."""
    st = synth.generate(**synth.config_c3(n_frames=1024))
    data = synth.tile_flac(st, 64)
    assert len(data) > 16384 * 32768
    d = zflac_amd.decode(data)
    assert d.samples.values.size == st.pcm.size * 64
    np.testing.assert_array_equal(d.samples.values[: st.pcm.size], expected_samples(st))


@pytest.mark.parametrize("chunks", [4097, 8193])
def test_chunk_scan_tile_boundary(gpu_ready, chunks):
    """k_scan_chunks carries its candidate and sample-unit sums from one 4,096-chunk tile to
    the next: a batch whose scan chunks end just past one and two tiles, with streams before
    and after the long one. A wrong carry misplaces frames, which the STREAMINFO MD5 of every
    stream (checked by read) and the oracle comparison catch."""
    st = synth.generate(**synth.config_c3(n_frames=64))
    seg = len(st.flac) - int(st.frame_offsets[0])
    big = synth.tile_flac(st, -(-(chunks * 32768) // seg))
    small = [synth.generate(**synth.config_c5(i, n_frames=4)).flac for i in range(3)]
    streams = [small[0], big, small[1], small[2]]
    b = zflac_amd.Batch(streams)
    b.run()
    for i, data in enumerate(streams):
        d = b.read(i, verify_md5=True)
        if data is big:
            assert d.samples.values.size == st.pcm.size * (-(-(chunks * 32768) // seg))
            np.testing.assert_array_equal(d.samples.values[: st.pcm.size], expected_samples(st))
        else:
            np.testing.assert_array_equal(d.samples.values, oracle.decode(data).samples)
    b.close()
