"""Parity edges (tests/edges.py): zflac's constant-side quirk, planted false frame syncs,
out-of-domain values (Debug-zflac traps), bit-flip mutants of the committed fixtures, the
reference's faulty/11 case and its expected-output convention (.raw slices).

CPU tests pin the oracle's answers; `gpu` tests hold the HIP path (through the C ABI) to
the oracle: same zflac error name, and bit-exact samples whenever samples exist (OK, and
InvalidChecksum, whose decoded samples both sides still produce)."""
import time

import numpy as np
import pytest

import oracle
import synth
import zflac_amd
from zflac_amd import errors

from . import edges
from .util import expected_samples

_CONST = edges.const_side_cases()
_PLANT = edges.planted_sync_cases()
_OOD = edges.out_of_domain_cases()
_ALL = {**_CONST, **_PLANT, **_OOD}


# ---------------------------------------------------------------------------- CPU
@pytest.mark.parametrize("name", sorted(_ALL))
def test_oracle_edge_expectations(name):
    data, exp, pcm = _ALL[name]
    r = oracle.decode(data)
    if exp is not None:
        assert r.error == exp, name
    if exp == "OK" and pcm is not None:
        assert np.array_equal(r.samples.astype(np.int64) >> _js(r.bits_per_sample), pcm)


def _js(bps):
    return 16 - bps if 9 <= bps <= 15 else 32 - bps if 17 <= bps <= 31 else 0


def test_planted_sync_is_present():
    """Every other frame of each planted stream carries a byte-exact copy of its own header
    (CRC-8 included) inside the frame, off the frame chain."""
    for name, (data, _, _) in _PLANT.items():
        offs = edges.PLANT_FRAME_OFFSETS[name]
        ends = offs[1:] + [len(data)]
        planted = 0
        for fo, fe in zip(offs, ends):
            hdr = data[fo:fo + 5]  # sync, block size / rate, channels / depth, coded number
            if data.find(hdr, fo + 1, fe) > 0:
                planted += 1
        assert planted >= len(offs) // 2, (name, planted, len(offs))


def test_faulty11_incorrect_metadata_length():
    st = synth.generate(**edges.STEREO16)
    assert oracle.decode(edges.incorrect_metadata_length_case(st.flac, st.frames_begin)).error == \
        "InvalidMetadataHeader"


def test_mutants_decode_on_the_oracle():
    """The mutant set covers several error classes (so the GPU comparison means something)."""
    names = {oracle.decode(d).error for d, _, _ in edges.fixture_mutants().values()}
    assert {"InvalidChecksum", "OK", "OutOfDomain"} <= names and len(names) >= 5


def test_raw_slices_convention():
    """The reference's expected outputs are left-justified (src/zflac.zig:287-306): 12-bit
    values are multiples of 16, 20-bit of 4096, 24-bit of 256; 8-bit files are unsigned."""
    for meta, v in edges.load_raw_slices():
        bps = meta["bps"]
        assert v.size == meta["n_values"]
        if meta["container"] == "s8u":
            assert v.dtype == np.int8
            continue
        js = _js(bps)
        assert np.all((v.astype(np.int64) & ((1 << js) - 1)) == 0), meta["file"]
        if js:
            assert meta["trailing_zeros"] >= js


def test_raw_slices_roundtrip_oracle():
    """Re-encode each slice (un-justified) with the writer; the oracle reproduces it."""
    for meta, v in edges.load_raw_slices():
        st = synth.generate(pcm=edges.unjustify(v, meta["bps"]), channels=meta["channels"], bps=meta["bps"],
                            stereo_mode=-1 if meta["channels"] == 2 else 1, block_size=4096, order=8, seed=5)
        r = oracle.decode(st.flac)
        assert r.error == "OK", meta["file"]
        assert np.array_equal(r.samples, v), meta["file"]


# ---------------------------------------------------------------------------- GPU
def _gpu_result(b, i):
    """(error name, samples or None) of batch member i, samples also on InvalidChecksum."""
    rc, _ = b.info(i)
    if rc:
        return errors.NAMES.get(rc, f"E{rc}"), None
    d = b.read(i, verify_md5=False)
    try:
        b.read(i, verify_md5=True)
        return "OK", d.samples.values
    except errors.ZflacError as e:
        return type(e).__name__, d.samples.values


def _check_batch(cases, gpu_ready, label):
    names = sorted(cases)
    b = zflac_amd.Batch([cases[n][0] for n in names])
    b.run()
    bad = []
    for i, n in enumerate(names):
        data, exp, _ = cases[n]
        r = oracle.decode(data)
        err, samples = _gpu_result(b, i)
        if err != r.error:
            bad.append((n, "error", err, r.error))
            continue
        if r.samples is not None and not np.array_equal(samples, r.samples):
            bad.append((n, "samples"))
    b.close()
    assert not bad, f"{label}: {bad[:8]} ({len(bad)} of {len(names)})"


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(_ALL))
def test_gpu_edge_single(gpu_ready, name):
    """decode() (open + read) of each edge stream: error name and samples equal the oracle's."""
    data, exp, pcm = _ALL[name]
    r = oracle.decode(data)
    try:
        d = zflac_amd.decode(data)
        err, got = "OK", d.samples.values
    except errors.ZflacError as e:
        err, got = type(e).__name__, None
    assert err == r.error, (name, err, r.error)
    if err == "OK":
        np.testing.assert_array_equal(got, r.samples)


@pytest.mark.gpu
def test_gpu_edges_batched(gpu_ready):
    """All edge streams in one mixed batch (several classes, repair paths side by side)."""
    _check_batch(_ALL, gpu_ready, "edges")


@pytest.mark.gpu
def test_gpu_planted_sync_repair(gpu_ready):
    """The false candidates really send the streams down the repair path (sequential
    planner), the output is still the source PCM, and the repair cost is reported."""
    for name, (data, _, pcm) in _PLANT.items():
        t0 = time.perf_counter()
        d = zflac_amd.decode(data)
        dt = time.perf_counter() - t0
        ref = oracle.decode(data)
        np.testing.assert_array_equal(d.samples.values, ref.samples)
        print(f"{name}: {len(data)} B, repair-path decode() {dt * 1e3:.2f} ms")
    # the fast path alone cannot certify a planted stream: force the comparison
    data = _PLANT["plant_lr16"][0]
    b = zflac_amd.Batch([data], force_slow=True)
    b.run()
    np.testing.assert_array_equal(b.read(0).samples.values, oracle.decode(data).samples)
    b.close()


def test_bad_crc8_case_on_the_oracle():
    data, pcm = edges.bad_crc8_case(frames=6)
    r = oracle.decode(data)
    assert r.error == "OK"
    np.testing.assert_array_equal(r.samples, pcm.reshape(-1))


@pytest.mark.gpu
@pytest.mark.parametrize("total", [1, 0])
def test_gpu_bad_crc8_headers_batched_probes(gpu_ready, total):
    """No header passes the indexer's CRC-8 filter: the sequential planner gets every record
    from its batched probes (a handful of launches, not one per frame)."""
    data, pcm = edges.bad_crc8_case(frames=300, write_total=total)
    t0 = time.perf_counter()
    d = zflac_amd.decode(data)
    dt = time.perf_counter() - t0
    np.testing.assert_array_equal(d.samples.values, pcm.reshape(-1))
    print(f"300 frames, every CRC-8 wrong: decode() {dt * 1e3:.1f} ms")
    assert dt < 10.0


@pytest.mark.gpu
def test_gpu_faulty11(gpu_ready):
    st = synth.generate(**edges.STEREO16)
    with pytest.raises(errors.InvalidMetadataHeader):
        zflac_amd.decode(edges.incorrect_metadata_length_case(st.flac, st.frames_begin))


@pytest.mark.gpu
def test_gpu_bitflip_mutants(gpu_ready):
    """200 seeded bit-flip mutants of the C3 / C4 fixtures: same error name as the oracle,
    identical samples whenever both produce them, no device fault."""
    _check_batch(edges.fixture_mutants(), gpu_ready, "mutants")


@pytest.mark.gpu
def test_gpu_raw_slices(gpu_ready):
    """The reference's expected outputs (slices), re-encoded by the writer, decode on the
    GPU to exactly the reference's bytes: left-justify and 8-bit conventions included."""
    for meta, v in edges.load_raw_slices():
        st = synth.generate(pcm=edges.unjustify(v, meta["bps"]), channels=meta["channels"], bps=meta["bps"],
                            stereo_mode=-1 if meta["channels"] == 2 else 1, block_size=4096, order=8, seed=5)
        d = zflac_amd.decode(st.flac)
        assert d.samples.values.dtype == v.dtype, meta["file"]
        np.testing.assert_array_equal(d.samples.values, v, err_msg=meta["file"])


@pytest.mark.gpu
def test_gpu_ragged_batch_alignment(gpu_ready):
    """Streams whose sample counts are not multiples of 8 do not misalign the ones after
    them: every stream's device region starts 32-byte aligned and decodes bit-exactly."""
    cfgs = [synth.config_c5(i, n_frames=3) for i in range(12)]
    for i, c in enumerate(cfgs):
        c["n_samples"] = 4096 * 3 - (i * 37) % 4096 + 1  # ragged tails
    sts = synth.generate_many(cfgs)
    b = zflac_amd.Batch([s.flac for s in sts])
    b.run()
    for i, s in enumerate(sts):
        assert b.device_samples(i) % 32 == 0, i
        np.testing.assert_array_equal(b.read(i).samples.values, expected_samples(s))
    b.close()


@pytest.mark.gpu
def test_gpu_batch_queries_before_run(gpu_ready):
    st = synth.generate(**synth.config_c3(n_frames=2))
    b = zflac_amd.Batch([st.flac])
    assert b.info(0)[0] == 14  # InvalidArgument until run()
    assert b.device_samples(0) == 0
    b.run()
    assert b.info(0)[0] == 0
    b.close()
