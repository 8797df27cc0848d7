"""Optional frame CRC-16 check (ZFLAC_FLAG_CHECK_CRC16).

zflac reads each frame's CRC-16 trailer and ignores it (src/zflac.zig:548-551), so the
check is opt-in: without the flag every stream here must decode exactly as zflac does
(oracle), with it a frame whose trailer differs makes the stream FrameCrcMismatch, ahead of
a later frame's error and of the STREAMINFO MD5 check (zflac's read order).

The expected CRCs come from crc16_ref below (x^16 + x^15 + x^2 + 1, MSB first, init 0,
RFC 9639 9.1.8), pinned on the CPU against the trailers the generator writes."""
import numpy as np
import pytest

import oracle
import synth

STEREO = dict(channels=2, bps=16, stereo_mode=10, order=8, block_size=4096, n_samples=4096 * 6, seed=71)


def crc16_ref(data: bytes) -> int:
    crc = 0
    for b in data:
        crc ^= b << 8
        for _ in range(8):
            crc = ((crc << 1) ^ 0x8005) if crc & 0x8000 else (crc << 1)
            crc &= 0xFFFF
    return crc


def _frames(st):
    offs = [int(x) for x in st.frame_offsets] + [len(st.flac)]
    return list(zip(offs[:-1], offs[1:]))


def _flip(data: bytes, pos: int, bit: int = 0) -> bytes:
    b = bytearray(data)
    b[pos] ^= 1 << bit
    return bytes(b)


CONFIGS = {
    "ms16": STEREO,
    "mono8": dict(channels=1, bps=8, order=4, precision=7, block_size=1152, n_samples=1152 * 7, noise_lsb=1.0,
                  tone_amp=0.3, seed=72),
    "lr24": dict(channels=2, bps=24, stereo_mode=1, order=12, precision=14, block_size=4608, n_samples=4608 * 3,
                 noise_lsb=64.0, seed=73),
    "ch6_16": dict(channels=6, bps=16, order=6, block_size=1024, n_samples=1024 * 5, seed=74),
    "tiny_blocks": dict(channels=2, bps=16, stereo_mode=1, order=2, block_size=16, n_samples=16 * 40, seed=75),
    "verbatim": dict(channels=2, bps=16, predictor=0, stereo_mode=1, block_size=2048, n_samples=2048 * 4, seed=76),
    "unknown_total": dict(STEREO, write_total=0, seed=77),
}


@pytest.mark.parametrize("name", sorted(CONFIGS))
def test_generator_trailers_match_reference_crc(name):
    st = synth.generate(**CONFIGS[name])
    for a, e in _frames(st):
        assert crc16_ref(st.flac[a:e - 2]) == int.from_bytes(st.flac[e - 2:e], "big"), (name, a)


def test_crc16_ref_known_answer():
    # CRC-16/BUYPASS (= FLAC's frame CRC) check value of "123456789"
    assert crc16_ref(b"123456789") == 0xFEE8


# ---- GPU --------------------------------------------------------------------------------

def _decode(data, crc):
    import zflac_amd
    from zflac_amd import errors

    try:
        d = zflac_amd.decode(data, check_crc16=crc)
        return "OK", d.samples.values
    except errors.ZflacError as e:
        return type(e).__name__, None


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(CONFIGS))
def test_crc16_clean_streams_decode_unchanged(name):
    st = synth.generate(**CONFIGS[name])
    err, v = _decode(st.flac, True)
    ref = oracle.decode(st.flac)
    assert err == ref.error == "OK"
    np.testing.assert_array_equal(v, ref.samples)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["ms16", "unknown_total", "ch6_16", "tiny_blocks"])
@pytest.mark.parametrize("which", [0, 2, -1])
def test_crc16_bad_trailer(name, which):
    """A flipped trailer bit: zflac (and the default path) decode it; the check reports it on
    the certified path, a stream whose STREAMINFO total is unknown included (certified by the
    parallel pass since round 6; the planner's case is test_crc16_before_later_frame_error)."""
    st = synth.generate(**CONFIGS[name])
    fr = _frames(st)
    a, e = fr[which]
    bad = _flip(st.flac, e - 1, 3)
    err0, v0 = _decode(bad, False)
    ref = oracle.decode(bad)
    assert err0 == ref.error == "OK"
    np.testing.assert_array_equal(v0, ref.samples)
    assert _decode(bad, True)[0] == "FrameCrcMismatch"


@pytest.mark.gpu
def test_crc16_before_md5():
    """Verbatim sample bits flipped: zflac decodes other samples and fails the MD5 check
    (InvalidChecksum); with the check, frame 1's CRC mismatch comes first."""
    st = synth.generate(**CONFIGS["verbatim"])
    a, e = _frames(st)[1]
    bad = _flip(st.flac, (a + e) // 2, 5)
    assert oracle.decode(bad).error == "InvalidChecksum"
    assert _decode(bad, False)[0] == "InvalidChecksum"
    assert _decode(bad, True)[0] == "FrameCrcMismatch"


@pytest.mark.gpu
def test_crc16_before_later_frame_error():
    """Frame 1's trailer is wrong and frame 3's header is broken: zflac stops at frame 3;
    with the check the earlier CRC mismatch is the stream's error (sequential planner)."""
    st = synth.generate(**STEREO)
    fr = _frames(st)
    bad = _flip(st.flac, fr[1][1] - 1, 0)
    bad = _flip(bad, fr[3][0] + 1, 7)  # sync code 0xFFF8 -> 0xFF78
    ref = oracle.decode(bad).error
    assert ref not in ("OK", "InvalidChecksum")
    assert _decode(bad, False)[0] == ref
    assert _decode(bad, True)[0] == "FrameCrcMismatch"


@pytest.mark.gpu
def test_crc16_batch_mixed():
    """A batch where only some streams carry a bad trailer; the others are unaffected, and
    crc16_ms is reported."""
    import zflac_amd

    good = [synth.generate(**dict(STEREO, seed=80 + i, n_samples=4096 * 3)).flac for i in range(6)]
    streams = list(good)
    for i in (1, 4):
        a, e = _frames(synth.generate(**dict(STEREO, seed=80 + i, n_samples=4096 * 3)))[1]
        streams[i] = _flip(good[i], e - 2, 1)
    b = zflac_amd.Batch(streams, timing=True, check_crc16=True)
    try:
        b.run()
        names = [b.error_name(i) for i in range(len(streams))]
        assert names == ["OK", "FrameCrcMismatch", "OK", "OK", "FrameCrcMismatch", "OK"]
        assert b.timings().crc16_ms > 0
        for i in (0, 2):
            np.testing.assert_array_equal(b.read(i).samples.values, oracle.decode(streams[i]).samples)
    finally:
        b.close()


@pytest.mark.gpu
def test_crc16_frames_past_total_are_not_checked():
    """A whole extra frame with a corrupted trailer after the STREAMINFO total (its header is
    a CRC-8-valid sync): zflac stops reading at the total (src/zflac.zig:341), so the stream
    decodes and, with the check, stays OK; the same on the batch path."""
    import zflac_amd

    st = synth.generate(**STEREO)
    a, e = _frames(st)[1]
    extra = _flip(st.flac[a:e], e - a - 1, 2)
    data = st.flac + extra
    ref = oracle.decode(data)
    assert ref.error == "OK"
    for crc in (False, True):
        err, v = _decode(data, crc)
        assert err == "OK", crc
        np.testing.assert_array_equal(v, ref.samples)
    b = zflac_amd.Batch([data, st.flac], check_crc16=True)
    try:
        b.run()
        assert [b.error_name(i) for i in range(2)] == ["OK", "OK"]
    finally:
        b.close()
