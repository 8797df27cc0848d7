"""CPU tests: the oracle (C restatement of zflac decode) against the reference's golden
vectors, RFC 1321 MD5 vectors, the synthetic writer's ground truth, and the reference's
expected error names. No GPU involved."""
import hashlib

import numpy as np
import pytest

import oracle
import synth

from . import malformed
from .util import PARITY_CONFIGS, expected_samples, load_fixture_manifest, load_kats, GOLDEN


@pytest.mark.parametrize("kat", load_kats(), ids=lambda k: k["name"])
def test_kat_basic_zig(kat):
    """tests/basic.zig:4-95 known answers (RFC 9639 Appendix D streams)."""
    r = oracle.decode(bytes.fromhex(kat["flac_hex"]))
    assert r.error == "OK"
    assert r.channels == kat["channels"]
    assert {"s8": np.int8, "s16": np.int16, "s32": np.int32}[kat["sample_kind"]] == r.samples.dtype
    assert r.samples.tolist() == kat["expected"]


@pytest.mark.parametrize("flavor", ["checked", "fast"])
def test_kat_flavors_agree(flavor):
    for kat in load_kats():
        r = oracle.decode(bytes.fromhex(kat["flac_hex"]), flavor)
        assert r.samples.tolist() == kat["expected"]


@pytest.mark.parametrize("msg", [b"", b"a", b"abc", b"message digest", b"abcdefghijklmnopqrstuvwxyz",
                                 b"1234567890" * 8, bytes(range(256)) * 5])
def test_md5_rfc1321(msg):
    assert oracle.md5(msg) == hashlib.md5(msg).digest()


@pytest.mark.parametrize("name", sorted(PARITY_CONFIGS))
def test_generator_roundtrip(name):
    """writer -> oracle reproduces the writer's source PCM exactly (and its MD5)."""
    st = synth.generate(**PARITY_CONFIGS[name])
    r = oracle.decode(st.flac)
    assert r.error == "OK", name
    np.testing.assert_array_equal(r.samples, expected_samples(st))
    assert r.channels == st.config["channels"]


def test_release_fast_matches_checked():
    for name in ["c3_ms16_lpc8", "c4_24bit_lpc32_wasted", "mono8_lpc3", "ch6_24_wasted"]:
        st = synth.generate(**PARITY_CONFIGS[name])
        a = oracle.decode(st.flac, "checked")
        b = oracle.decode(st.flac, "fast")
        np.testing.assert_array_equal(a.samples, b.samples)


_CASES = malformed.cases()


@pytest.mark.parametrize("case", sorted(_CASES))
def test_malformed_expected_errors(case):
    data, expected = _CASES[case]
    r = oracle.decode(data)
    if expected is not None:
        assert r.error == expected, case


def test_golden_fixtures_pinned():
    """Committed fixtures: oracle output digest == manifest (made by tools/make_fixtures.py)."""
    import os

    man = load_fixture_manifest()
    assert len(man["fixtures"]) >= 5
    for fx in man["fixtures"]:
        data = open(os.path.join(GOLDEN, fx["file"]), "rb").read()
        r = oracle.decode(data)
        assert r.error == fx["error"], fx["file"]
        if r.error == "OK":
            assert hashlib.sha256(r.samples.tobytes()).hexdigest() == fx["samples_sha256"], fx["file"]
            assert r.samples.size == fx["n_samples"]
