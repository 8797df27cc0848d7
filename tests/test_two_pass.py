"""Two-pass stereo decode (ZFLAC_TWO_PASS=1, 16-bit stereo classes): pass
S0 decodes channel 0 of every frame into scratch rows and records where channel 1 starts,
pass S1 decodes channel 1 and decorrelates it with channel 0 read back; no walk. Held to
the oracle exactly like the walk path: same zflac error name, bit-exact samples, and the
fallback to the walk path when a class meets a bucket the plan did not predict (constant /
verbatim subframes, an unpredicted order)."""
import numpy as np
import pytest

import oracle
import synth
import zflac_amd
from zflac_amd import errors

from . import edges
from .util import PARITY_CONFIGS, expected_samples

pytestmark = pytest.mark.gpu

# every 16-bit-container stereo config (9..16 bits per sample)
_STEREO16 = sorted(n for n, c in PARITY_CONFIGS.items() if c.get("channels") == 2 and 9 <= c.get("bps", 16) <= 16)
# constant / verbatim subframes in the first frame: the plan predicts a MIX bucket, so these
# classes keep the walk path from the start
_MIX_FIRST = {"silence_constant", "verbatim_all"}
# one predictor order and no constant / verbatim subframes anywhere: two-pass on every run
_SIMPLE = {"c3_ms16_lpc8", "rs16_lpc5", "lpc32_16bit", "longcodes16_k3", "stereo12_ms", "odd_block_4095"}


@pytest.fixture
def two_pass(monkeypatch):
    monkeypatch.setenv("ZFLAC_TWO_PASS", "1")


def _result(b, i):
    try:
        return "OK", b.read(i).samples.values
    except errors.ZflacError as e:
        return type(e).__name__, None


@pytest.mark.parametrize("name", _STEREO16)
def test_two_pass_parity_configs(gpu_ready, two_pass, name):
    """Each 16-bit stereo config as its own class (three seeds, run twice): bit-exact with
    the oracle and the writer's PCM. A class that did not fall back on its first run stays
    two-pass; one that fell back (or started with a MIX bucket) stays on the walk path."""
    sts = [synth.generate(**dict(PARITY_CONFIGS[name], seed=7000 + k)) for k in range(3)]
    b = zflac_amd.Batch([s.flac for s in sts], timing=True)
    modes = []
    for run in range(2):
        b.run()
        for i, st in enumerate(sts):
            r = oracle.decode(st.flac)
            err, got = _result(b, i)
            assert err == r.error, (name, i, err, r.error)
            if err == "OK":
                np.testing.assert_array_equal(got, r.samples)
                np.testing.assert_array_equal(got, expected_samples(st))
        modes.append((b.timings().two_pass, b.timings().rest_launches))
    if name in _MIX_FIRST:
        assert modes[0][0] == 0 and modes[1][0] == 0
    if name in _SIMPLE:
        assert modes == [(1, 0), (1, 0)], modes
    assert modes[1][1] == 0  # whatever happened in run 0 was learned
    b.close()


def test_two_pass_is_taken_for_c3(gpu_ready, two_pass):
    """A C3-shaped class (M/S, LPC-8) runs two-pass on every run (no fallback)."""
    sts = [synth.generate(**synth.config_c3(n_frames=6, seed=8100 + k)) for k in range(70)]
    b = zflac_amd.Batch([s.flac for s in sts], timing=True)
    for _ in range(2):
        b.run()
        assert b.timings().two_pass == 1
        assert b.timings().rest_launches == 0
        for i, st in enumerate(sts):
            np.testing.assert_array_equal(b.read(i).samples.values, expected_samples(st))
    b.close()


def test_two_pass_unpredicted_bucket_falls_back(gpu_ready, two_pass):
    """Frames 0-2 LPC order 8, frames 3-5 order 32 (test_gpu's spliced stream): the plan has
    no order-32 launch, so the first run falls back to the walk path (one synchronous rerun
    of the class) and stays exact; the next run uses the walk path with the learned launch
    set, no fallback."""
    from .test_gpu import _spliced_order_change

    data = _spliced_order_change()
    r = oracle.decode(data)
    b = zflac_amd.Batch([data] * 70, timing=True)
    b.run()
    assert b.timings().rest_launches == 1 and b.timings().two_pass == 0
    for i in range(0, 70, 9):
        np.testing.assert_array_equal(b.read(i).samples.values, r.samples)
    b.run()
    assert b.timings().rest_launches == 0 and b.timings().two_pass == 0
    for i in range(0, 70, 9):
        np.testing.assert_array_equal(b.read(i).samples.values, r.samples)
    b.close()


_OOD16 = {k: v for k, v in {**edges.out_of_domain_cases(), **edges.const_side_cases()}.items()
          if k.endswith(("_ms", "_ls", "_rs", "_rs_verbatim", "16")) or "const" in k}


@pytest.mark.parametrize("name", sorted(_OOD16))
def test_two_pass_edges(gpu_ready, two_pass, name):
    """Out-of-domain (side and decorrelation overflow, LPC sum overflow) and constant-side
    streams, each alone in its batch: the oracle's error and samples."""
    data, _, _ = _OOD16[name]
    r = oracle.decode(data)
    b = zflac_amd.Batch([data])
    b.run()
    err, got = _result(b, 0)
    assert err == r.error, (name, err, r.error)
    if err == "OK":
        np.testing.assert_array_equal(got, r.samples)
    b.close()


def test_two_pass_mutants(gpu_ready, two_pass):
    """The 200 bit-flip mutants of the C3 / C4 fixtures (the C3 ones form a 16-bit stereo
    class): the oracle's error name and samples, no device fault."""
    cases = edges.fixture_mutants()
    names = sorted(cases)
    b = zflac_amd.Batch([cases[n][0] for n in names])
    b.run()
    bad = []
    for i, n in enumerate(names):
        r = oracle.decode(cases[n][0])
        err, got = _result(b, i)
        if err != r.error:
            bad.append((n, err, r.error))
        elif r.samples is not None and got is not None and not np.array_equal(got, r.samples):
            bad.append((n, "samples"))
    b.close()
    assert not bad, bad[:8]
