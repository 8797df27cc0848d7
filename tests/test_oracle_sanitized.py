"""The oracle's checked build under AddressSanitizer + UndefinedBehaviorSanitizer (CPU).

Every stream the other suites feed the oracle (committed fixtures, the reference's KATs,
the generator configs, the malformed catalogue, the parity edges and the 200 bit-flip
mutants) is decoded by oracle/sanitize_main.c built with -fsanitize=address,undefined
-fno-sanitize-recover=all; the run must be clean and agree with the unsanitized oracle
(error name, sample count, sample digest)."""
import os
import shutil
import subprocess

import pytest

import oracle
import synth

from . import edges, malformed
from .util import GOLDEN, PARITY_CONFIGS, load_fixture_manifest, load_kats

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE = os.path.join(os.path.dirname(HERE), "oracle")


def _fnv(b: bytes) -> str:
    h = 0xcbf29ce484222325
    for x in b:
        h = ((h ^ x) * 0x100000001b3) & 0xFFFFFFFFFFFFFFFF
    return f"{h:016x}"


def _streams():
    out = {}
    for fx in load_fixture_manifest()["fixtures"]:
        out["fx_" + fx["file"]] = open(os.path.join(GOLDEN, fx["file"]), "rb").read()
    for k in load_kats():
        out["kat_" + k["name"]] = bytes.fromhex(k["flac_hex"])
    for n, c in PARITY_CONFIGS.items():
        if c.get("block_size", 0) < 32768:  # the two 32 Ki+ block configs are slow under ASan
            out["cfg_" + n] = synth.generate(**c).flac
    for n, (d, _) in malformed.cases().items():
        out["mal_" + n] = d
    for fn in (edges.const_side_cases, edges.planted_sync_cases, edges.out_of_domain_cases):
        for n, (d, _, _) in fn().items():
            out["edge_" + n] = d
    for n, (d, _, _) in edges.fixture_mutants().items():
        out["mut_" + n] = d
    return out


@pytest.mark.skipif(shutil.which("gcc") is None, reason="needs gcc")
def test_oracle_asan_ubsan(tmp_path):
    exe = tmp_path / "zfo_sanitized"
    subprocess.check_call(["gcc", "-O1", "-g", "-std=c11", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
                           "-fno-omit-frame-pointer", "-I", ORACLE, os.path.join(ORACLE, "zflac_oracle.c"),
                           os.path.join(ORACLE, "sanitize_main.c"), "-o", str(exe)])
    streams = _streams()
    names = sorted(streams)
    paths = []
    for i, n in enumerate(names):
        p = tmp_path / f"{i:04d}.flac"
        p.write_bytes(streams[n])
        paths.append(str(p))
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1")
    env.pop("LD_PRELOAD", None)
    r = subprocess.run([str(exe)] + paths, capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "runtime error" not in r.stderr, r.stderr[-4000:]
    lines = r.stdout.splitlines()
    assert len(lines) == len(names)
    for n, ln in zip(names, lines):
        err, ns, dig = ln.split()
        ref = oracle.decode(streams[n])
        assert err == ref.error, n
        if ref.samples is not None:
            assert int(ns) == ref.samples.size, n
            # justify is applied after the digest's bytes in both builds: compare like with like
            assert dig == _fnv(ref.samples.tobytes()), n
