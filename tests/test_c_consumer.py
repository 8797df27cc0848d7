"""The C twin of the Zig shim (tests/c/abi_consumer.c, mirroring zig/zflac_hip.zig) against
libzflac_hip.so: built with `gcc -std=c11 -Wall -Wextra -Werror -pedantic` from the header
alone, its struct-layout static_asserts are the layout a Zig `extern struct` binds, its
error switch is the shim's, and on the GPU it runs the shim's two-phase contract
(open -> aligned_alloc(32) -> read -> close) on the reference's KATs and the fixtures."""
import hashlib
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from .util import GOLDEN, load_fixture_manifest, load_kats

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from __graft_entry__ import build_c_consumer  # noqa: E402

ZIG = os.path.join(ROOT, "zig", "zflac_hip.zig")


@pytest.fixture(scope="module")
def consumer():
    return build_c_consumer()


def _run_all(exe, *args):
    p = subprocess.run([exe, *args], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr + p.stdout
    return [json.loads(x) for x in p.stdout.strip().splitlines() if x.startswith("{")]


def _run(exe, *args):
    return _run_all(exe, *args)[-1]


def test_builds_with_werror_and_names_match(consumer):
    """Compiles warning-free as C11 (static_asserts included) and the shim's error switch
    names every ZFLAC_E_* code as the library does."""
    r = _run(consumer, "names")
    assert r == {"names": True, "abi": 5}


def test_zig_shim_is_the_mirrored_switch():
    """zig/zflac_hip.zig's `check` has one arm per ZFLAC_E_* code of the header (the same set
    the C twin switches on), casts every Samples arm through [*]align(32) T as
    src/zflac.zig:334 does, and asserts the same zflac_info offsets as the C twin."""
    import re

    zig = open(ZIG).read()
    hdr = open(os.path.join(ROOT, "include", "zflac_hip.h")).read()
    codes = re.findall(r"#define (ZFLAC_E_\w+) \d+", hdr)
    assert len(codes) == 16
    for code in codes + ["ZFLAC_OK"]:
        assert f"c.{code} =>" in zig, code
    for t in ("i8", "i16", "i32"):
        assert f"@as([*]align(32) {t}, @alignCast(@ptrCast(samples_backing.ptr)))" in zig
    assert "allocWithOptions(u8, @intCast(info.samples_bytes), 32, null)" in zig
    c_src = open(os.path.join(ROOT, "tests", "c", "abi_consumer.c")).read()
    for field, off in (("channels", 0), ("bits_per_sample", 1), ("sample_kind", 2), ("sample_rate", 4),
                       ("n_samples", 8), ("samples_bytes", 16)):
        assert f'@offsetOf(c.zflac_info, "{field}") == {off}' in zig
        assert f"offsetof(zflac_info, {field}) == {off}" in c_src


def test_no_gpu_is_device_error(consumer, tmp_path):
    import zflac_amd

    if zflac_amd.device_count() > 0:
        pytest.skip("a GPU is visible; this checks the no-GPU behaviour")
    src = tmp_path / "k.flac"
    src.write_bytes(bytes.fromhex(load_kats()[0]["flac_hex"]))
    r = _run(consumer, "decode", str(src), str(tmp_path / "k.raw"))
    assert r["rc"] == 13 and r["error"] == "DeviceError"


@pytest.mark.gpu
@pytest.mark.parametrize("kat", load_kats(), ids=lambda k: k["name"])
def test_c_consumer_kats_gpu(gpu_ready, consumer, tmp_path, kat):
    src, out = tmp_path / "k.flac", tmp_path / "k.raw"
    src.write_bytes(bytes.fromhex(kat["flac_hex"]))
    r = _run(consumer, "decode", str(src), str(out))
    assert r["error"] == "OK" and r["library_name"] == "OK"
    assert r["channels"] == int(kat["channels"])
    dt = {"s8": np.int8, "s16": np.int16, "s32": np.int32}[kat["sample_kind"]]
    assert r["sample_kind"] == {"s8": 0, "s16": 1, "s32": 2}[kat["sample_kind"]]
    got = np.frombuffer(out.read_bytes(), dtype=dt)
    assert got.tolist() == kat["expected"]


@pytest.mark.gpu
@pytest.mark.parametrize("fx", load_fixture_manifest()["fixtures"], ids=lambda f: f["file"])
def test_c_consumer_fixtures_gpu(gpu_ready, consumer, tmp_path, fx):
    """Every committed fixture (C2, C3, C4 24-bit LPC-32, ...) through the C consumer: the
    sample bytes in the 32-byte aligned caller buffer hash to the manifest's digest."""
    out = tmp_path / "f.raw"
    r = _run(consumer, "decode", os.path.join(GOLDEN, fx["file"]), str(out))
    assert r["error"] == fx["error"]
    if fx["error"] == "OK":
        assert r["n_samples"] == fx["n_samples"] and r["channels"] == fx["channels"]
        assert hashlib.sha256(out.read_bytes()).hexdigest() == fx["samples_sha256"]


@pytest.mark.gpu
def test_c_consumer_errors_gpu(gpu_ready, consumer, tmp_path):
    """The malformed-stream catalogue: the C consumer's (= the shim's) error name is the one
    the reference's tests expect, which is also the oracle's."""
    import oracle

    from . import malformed

    cases = malformed.cases()
    assert len(cases) > 10
    args = []
    for i, (name, (data, _)) in enumerate(cases.items()):
        (tmp_path / f"m{i}.flac").write_bytes(data)
        args += [str(tmp_path / f"m{i}.flac"), str(tmp_path / f"m{i}.raw")]
    rs = _run_all(consumer, "decode", *args)  # one process for the whole catalogue
    assert len(rs) == len(cases)
    for r, (name, (data, want)) in zip(rs, cases.items()):
        assert r["error"] == want == oracle.decode(data).error, name
        assert r["error"] == r["library_name"], name
