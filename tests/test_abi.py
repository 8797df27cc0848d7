"""CPU tests of the C-ABI boundary: the library loads, exports every symbol the header
declares, error codes/names are the zflac set, and without a GPU it fails loudly."""
import ctypes
import os
import re

import pytest

import zflac_amd
from zflac_amd import _lib, errors

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _header_functions():
    text = open(os.path.join(ROOT, "include", "zflac_hip.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(zflac_hip_\w+)\s*\(", text)))


def test_library_exports_every_header_symbol():
    L = _lib.load()
    funcs = _header_functions()
    assert len(funcs) >= 14
    for name in funcs:
        assert hasattr(L, name), name
        assert name in _lib.SIGNATURES, f"{name} lacks a ctypes signature"


def test_error_names_match_zflac_set():
    L = _lib.load()
    import oracle

    for code, name in errors.NAMES.items():
        assert L.zflac_hip_error_name(code).decode() == name
        assert oracle.ERROR_NAMES[code] == name
    assert issubclass(errors.InvalidChecksum, errors.ZflacError)
    assert errors.error_class(5) is errors.InvalidChecksum


def test_version_and_device_count():
    L = _lib.load()
    assert b"gfx950" in L.zflac_hip_version()
    assert zflac_amd.device_count() >= 0


def test_no_gpu_fails_loudly():
    if zflac_amd.device_count() > 0:
        pytest.skip("a GPU is visible; this checks the no-GPU behaviour")
    with pytest.raises(errors.DeviceError):
        zflac_amd.decode(b"fLaC\x80\x00\x00\x22" + bytes(34))
    h = ctypes.c_void_p()
    rc = _lib.load().zflac_hip_batch_create(None, 0, 0, 0, ctypes.byref(h))
    assert rc == 13


def test_invalid_arguments():
    L = _lib.load()
    assert L.zflac_hip_batch_run(None) == 14
    assert L.zflac_hip_batch_submit(None) == 14
    assert L.zflac_hip_batch_wait(None) == 14
    assert L.zflac_hip_batch_ready(None) == -14
    assert L.zflac_hip_batch_info(None, 0, None) == 14
    assert L.zflac_hip_batch_read(None, 0, None, 0, 0) == 14
    assert L.zflac_hip_batch_size(None) == 0
    L.zflac_hip_batch_destroy(None)
    L.zflac_hip_close(None)


def test_kernels_compiled_for_gfx950():
    """The shared library embeds a gfx950 code object (hipcc --offload-arch=gfx950)."""
    blob = open(_lib.lib_path, "rb").read()
    assert b"gfx950" in blob


def test_abi_version_and_timings_struct():
    """ABI revision 5; zflac_hip_batch_timings_ex takes the caller's struct size, and the
    legacy entry point writes only the first-version layout (scan_ms .. md5_ms)."""
    L = _lib.load()
    assert L.zflac_hip_abi_version() == 5
    t = _lib.zflac_timings()
    assert ctypes.sizeof(t) == 136
    assert _lib.zflac_timings.rest_launches.offset == 128
    assert _lib.zflac_timings.sequential_streams.offset == 132
    assert _lib.zflac_timings.plan_ms.offset == 80  # ZFLAC_TIMINGS_V1_SIZE
    assert L.zflac_hip_batch_timings_ex(None, ctypes.byref(t), ctypes.sizeof(t)) == 14
    assert L.zflac_hip_batch_timings(None, ctypes.byref(t)) == 14


def test_build_id_names_the_sources():
    """The library embeds the fingerprint of the sources it was built from (build.py), and
    the loaded library reports the same string the file holds."""
    from zflac_amd import build

    L = _lib.load()
    bid = L.zflac_hip_build_id().decode()
    assert re.fullmatch(r"src=[0-9a-f]{64}", bid)
    assert build.lib_build_id(_lib.lib_path) == bid
    if _lib.lib_path == build.LIB and not build.needs_build():
        assert bid == "src=" + build.source_fingerprint()
