"""TEST INFRASTRUCTURE ONLY: ctypes access to the C restatement of zflac decode().

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
module; the product (zflac_amd / libzflac_hip.so) never does. See zflac_oracle.h.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_BUILD = os.path.join(_HERE, "_build")
_LIBS = {"checked": os.path.join(_BUILD, "libzflac_oracle.so"),
         "fast": os.path.join(_BUILD, "libzflac_oracle_fast.so")}

ERROR_NAMES = {
    0: "OK", 1: "InvalidSignature", 2: "InvalidMetadataHeader", 3: "MissingStreaminfo", 4: "Unimplemented",
    5: "InvalidChecksum", 6: "InvalidFrameHeader", 7: "InconsistentParameters", 8: "InvalidCodedNumber",
    9: "InvalidSubframeHeader", 10: "InvalidResidualCodingMethod", 11: "EndOfStream", 12: "OutOfMemory",
    13: "DeviceError", 14: "InvalidArgument", 15: "OutOfDomain",
    16: "FrameCrcMismatch",  # never returned here: zflac ignores the CRC-16 trailer (src/zflac.zig:548-551)
}
_KIND_DTYPE = {0: np.int8, 1: np.int16, 2: np.int32}


class _Result(ctypes.Structure):
    _fields_ = [("err", ctypes.c_int), ("channels", ctypes.c_uint8), ("bits_per_sample", ctypes.c_uint8),
                ("sample_kind", ctypes.c_uint8), ("_pad", ctypes.c_uint8), ("sample_rate", ctypes.c_uint32),
                ("n_samples", ctypes.c_uint64), ("samples", ctypes.c_void_p)]


def build(force: bool = False) -> None:
    src = [os.path.join(_HERE, "zflac_oracle.c"), os.path.join(_HERE, "zflac_oracle.h")]
    newest = max(os.path.getmtime(s) for s in src)
    if force or any(not os.path.exists(p) or os.path.getmtime(p) < newest for p in _LIBS.values()):
        subprocess.check_call(["sh", os.path.join(_HERE, "build.sh")])


_loaded = {}


def _lib(flavor="checked"):
    if flavor not in _loaded:
        build()
        lib = ctypes.CDLL(_LIBS[flavor])
        lib.zfo_decode.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(_Result)]
        lib.zfo_decode.restype = ctypes.c_int
        lib.zfo_decode_ex.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int, ctypes.POINTER(_Result)]
        lib.zfo_decode_ex.restype = ctypes.c_int
        lib.zfo_free.argtypes = [ctypes.POINTER(_Result)]
        lib.zfo_md5.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p]
        lib.zfo_error_name.restype = ctypes.c_char_p
        _loaded[flavor] = lib
    return _loaded[flavor]


class OracleResult:
    def __init__(self, err, channels=0, sample_rate=0, bits_per_sample=0, samples=None):
        self.err = err
        self.error = ERROR_NAMES.get(err, f"E{err}")
        self.channels = channels
        self.sample_rate = sample_rate
        self.bits_per_sample = bits_per_sample
        self.samples = samples


def decode(data: bytes, flavor: str = "checked") -> OracleResult:
    lib = _lib(flavor)
    r = _Result()
    err = lib.zfo_decode(data, len(data), ctypes.byref(r))
    try:
        if err and not r.samples:
            return OracleResult(err)
        # OK, or InvalidChecksum with the decoded (justified) samples kept for comparison
        dt = np.dtype(_KIND_DTYPE[r.sample_kind])
        nbytes = r.n_samples * dt.itemsize
        arr = np.frombuffer(ctypes.string_at(r.samples, nbytes), dtype=dt).copy() if nbytes else np.zeros(0, dt)
        return OracleResult(err, r.channels, r.sample_rate, r.bits_per_sample, arr)
    finally:
        lib.zfo_free(ctypes.byref(r))


def decode_count_only(data: bytes, flavor: str = "fast", md5: bool = True) -> tuple[int, int]:
    """Decode and return (err, n_samples) without copying samples (for timing); md5=False
    skips the STREAMINFO MD5 (the decode alone)."""
    lib = _lib(flavor)
    r = _Result()
    err = lib.zfo_decode_ex(data, len(data), 0 if md5 else 1, ctypes.byref(r))
    n = r.n_samples
    lib.zfo_free(ctypes.byref(r))
    return err, n


def md5(data: bytes) -> bytes:
    out = ctypes.create_string_buffer(16)
    _lib().zfo_md5(data, len(data), out)
    return out.raw
