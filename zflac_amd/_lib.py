"""ctypes binding of libzflac_hip.so (include/zflac_hip.h).

The library is built in-tree by zflac_amd/build.py (hipcc --offload-arch=gfx950). If it
is missing this module raises ImportError-like RuntimeError: there is no fallback.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# ZFLAC_HIP_LIB selects another build of the same library (timing experiments)
lib_path = os.environ.get("ZFLAC_HIP_LIB") or os.path.join(_HERE, "libzflac_hip.so")


class zflac_info(ctypes.Structure):
    _fields_ = [("channels", ctypes.c_uint8), ("bits_per_sample", ctypes.c_uint8),
                ("sample_kind", ctypes.c_uint8), ("reserved", ctypes.c_uint8),
                ("sample_rate", ctypes.c_uint32), ("n_samples", ctypes.c_uint64),
                ("samples_bytes", ctypes.c_uint64)]


class zflac_stream(ctypes.Structure):
    _fields_ = [("data", ctypes.c_void_p), ("len", ctypes.c_size_t)]


class zflac_timings(ctypes.Structure):
    _fields_ = [("scan_ms", ctypes.c_double), ("decode_ms", ctypes.c_double), ("verify_ms", ctypes.c_double),
                ("total_ms", ctypes.c_double), ("frames", ctypes.c_uint64), ("input_bytes", ctypes.c_uint64),
                ("output_bytes", ctypes.c_uint64), ("samples", ctypes.c_uint64), ("walk_ms", ctypes.c_double),
                ("md5_ms", ctypes.c_double), ("plan_ms", ctypes.c_double), ("upload_ms", ctypes.c_double),
                ("run_wall_ms", ctypes.c_double), ("read_ms", ctypes.c_double), ("host_md5_ms", ctypes.c_double),
                ("crc16_ms", ctypes.c_double), ("rest_launches", ctypes.c_uint32), ("sequential_streams", ctypes.c_uint32)]


# every symbol include/zflac_hip.h declares, with (restype, argtypes)
_P = ctypes.c_void_p
SIGNATURES = {
    "zflac_hip_open": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int, ctypes.POINTER(_P),
                                      ctypes.POINTER(zflac_info)]),
    "zflac_hip_open_ex": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int,
                                         ctypes.POINTER(_P), ctypes.POINTER(zflac_info)]),
    "zflac_hip_read": (ctypes.c_int, [_P, _P, ctypes.c_size_t]),
    "zflac_hip_close": (None, [_P]),
    "zflac_hip_batch_create": (ctypes.c_int, [ctypes.POINTER(zflac_stream), ctypes.c_size_t, ctypes.c_int,
                                              ctypes.c_int, ctypes.POINTER(_P)]),
    "zflac_hip_batch_run": (ctypes.c_int, [_P]),
    "zflac_hip_batch_submit": (ctypes.c_int, [_P]),
    "zflac_hip_batch_wait": (ctypes.c_int, [_P]),
    "zflac_hip_batch_ready": (ctypes.c_int, [_P]),
    "zflac_hip_batch_info": (ctypes.c_int, [_P, ctypes.c_size_t, ctypes.POINTER(zflac_info)]),
    "zflac_hip_batch_read": (ctypes.c_int, [_P, ctypes.c_size_t, _P, ctypes.c_size_t, ctypes.c_int]),
    "zflac_hip_batch_md5": (ctypes.c_int, [_P, ctypes.c_size_t, ctypes.c_char_p]),
    "zflac_hip_batch_device_samples": (_P, [_P, ctypes.c_size_t]),
    "zflac_hip_batch_timings": (ctypes.c_int, [_P, ctypes.POINTER(zflac_timings)]),
    "zflac_hip_batch_timings_ex": (ctypes.c_int, [_P, ctypes.POINTER(zflac_timings), ctypes.c_size_t]),
    "zflac_hip_abi_version": (ctypes.c_int, []),
    "zflac_hip_batch_size": (ctypes.c_size_t, [_P]),
    "zflac_hip_batch_destroy": (None, [_P]),
    "zflac_hip_error_name": (ctypes.c_char_p, [ctypes.c_int]),
    "zflac_hip_device_count": (ctypes.c_int, []),
    "zflac_hip_version": (ctypes.c_char_p, []),
    "zflac_hip_build_id": (ctypes.c_char_p, []),
}

FLAG_TIMING = 1
FLAG_FORCE_SLOW = 2
FLAG_DEVICE_MD5 = 4
FLAG_CHECK_CRC16 = 8  # beyond zflac (src/zflac.zig:548-551 ignores the trailer)
FLAG_WALK_LANE = 16
FLAG_WALK_WAVE = 32

_lib = None


def load():
    """Load libzflac_hip.so (building it first if sources are newer)."""
    global _lib
    if _lib is None:
        if not os.path.exists(lib_path):
            try:
                from . import build as _build

                _build.build()
            except Exception as e:  # noqa: BLE001
                raise RuntimeError(f"libzflac_hip.so is missing and could not be built: {e}") from e
        lib = ctypes.CDLL(lib_path)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
    return _lib
