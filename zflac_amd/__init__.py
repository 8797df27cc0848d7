"""zflac_amd: MI355X-native FLAC decode path behind zflac's decode() interface.

Python mirror of Senryoku/zflac's public API (src/zflac.zig:12-28, :216-310):

    decoded = zflac_amd.decode(reader)      # reader: bytes-like or object with .read()
    decoded.channels, decoded.sample_rate, decoded.bits_per_sample
    decoded.samples                          # Samples union: .s8 / .s16 / .s32 numpy view
    decoded.deinit()                         # frees nothing extra; kept for API parity

Errors are raised as `ZflacError` subclasses named exactly like zflac's error set
(`zflac_amd.errors.InvalidChecksum`, ...). All decode work runs in the HIP kernels of
libzflac_hip.so (see include/zflac_hip.h); there is no CPU decode path, and without a
GPU every call raises `DeviceError`.
"""
from __future__ import annotations

from . import errors
from ._lib import lib_path
from .api import Batch, DecodedFLAC, Samples, build_id, decode, decode_many, device_count

__all__ = ["decode", "decode_many", "DecodedFLAC", "Samples", "Batch", "errors", "device_count", "build_id", "lib_path"]
