"""Seeded synthetic FLAC streams (test / benchmark input; see synth/flacgen.h).

`generate(**cfg)` returns a `Stream` with the FLAC bytes, the source PCM (ground
truth, interleaved, un-justified) and the frame byte offsets. The BASELINE.json
configurations are available as `config_c2()` .. `config_c5()`.
"""
from __future__ import annotations

import ctypes
import dataclasses
import os
import subprocess
from concurrent.futures import ThreadPoolExecutor

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "libflacgen.so")

FG_VERBATIM, FG_FIXED, FG_LPC = 0, 2, 3


class _Config(ctypes.Structure):
    _fields_ = [
        ("channels", ctypes.c_int), ("bps", ctypes.c_int), ("block_size", ctypes.c_int),
        ("predictor", ctypes.c_int), ("order", ctypes.c_int), ("precision", ctypes.c_int),
        ("max_shift", ctypes.c_int), ("stereo_mode", ctypes.c_int), ("partition_order", ctypes.c_int),
        ("rice_k", ctypes.c_int), ("rice2", ctypes.c_int), ("escape_every", ctypes.c_int),
        ("wasted_bits", ctypes.c_int), ("sample_rate", ctypes.c_int), ("variable_blocking", ctypes.c_int),
        ("write_total", ctypes.c_int), ("extra_metadata", ctypes.c_int), ("verbatim_every", ctypes.c_int),
        ("silence_every", ctypes.c_int), ("rate_code_mode", ctypes.c_int),
        ("tone_amp", ctypes.c_double), ("noise_lsb", ctypes.c_double), ("stereo_corr", ctypes.c_double),
        ("fault_frame", ctypes.c_int), ("fault_kind", ctypes.c_int),
        ("n_samples", ctypes.c_uint64), ("seed", ctypes.c_uint64),
        ("dual_mono_every", ctypes.c_int), ("dual_mono_offset", ctypes.c_int), ("const_side", ctypes.c_int),
        ("plant_sync_every", ctypes.c_int), ("allow_side_overflow", ctypes.c_int),
    ]


class _Output(ctypes.Structure):
    _fields_ = [
        ("flac", ctypes.POINTER(ctypes.c_uint8)), ("flac_len", ctypes.c_size_t),
        ("pcm", ctypes.POINTER(ctypes.c_int32)), ("pcm_len", ctypes.c_uint64),
        ("frame_offsets", ctypes.POINTER(ctypes.c_uint64)), ("n_frames", ctypes.c_uint32),
        ("frames_begin", ctypes.c_size_t), ("md5", ctypes.c_uint8 * 16),
    ]


def build(force: bool = False) -> str:
    src = os.path.join(_HERE, "flacgen.cpp")
    deps = [src, os.path.join(_HERE, "flacgen.h"), os.path.join(_HERE, "..", "zflac_amd", "csrc", "md5.hpp")]
    if force or not os.path.exists(_LIB_PATH) or os.path.getmtime(_LIB_PATH) < max(os.path.getmtime(d) for d in deps):
        subprocess.check_call(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", src, "-o", _LIB_PATH])
    return _LIB_PATH


_lib = None


def _load():
    global _lib
    if _lib is None:
        build()
        lib = ctypes.CDLL(_LIB_PATH)
        lib.flacgen_default_config.argtypes = [ctypes.POINTER(_Config)]
        lib.flacgen_generate.argtypes = [ctypes.POINTER(_Config), ctypes.POINTER(_Output)]
        lib.flacgen_generate.restype = ctypes.c_int
        lib.flacgen_generate_pcm.argtypes = [ctypes.POINTER(_Config), ctypes.POINTER(ctypes.c_int32), ctypes.c_uint64,
                                             ctypes.POINTER(_Output)]
        lib.flacgen_generate_pcm.restype = ctypes.c_int
        lib.flacgen_free.argtypes = [ctypes.POINTER(_Output)]
        _lib = lib
    return _lib


@dataclasses.dataclass
class Stream:
    flac: bytes
    pcm: np.ndarray            # int32, interleaved, un-justified
    frame_offsets: np.ndarray  # uint64 byte offsets of frame headers
    frames_begin: int
    md5: bytes
    config: dict


def default_config() -> dict:
    lib = _load()
    c = _Config()
    lib.flacgen_default_config(ctypes.byref(c))
    return {name: getattr(c, name) for name, _ in _Config._fields_}


def generate(pcm: np.ndarray | None = None, **overrides) -> Stream:
    """Encode the seeded synthetic signal, or `pcm` (interleaved int32, unjustified,
    `channels` per sample; n_samples is then taken from its length)."""
    lib = _load()
    c = _Config()
    lib.flacgen_default_config(ctypes.byref(c))
    cfg = {name: getattr(c, name) for name, _ in _Config._fields_}
    for k, v in overrides.items():
        if k not in cfg:
            raise KeyError(f"unknown flacgen option {k!r}")
        setattr(c, k, v)
        cfg[k] = v
    out = _Output()
    if pcm is None:
        rc = lib.flacgen_generate(ctypes.byref(c), ctypes.byref(out))
    else:
        src = np.ascontiguousarray(pcm, dtype=np.int32)
        cfg["n_samples"] = src.size // max(1, c.channels)
        rc = lib.flacgen_generate_pcm(ctypes.byref(c), src.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), src.size,
                                      ctypes.byref(out))
    if rc != 0:
        raise ValueError(f"flacgen_generate failed ({rc}) for {cfg}")
    try:
        flac = ctypes.string_at(out.flac, out.flac_len)
        pcm = np.ctypeslib.as_array(out.pcm, shape=(max(1, out.pcm_len),))[: out.pcm_len].copy()
        offs = np.ctypeslib.as_array(out.frame_offsets, shape=(max(1, out.n_frames),))[: out.n_frames].copy()
        return Stream(flac, pcm, offs, out.frames_begin, bytes(out.md5), cfg)
    finally:
        lib.flacgen_free(ctypes.byref(out))


def generate_many(configs, workers: int | None = None):
    """Generate several streams in parallel (ctypes releases the GIL)."""
    workers = workers or min(16, os.cpu_count() or 1)
    with ThreadPoolExecutor(workers) as ex:
        return list(ex.map(lambda kw: generate(**kw), configs))


# ---- BASELINE.json configurations ---------------------------------------------
def config_c2(n_frames=64, seed=0x5EED0002):
    """C2: mono 16-bit, block 4096, fixed order 2, Rice k=4."""
    return dict(channels=1, bps=16, block_size=4096, predictor=FG_FIXED, order=2, partition_order=0,
                rice_k=4, tone_amp=0.05, noise_lsb=4.5, n_samples=4096 * n_frames, seed=seed)


def config_c3(n_frames=64, seed=0x5EED0003):
    """C3: stereo mid/side 16-bit, block 4096, LPC order 8."""
    return dict(channels=2, bps=16, block_size=4096, predictor=FG_LPC, order=8, precision=12,
                max_shift=12, stereo_mode=10, partition_order=4, rice_k=-1, tone_amp=0.25,
                noise_lsb=64.0, n_samples=4096 * n_frames, seed=seed)


def config_c4(n_frames=64, seed=0x5EED0004):
    """C4: stereo 24-bit, block 4096, LPC order 32, qlp shift 15, 4 wasted bits."""
    return dict(channels=2, bps=24, block_size=4096, predictor=FG_LPC, order=32, precision=15,
                max_shift=15, stereo_mode=1, partition_order=4, rice_k=-1, wasted_bits=4,
                tone_amp=0.25, noise_lsb=256.0, escape_every=97, n_samples=4096 * n_frames, seed=seed)


def config_c5(stream_index: int, n_frames=32):
    """C5: one of 10k independent stereo 16-bit mid/side LPC-8 streams (block 4096)."""
    return config_c3(n_frames=n_frames, seed=0x5EED0005_00000000 + stream_index)


def md5_message(pcm: np.ndarray, bps: int) -> bytes:
    """The bytes zflac's decode() hashes for `pcm` (src/zflac.zig:267-277): the container
    values before left-justify, little-endian; 17..24-bit containers hash 3 bytes each."""
    a = (bps + 7) // 8
    if a == 1:
        return pcm.astype(np.int8).tobytes()
    if a == 2:
        return pcm.astype("<i2").tobytes()
    b = pcm.astype("<i4").view(np.uint8).reshape(-1, 4)
    return np.ascontiguousarray(b[:, :3] if a == 3 else b).tobytes()


def tile_flac(st: Stream, reps: int, unknown_total: bool = False) -> bytes:
    """`st` with its frame section repeated `reps` times: a long stream for throughput
    runs without generating every frame (LPC analysis is the slow part of the writer).
    STREAMINFO's total samples and MD5 are rewritten for the repeated PCM, so decode()
    verifies the whole output. Frame numbers repeat: zflac never checks them (the coded
    number is only parsed, src/zflac.zig:354) and each header keeps its valid CRC-8.
    Fixed-blocksize streams with STREAMINFO first (the writer's layout) only."""
    import hashlib

    cfg = st.config
    if cfg.get("variable_blocking"):
        raise ValueError("tile_flac: fixed-blocksize streams only")
    d = bytearray(st.flac[: st.frames_begin])
    assert d[:4] == b"fLaC" and (d[4] & 0x7F) == 0
    o = 8
    total = 0 if unknown_total else int(st.pcm.size // cfg["channels"]) * reps
    if total >= 1 << 36:
        raise ValueError("tile_flac: total samples exceed STREAMINFO's 36 bits")
    d[o + 13] = (d[o + 13] & 0xF0) | ((total >> 32) & 15)
    for i in range(4):
        d[o + 14 + i] = (total >> (8 * (3 - i))) & 0xFF
    msg = md5_message(st.pcm, cfg["bps"])
    h = hashlib.md5()
    for _ in range(reps):
        h.update(msg)
    d[o + 18:o + 34] = h.digest()
    return bytes(d) + st.flac[st.frames_begin:] * reps


def header_crc8_index(flac: bytes, off: int) -> int:
    """Offset of the CRC-8 byte of the frame header at `off` (src/zflac.zig:343-407 layout:
    sync + 2 bytes, UTF-8-style coded number, uncommon block size / rate bytes)."""
    b2, first = flac[off + 2], flac[off + 4]
    ones = 0
    while ones < 8 and first & (0x80 >> ones):
        ones += 1
    idx = 5 + (ones - 1 if ones >= 2 else 0)
    idx += {6: 1, 7: 2}.get(b2 >> 4, 0)
    idx += {12: 1, 13: 2, 14: 2}.get(b2 & 15, 0)
    return off + idx
