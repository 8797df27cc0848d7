"""decode() / DecodedFLAC mirror of zflac's public API, over libzflac_hip.so.

zflac (src/zflac.zig:216-217):  pub fn decode(allocator, reader: anytype) !DecodedFLAC
Here: decode(reader) -> DecodedFLAC, raising zflac-named errors.
"""
from __future__ import annotations

import ctypes
import dataclasses

import numpy as np

from . import _lib, errors

_DTYPES = {0: np.int8, 1: np.int16, 2: np.int32}
_TAGS = {0: "s8", 1: "s16", 2: "s32"}


@dataclasses.dataclass
class Samples:
    """zflac's `Samples = union(enum) { s8, s16, s32 }` (src/zflac.zig:12-16)."""

    tag: str
    values: np.ndarray

    @property
    def s8(self) -> np.ndarray:
        return self._arm("s8")

    @property
    def s16(self) -> np.ndarray:
        return self._arm("s16")

    @property
    def s32(self) -> np.ndarray:
        return self._arm("s32")

    def _arm(self, tag):
        if self.tag != tag:
            raise AttributeError(f"inactive union field {tag!r} (active: {self.tag!r})")
        return self.values


@dataclasses.dataclass
class DecodedFLAC:
    """zflac.DecodedFLAC (src/zflac.zig:18-28)."""

    channels: int
    sample_rate: int
    bits_per_sample: int
    samples: Samples

    def deinit(self, allocator=None) -> None:  # parity with DecodedFLAC.deinit
        self.samples = Samples(self.samples.tag, self.samples.values[:0])


def _read_all(reader) -> bytes:
    if isinstance(reader, (bytes, bytearray, memoryview)):
        return bytes(reader)
    if hasattr(reader, "read"):
        return reader.read()
    raise TypeError("decode() expects bytes or a reader with .read()")


def device_count() -> int:
    return _lib.load().zflac_hip_device_count()


def build_id() -> str:
    """"src=<fingerprint>" of the loaded library's sources (zflac_hip_build_id)."""
    return _lib.load().zflac_hip_build_id().decode()


def _aligned_empty(nbytes: int, dtype) -> np.ndarray:
    """32-byte aligned buffer, as zflac allocates its samples (src/zflac.zig:331)."""
    raw = np.empty(nbytes + 32, dtype=np.uint8)
    off = (-raw.ctypes.data) % 32
    return raw[off:off + nbytes].view(dtype)


def decode(reader, device: int = 0, timings: dict | None = None, check_crc16: bool = False) -> DecodedFLAC:
    """Decode one FLAC stream on `device`; raises zflac-named errors (errors.*).
    `timings` (a dict) receives the library's host wall-clock breakdown of the call.
    `check_crc16` also checks every frame's CRC-16 trailer on the device (FrameCrcMismatch);
    zflac itself ignores it (src/zflac.zig:548-551)."""
    data = _read_all(reader)
    L = _lib.load()
    handle = ctypes.c_void_p()
    info = _lib.zflac_info()
    flags = _lib.FLAG_CHECK_CRC16 if check_crc16 else 0
    rc = L.zflac_hip_open_ex(data, len(data), device, flags, ctypes.byref(handle), ctypes.byref(info))
    try:
        errors.check(rc)
        out = _aligned_empty(info.samples_bytes, _DTYPES[info.sample_kind])
        rc = L.zflac_hip_read(handle, out.ctypes.data_as(ctypes.c_void_p) if info.samples_bytes else None,
                              info.samples_bytes)
        errors.check(rc)
        if timings is not None:
            t = _lib.zflac_timings()
            L.zflac_hip_batch_timings_ex(handle, ctypes.byref(t), ctypes.sizeof(t))
            timings.update({name: getattr(t, name) for name, _ in _lib.zflac_timings._fields_})
        return DecodedFLAC(info.channels, info.sample_rate, info.bits_per_sample,
                           Samples(_TAGS[info.sample_kind], out))
    finally:
        if handle:
            L.zflac_hip_close(handle)


class Batch:
    """A batch of independent streams resident in HBM (C5-style shard).

    create -> run() (device-resident decode, repeatable) -> info(i) / read(i).
    """

    def __init__(self, streams, device: int = 0, timing: bool = False, force_slow: bool = False,
                 device_md5: bool = False, check_crc16: bool = False, walk: str | None = None):
        self._L = _lib.load()
        self._bufs = [bytes(s) for s in streams]
        arr = (_lib.zflac_stream * len(self._bufs))()
        self._keep = []
        for i, b in enumerate(self._bufs):
            cb = ctypes.create_string_buffer(b, len(b))
            self._keep.append(cb)
            arr[i].data = ctypes.cast(cb, ctypes.c_void_p)
            arr[i].len = len(b)
        flags = ((_lib.FLAG_TIMING if timing else 0) | (_lib.FLAG_FORCE_SLOW if force_slow else 0)
                 | (_lib.FLAG_DEVICE_MD5 if device_md5 else 0) | (_lib.FLAG_CHECK_CRC16 if check_crc16 else 0)
                 | {None: 0, "lane": _lib.FLAG_WALK_LANE, "wave": _lib.FLAG_WALK_WAVE}[walk])
        self._h = ctypes.c_void_p()
        rc = self._L.zflac_hip_batch_create(arr, len(self._bufs), device, flags, ctypes.byref(self._h))
        self._keep = None  # the library copied the bytes to HBM
        errors.check(rc, "batch_create")

    def __len__(self):
        return len(self._bufs)

    def run(self) -> None:
        errors.check(self._L.zflac_hip_batch_run(self._h), "batch_run")

    def submit(self) -> None:
        """Enqueue a run and return (zflac_hip_batch_submit); results after wait()."""
        errors.check(self._L.zflac_hip_batch_submit(self._h), "batch_submit")

    def wait(self) -> None:
        errors.check(self._L.zflac_hip_batch_wait(self._h), "batch_wait")

    def ready(self) -> bool:
        """The submitted run's device work has finished (zflac_hip_batch_ready, non-blocking)."""
        rc = self._L.zflac_hip_batch_ready(self._h)
        if rc < 0:
            errors.check(-rc, "batch_ready")
        return rc == 1

    def info(self, i: int):
        inf = _lib.zflac_info()
        rc = self._L.zflac_hip_batch_info(self._h, i, ctypes.byref(inf))
        return rc, inf

    def error_name(self, i: int) -> str:
        return errors.NAMES.get(self.info(i)[0], "Unknown")

    def read(self, i: int, verify_md5: bool = True) -> DecodedFLAC:
        rc, inf = self.info(i)
        errors.check(rc)
        out = _aligned_empty(inf.samples_bytes, _DTYPES[inf.sample_kind])
        rc = self._L.zflac_hip_batch_read(self._h, i, out.ctypes.data_as(ctypes.c_void_p) if inf.samples_bytes
                                          else None, inf.samples_bytes, 1 if verify_md5 else 0)
        errors.check(rc)
        return DecodedFLAC(inf.channels, inf.sample_rate, inf.bits_per_sample, Samples(_TAGS[inf.sample_kind], out))

    def md5(self, i: int):
        """Device MD5 digest of stream i (batches created with device_md5=True), else None."""
        buf = ctypes.create_string_buffer(16)
        rc = self._L.zflac_hip_batch_md5(self._h, i, buf)
        return None if rc else buf.raw

    def timings(self):
        t = _lib.zflac_timings()
        rc = self._L.zflac_hip_batch_timings_ex(self._h, ctypes.byref(t), ctypes.sizeof(t))
        return None if rc else t

    def device_samples(self, i: int) -> int:
        return self._L.zflac_hip_batch_device_samples(self._h, i) or 0

    def close(self):
        if getattr(self, "_h", None):
            self._L.zflac_hip_batch_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass


def decode_many(streams, device: int = 0, verify_md5: bool = True, device_md5: bool = True):
    """Decode independent streams in one batch; returns DecodedFLAC or exception per stream.

    With device_md5 the STREAMINFO MD5s are checked by k_md5 on the GPU (one lane per
    stream) instead of on the host after the copy back."""
    b = Batch(streams, device, device_md5=device_md5 and verify_md5)
    try:
        b.run()
        out = []
        for i in range(len(b)):
            try:
                out.append(b.read(i, verify_md5))
            except errors.ZflacError as e:
                out.append(e)
        return out
    finally:
        b.close()
