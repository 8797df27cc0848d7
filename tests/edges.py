"""Parity-edge streams: zflac quirks, false frame syncs, out-of-domain values, bit-flip
mutants and the reference's expected-output convention. Each builder returns
name -> (flac bytes, expected zflac error or None, source PCM or None); None for the error
means "whatever the oracle says" (GPU-vs-oracle parity only)."""
from __future__ import annotations

import json
import os
import random

import numpy as np

import synth

from .util import GOLDEN

STEREO16 = dict(channels=2, bps=16, block_size=4096, order=8, n_samples=4096 * 6, seed=91)
STEREO32 = dict(channels=2, bps=32, order=8, precision=15, block_size=4096, n_samples=4096 * 3, tone_amp=0.2,
                noise_lsb=1e6)


def const_side_cases():
    """Constant side-channel subframes (src/zflac.zig:445-454 read `bits_per_sample`, not
    the side width). const_side=1 writes zflac's width (decodes to the source PCM),
    const_side=2 writes the RFC width (one bit more: zflac misreads it, whatever follows)."""
    out = {}
    for mode, tag in ((10, "ms"), (8, "ls"), (9, "rs")):
        for cs in (1, 2):
            for off in (0, 5, -3):
                st = synth.generate(**dict(STEREO16, stereo_mode=mode, dual_mono_every=2, dual_mono_offset=off,
                                           const_side=cs))
                exp = "OK" if cs == 1 else None
                out[f"const_side_{tag}_{'zflac' if cs == 1 else 'rfc'}_off{off}"] = (st.flac, exp, st.pcm)
    return out


def planted_sync_cases():
    """A CRC-8-valid copy of a frame header inside VERBATIM sample data (every other frame):
    the device frame indexer takes it as a candidate, the chain check rejects the stream and
    the sequential planner must still reproduce the source exactly (src/zflac.zig:340-352
    never sync-searches)."""
    base = dict(predictor=3, order=8, plant_sync_every=2, seed=93)
    cfgs = {
        "plant_mono16": dict(channels=1, bps=16, block_size=4096, n_samples=4096 * 6),
        "plant_lr16": dict(channels=2, bps=16, stereo_mode=1, block_size=4096, n_samples=4096 * 6),
        "plant_mono8": dict(channels=1, bps=8, order=3, precision=7, block_size=1152, n_samples=1152 * 8,
                            noise_lsb=1.0, tone_amp=0.3),
        "plant_lr24": dict(channels=2, bps=24, stereo_mode=1, block_size=4608, n_samples=4608 * 4, noise_lsb=256.0),
        "plant_lr16_unknown_total": dict(channels=2, bps=16, stereo_mode=1, block_size=4096, n_samples=4096 * 5,
                                         write_total=0),
        "plant_ch3_16": dict(channels=3, bps=16, block_size=2048, n_samples=2048 * 6),
    }
    out = {}
    for name, c in cfgs.items():
        st = synth.generate(**dict(base, **c))
        out[name] = (st.flac, "OK", st.pcm)
        PLANT_FRAME_OFFSETS[name] = [int(x) for x in st.frame_offsets]
    return out


PLANT_FRAME_OFFSETS: dict = {}


def out_of_domain_cases():
    """Streams on which Debug zflac traps, reported as OutOfDomain by
    the oracle's checked build and, through the device's range checks, by the HIP path."""
    mk = synth.generate
    out = {
        # side channel outside i16 (LPC-predicted, warm-up and verbatim forms) (:494,537)
        "side_overflow_ms": mk(**dict(STEREO16, stereo_mode=10, allow_side_overflow=1, stereo_corr=-1.0,
                                      tone_amp=0.9)),
        "side_overflow_ls": mk(**dict(STEREO16, stereo_mode=8, allow_side_overflow=1, stereo_corr=-1.0,
                                      tone_amp=0.9)),
        "side_overflow_rs_verbatim": mk(**dict(STEREO16, stereo_mode=9, allow_side_overflow=1, stereo_corr=-1.0,
                                               tone_amp=0.9, verbatim_every=2)),
        # decorrelated output outside i16 / i8 (:558,564,573-574)
        "decor_overflow_ms": mk(**dict(STEREO16, stereo_mode=10, fault_frame=2, fault_kind=6)),
        "decor_overflow_ls": mk(**dict(STEREO16, stereo_mode=8, fault_frame=2, fault_kind=6)),
        "decor_overflow_rs": mk(**dict(STEREO16, stereo_mode=9, fault_frame=2, fault_kind=6)),
        "decor_overflow_ms8": mk(channels=2, bps=8, stereo_mode=10, order=4, precision=7, fault_frame=1,
                                 fault_kind=6, noise_lsb=1.0, tone_amp=0.2, n_samples=4096 * 3),
        # 32-bit containers with 32-bit samples: the fast path's wrapping i32 decorrelation
        # must still see the overflow (src/zflac.zig:558,564,573-574)
        "decor_overflow_ls32": mk(**dict(STEREO32, stereo_mode=8, fault_frame=1, fault_kind=6)),
        "decor_overflow_rs32": mk(**dict(STEREO32, stereo_mode=9, fault_frame=1, fault_kind=6)),
        "decor_overflow_ms32": mk(**dict(STEREO32, stereo_mode=10, fault_frame=1, fault_kind=6)),
        # large coefficients: LPC sums overflow the InterType (:527-532)
        "lpc_sum_overflow16": mk(channels=2, bps=16, stereo_mode=1, fault_frame=1, fault_kind=8, order=32,
                                 precision=15, tone_amp=0.9, noise_lsb=2000.0, n_samples=4096 * 3),
        "lpc_sum_overflow8": mk(channels=1, bps=8, fault_frame=1, fault_kind=8, order=8, precision=7,
                                tone_amp=0.9, noise_lsb=8.0, n_samples=4096 * 3),
    }
    res = {k: (v.flac, "OutOfDomain", None) for k, v in out.items()}
    # the same large coefficients on a quiet signal: no sum overflows, zflac decodes it
    for name, cfg in {
        "lpc_large_coefs_quiet16": dict(channels=2, bps=16, stereo_mode=1, fault_frame=1, fault_kind=7, order=32,
                                        precision=15, tone_amp=0.0005, noise_lsb=1.0, n_samples=4096 * 3),
        "lpc_large_coefs_quiet8": dict(channels=1, bps=8, fault_frame=1, fault_kind=7, order=8, precision=7,
                                       tone_amp=0.01, noise_lsb=0.5, n_samples=4096 * 3),
        "lpc_large_coefs_loud_ok16": dict(channels=2, bps=16, stereo_mode=1, fault_frame=1, fault_kind=8,
                                          order=32, precision=15, n_samples=4096 * 3),
    }.items():
        st = mk(**cfg)
        res[name] = (st.flac, "OK", st.pcm)
    return res


def incorrect_metadata_length_case(flac: bytes, frames_begin: int) -> bytes:
    """faulty/11 (tests/std_faulty.zig:59-61 expects InvalidMetadataHeader): a PADDING
    block whose length field says 10 while 4 bytes follow; skipping 10 bytes lands inside
    the first frame header, whose third byte reads as a reserved block type (:243-248)."""
    assert flac[:4] == b"fLaC" and (flac[4] & 0x7F) == 0
    si = bytearray(flac[4:8 + 34])
    si[0] &= 0x7F  # STREAMINFO is no longer the last block
    pad_bad = bytes([0x01, 0, 0, 10]) + bytes(4)
    pad_last = bytes([0x81, 0, 0, 0])
    return b"fLaC" + bytes(si) + pad_bad + pad_last + flac[frames_begin:]


def bad_crc8_case(frames: int = 48, seed: int = 95, write_total: int = 1):
    """Every frame header's CRC-8 byte flipped. zflac never checks it (:407-410), so the
    stream decodes to the source PCM; the device indexer drops every header and the
    sequential planner reaches each frame through its batched probes."""
    st = synth.generate(**dict(STEREO16, stereo_mode=10, n_samples=4096 * frames, seed=seed,
                               write_total=write_total))
    b = bytearray(st.flac)
    for off in st.frame_offsets:
        b[synth.header_crc8_index(st.flac, int(off))] ^= 0x5A
    return bytes(b), st.pcm


def fixture_mutants(n_per_file: int = 100, seed: int = 0x0F1A):
    """Seeded bit-flip mutants of the committed C3 / C4 fixtures. Flips land in the frame
    section (90 %) or in the metadata outside the 36-bit total-samples field (whose huge
    values would only test the allocators of both sides)."""
    rng = random.Random(seed)
    out = {}
    for fx in ("c3_ms16_lpc8.flac", "c4_24bit_lpc32_wasted.flac"):
        data = open(os.path.join(GOLDEN, fx), "rb").read()
        fb = 42  # 'fLaC' + STREAMINFO header + body: frames start here in the fixtures
        for m in range(n_per_file):
            b = bytearray(data)
            for _ in range(rng.choice((1, 1, 1, 2, 3))):
                if rng.random() < 0.9:
                    pos = rng.randrange(fb, len(b))
                else:
                    pos = rng.choice([p for p in range(4, fb) if not 21 <= p <= 25])
                b[pos] ^= 1 << rng.randrange(8)
            out[f"{fx.split('.')[0]}_m{m:03d}"] = (bytes(b), None, None)
    return out


def load_raw_slices():
    """tests/golden/raw (tools/make_raw_fixtures.py): slices of the reference's expected
    outputs. Returns (meta, zflac-convention samples as the decoder returns them)."""
    d = os.path.join(GOLDEN, "raw")
    with open(os.path.join(d, "manifest.json")) as f:
        man = json.load(f)
    out = []
    for s in man["slices"]:
        raw = open(os.path.join(d, s["file"]), "rb").read()
        if s["container"] == "s8u":  # tests/std_subset.zig:24-30: expected[i] -% 128 as i8
            v = (np.frombuffer(raw, np.uint8).astype(np.int16) - 128).astype(np.int8)
        else:
            v = np.frombuffer(raw, {"s16": "<i2", "s32": "<i4"}[s["container"]]).copy()
        out.append((s, v))
    return out


def unjustify(v: np.ndarray, bps: int) -> np.ndarray:
    """Undo zflac's left-justify (src/zflac.zig:287-306) to get the coded PCM."""
    js = 16 - bps if 9 <= bps <= 15 else 32 - bps if 17 <= bps <= 31 else 0
    return (v.astype(np.int64) >> js).astype(np.int32)
