"""Shared helpers for the test suite: expected outputs and malformed-stream builders."""
from __future__ import annotations

import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def justified(pcm: np.ndarray, bps: int) -> np.ndarray:
    """zflac's output convention: left-justify after MD5 (src/zflac.zig:287-306)."""
    p = pcm.astype(np.int64)
    if 9 <= bps <= 15:
        p = p << (16 - bps)
    elif 17 <= bps <= 31:
        p = p << (32 - bps)
    return p


def container_dtype(bps: int):
    a = (bps + 7) // 8 * 8
    return {8: np.int8, 16: np.int16, 24: np.int32, 32: np.int32}[a]


def expected_samples(stream) -> np.ndarray:
    bps = stream.config["bps"]
    return justified(stream.pcm, bps).astype(container_dtype(bps))


def load_kats():
    with open(os.path.join(GOLDEN, "basic_kat.json")) as f:
        return json.load(f)["kats"]


def load_fixture_manifest():
    with open(os.path.join(GOLDEN, "fixtures.json")) as f:
        return json.load(f)


def patch(data: bytes, offset: int, value: int) -> bytes:
    b = bytearray(data)
    b[offset] = value
    return bytes(b)


def streaminfo_offset(data: bytes) -> int:
    """Byte offset of the STREAMINFO body (the generator always writes it first)."""
    assert data[:4] == b"fLaC" and (data[4] & 0x7F) == 0
    return 8


# Configurations exercised by parity tests (name -> flacgen overrides). Small sizes:
# the checked oracle decodes each in well under a second.
PARITY_CONFIGS = {
    "c2_mono16_fixed2_k4": dict(channels=1, bps=16, block_size=4096, predictor=2, order=2, partition_order=0,
                                rice_k=4, tone_amp=0.05, noise_lsb=4.5, n_samples=4096 * 6 + 100),
    "c3_ms16_lpc8": dict(channels=2, bps=16, block_size=4096, predictor=3, order=8, precision=12, max_shift=12,
                         stereo_mode=10, partition_order=4, n_samples=4096 * 6),
    "c4_24bit_lpc32_wasted": dict(channels=2, bps=24, block_size=4096, predictor=3, order=32, precision=15,
                                  max_shift=15, stereo_mode=1, partition_order=4, wasted_bits=4, noise_lsb=256.0,
                                  escape_every=97, n_samples=4096 * 4),
    "ls16_fixed_mix": dict(channels=2, bps=16, stereo_mode=8, predictor=2, order=3, block_size=1152,
                           n_samples=1152 * 7 + 5, verbatim_every=5),
    "rs16_lpc5": dict(channels=2, bps=16, stereo_mode=9, order=5, block_size=2304, n_samples=2304 * 5),
    "auto_stereo_lpc12": dict(channels=2, bps=16, stereo_mode=-1, order=12, precision=14, block_size=4608,
                              n_samples=4608 * 3 + 17, partition_order=3),
    "mono8_lpc3": dict(channels=1, bps=8, order=3, precision=7, block_size=576, n_samples=576 * 9 + 3),
    # 8-bit containers on the packed fast path (bytes four to a dword, 16-byte stores; stereo
    # interleaved after permlane32_swap), 4096-sample frames and a short last frame
    "mono8_lpc4_packed": dict(channels=1, bps=8, order=4, precision=7, block_size=4096, n_samples=4096 * 3 + 21,
                              noise_lsb=1.0, tone_amp=0.3, wasted_bits=1),
    "stereo8_ms_packed": dict(channels=2, bps=8, stereo_mode=10, order=4, precision=7, block_size=4096,
                              n_samples=4096 * 3 + 5, noise_lsb=1.0, tone_amp=0.3),
    "stereo8_ls_packed": dict(channels=2, bps=8, stereo_mode=8, order=6, precision=7, block_size=2048,
                              n_samples=2048 * 4, noise_lsb=2.0, tone_amp=0.25),
    "stereo12_ms": dict(channels=2, bps=12, stereo_mode=10, order=4, block_size=1024, n_samples=1024 * 6),
    # orders 9..12: the MB = 12 history bucket (16 history slots, 12 coefficients) of every container
    "mono8_lpc10": dict(channels=1, bps=8, order=10, precision=7, block_size=2048, n_samples=2048 * 3 + 9,
                        noise_lsb=1.0, tone_amp=0.3),
    "mono16_lpc9": dict(channels=1, bps=16, order=9, precision=13, block_size=4096, n_samples=4096 * 2 + 77),
    "stereo24_ls_lpc11": dict(channels=2, bps=24, stereo_mode=8, order=11, precision=14, block_size=4096,
                              n_samples=4096 * 2 + 5),
    "ch4_16_lpc12": dict(channels=4, bps=16, order=12, precision=13, block_size=2048, n_samples=2048 * 2 + 3),
    "ms20_lpc16_escape": dict(channels=2, bps=20, stereo_mode=10, order=16, precision=14, block_size=4096,
                              n_samples=4096 * 3, escape_every=7),
    "mono24_rice2": dict(channels=1, bps=24, order=8, block_size=4096, n_samples=4096 * 3, rice2=1),
    "ch3_16": dict(channels=3, bps=16, order=6, block_size=2048, n_samples=2048 * 4 + 1),
    "ch6_24_wasted": dict(channels=6, bps=24, order=10, precision=14, block_size=1024, n_samples=1024 * 3,
                          wasted_bits=2),
    "ch8_16_fixed": dict(channels=8, bps=16, predictor=2, order=2, block_size=512, n_samples=512 * 5),
    "stereo32": dict(channels=2, bps=32, stereo_mode=1, order=8, precision=15, block_size=4096,
                     n_samples=4096 * 2, tone_amp=0.2, noise_lsb=1e6),
    # 31/32-bit stereo on the fast path (wrapping i32 decorrelation, per-sample overflow checks)
    "stereo32_ms": dict(channels=2, bps=32, stereo_mode=10, order=8, precision=15, block_size=4096,
                        n_samples=4096 * 2, tone_amp=0.2, noise_lsb=1e6),
    "stereo31_ls_loud": dict(channels=2, bps=31, stereo_mode=8, order=8, precision=15, block_size=4096,
                             n_samples=4096 * 2, tone_amp=0.45, noise_lsb=1e6),
    "stereo32_rs": dict(channels=2, bps=32, stereo_mode=9, order=12, precision=15, block_size=2048,
                        n_samples=2048 * 3, tone_amp=0.3, noise_lsb=1e5),
    # long Rice codes: forced k with residuals ~2^k+4, so q + 1 + k crosses 32 bits often
    "longcodes24_k16": dict(channels=2, bps=24, stereo_mode=8, order=4, precision=14, block_size=4096,
                            n_samples=4096 * 2, rice_k=16, rice2=1, noise_lsb=float(2 ** 19)),
    "longcodes32_k26": dict(channels=1, bps=32, order=2, predictor=2, block_size=2048, n_samples=2048 * 3,
                            rice_k=26, rice2=1, noise_lsb=float(2 ** 29), tone_amp=0.0),
    "longcodes16_k3": dict(channels=2, bps=16, stereo_mode=10, order=8, precision=12, block_size=4096,
                           n_samples=4096 * 2, rice_k=3, partition_order=2, noise_lsb=300.0),
    # the reference's uncommon suite (tests/std_uncommon.zig:37-54)
    "uncommon_15bit": dict(channels=2, bps=15, stereo_mode=10, order=8, block_size=4096, n_samples=4096 * 3),
    "uncommon_768khz": dict(channels=2, bps=24, sample_rate=768000, order=12, precision=14, block_size=4096,
                            n_samples=4096 * 3, noise_lsb=64.0),
    "uncommon_block65535": dict(channels=2, bps=16, stereo_mode=10, order=8, block_size=65535,
                                n_samples=65535 * 2 + 100),
    "uncommon_po15": dict(channels=1, bps=16, predictor=2, order=1, block_size=32768, partition_order=15,
                          n_samples=32768 * 2),
    "variable_blocking": dict(channels=2, bps=16, variable_blocking=1, block_size=3000, n_samples=20000),
    "unknown_total": dict(channels=2, bps=16, write_total=0, block_size=4096, n_samples=4096 * 3 + 7),
    "silence_constant": dict(channels=2, bps=16, stereo_mode=1, silence_every=2, block_size=4096,
                             n_samples=4096 * 4),
    "extra_metadata": dict(channels=2, bps=16, extra_metadata=1, n_samples=4096 * 2, rate_code_mode=1,
                           sample_rate=37800),
    "blocksize16": dict(channels=1, bps=16, predictor=2, order=2, block_size=16, n_samples=16 * 300 + 1),
    "rate_div10": dict(channels=2, bps=16, rate_code_mode=2, sample_rate=44100, n_samples=4096 * 2),
    "rate_streaminfo": dict(channels=2, bps=16, rate_code_mode=3, sample_rate=96000, n_samples=4096 * 2),
    "verbatim_all": dict(channels=2, bps=16, predictor=0, stereo_mode=1, block_size=1024, n_samples=1024 * 4),
    "odd_block_4095": dict(channels=2, bps=16, block_size=4095, partition_order=0, n_samples=4095 * 3),
    "lpc32_16bit": dict(channels=2, bps=16, stereo_mode=10, order=32, precision=12, block_size=4096,
                        n_samples=4096 * 2),
}


def splice_frames(a, b, k: int) -> bytes:
    """Frames [0, k) of stream `a` then frames [k, n) of stream `b` (same shape: channels,
    depth, block size, rate, frame count), under `a`'s metadata with the STREAMINFO MD5 of
    the spliced PCM. zflac does not check frame numbers, so this is a valid stream whose
    frames change predictor between the two parts."""
    import hashlib

    ao = [int(x) for x in a.frame_offsets] + [len(a.flac)]
    bo = [int(x) for x in b.frame_offsets] + [len(b.flac)]
    assert len(ao) == len(bo)
    data = bytearray(a.flac[:ao[k]] + b.flac[bo[k]:])
    bps, ch = a.config["bps"], a.config["channels"]
    per = a.pcm.size // (len(ao) - 1)  # interleaved samples per (full) frame
    pcm = np.concatenate([a.pcm[:k * per], b.pcm[k * per:]])
    dt = container_dtype(bps)
    if (bps + 7) // 8 * 8 == 24:
        msg = np.ascontiguousarray(pcm.astype("<i4").view(np.uint8).reshape(-1, 4)[:, :3]).tobytes()
    else:
        msg = pcm.astype(np.dtype(dt).newbyteorder("<")).tobytes()
    assert ch == b.config["channels"]
    o = streaminfo_offset(bytes(data)) + 18
    data[o:o + 16] = hashlib.md5(msg).digest()
    return bytes(data)
