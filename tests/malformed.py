"""Malformed / uncommon streams and the zflac error each must produce.

Modelled on the reference's faulty and uncommon suites (tests/std_faulty.zig:17-61,
tests/std_uncommon.zig:17-59), whose input files are absent from the reference
snapshot: equivalent streams are built here from seeded synthetic ones. `expected`
is zflac's behaviour derived from src/zflac.zig (cited per case); None means
"whatever the oracle says" (used only for GPU-vs-oracle parity).
"""
from __future__ import annotations

import synth

from . import edges
from .util import patch, streaminfo_offset

BASE = dict(channels=2, bps=16, block_size=4096, order=8, stereo_mode=10, n_samples=4096 * 5, seed=77)


def _base(**kw):
    cfg = dict(BASE)
    cfg.update(kw)
    return synth.generate(**cfg)


def _set_si_field(data: bytes, fn) -> bytes:
    b = bytearray(data)
    o = streaminfo_offset(data)
    fn(b, o)
    return bytes(b)


def _si_channels(n):
    def f(b, o):
        b[o + 12] = (b[o + 12] & 0xF1) | (((n - 1) & 7) << 1)
    return f


def _si_bps(bps):
    def f(b, o):
        v = bps - 1
        b[o + 12] = (b[o + 12] & 0xFE) | (v >> 4)
        b[o + 13] = (b[o + 13] & 0x0F) | ((v & 15) << 4)
    return f


def _si_total(total):
    def f(b, o):
        b[o + 13] = (b[o + 13] & 0xF0) | ((total >> 32) & 15)
        for i in range(4):
            b[o + 14 + i] = (total >> (8 * (3 - i))) & 0xFF
    return f


def cases():
    st = _base()
    fo = [int(x) for x in st.frame_offsets]
    n = len(st.flac)
    out = {}

    out["bad_signature"] = (b"fLaX" + st.flac[4:], "InvalidSignature")  # :218-220
    out["starts_at_frame"] = (st.flac[st.frames_begin:], "InvalidSignature")  # uncommon/10
    out["unparsable_start"] = (b"\x00\x01garbage" + st.flac, "InvalidSignature")  # uncommon/11
    # STREAMINFO not last + a reserved metadata block type 7 (:248)
    b = bytearray(st.flac[:st.frames_begin])
    b[4] &= 0x7F
    out["reserved_metadata_type"] = (bytes(b) + bytes([0x87, 0, 0, 2, 1, 2]) + st.flac[st.frames_begin:],
                                     "InvalidMetadataHeader")
    out["metadata_type_127"] = (bytes(b) + bytes([0xFF, 0, 0, 0]) + st.flac[st.frames_begin:], "InvalidMetadataHeader")
    # STREAMINFO relabelled as PADDING -> no STREAMINFO (:309)
    out["missing_streaminfo"] = (patch(st.flac, 4, (st.flac[4] & 0x80) | 1), "MissingStreaminfo")
    # a STREAMINFO length field of 40: zflac reads STREAMINFO as a fixed 34 bytes whatever
    # the field says (:228-240), so the stream decodes. (faulty/11 proper, a skipped block
    # whose length is wrong -> InvalidMetadataHeader, is tests/edges.py's
    # incorrect_metadata_length_case.)
    out["streaminfo_length_40"] = (patch(st.flac, 7, 40), "OK")
    out["incorrect_metadata_length"] = (edges.incorrect_metadata_length_case(st.flac, st.frames_begin),
                                        "InvalidMetadataHeader")  # tests/std_faulty.zig:59-61
    md5o = streaminfo_offset(st.flac) + 18
    out["wrong_md5"] = (patch(st.flac, md5o, st.flac[md5o] ^ 0x5A), "InvalidChecksum")  # :279-280
    out["wrong_channel_count"] = (_set_si_field(st.flac, _si_channels(1)), "InconsistentParameters")  # :386
    out["wrong_bit_depth"] = (_set_si_field(st.flac, _si_bps(24)), "InvalidChecksum")  # faulty/03
    out["total_smaller"] = (_set_si_field(st.flac, _si_total(4096 * 2 + 5)), "OK")  # faulty/05, realloc (:394-402)
    out["total_larger"] = (_set_si_field(st.flac, _si_total(4096 * 7)), "EndOfStream")  # :344
    out["total_unknown"] = (_set_si_field(st.flac, _si_total(0)), "OK")
    out["truncated_mid_frame"] = (st.flac[: fo[3] + 1000], "EndOfStream")
    out["truncated_frame_header"] = (st.flac[: fo[3] + 3], "EndOfStream")
    out["truncated_boundary_unknown_total"] = (_set_si_field(st.flac[: fo[3]], _si_total(0)), "InvalidChecksum")
    out["bad_sync_frame2"] = (patch(st.flac, fo[2] + 1, 0xF0), "InvalidFrameHeader")  # :351-352
    out["bad_crc8_frame1"] = (patch(st.flac, fo[1] + 5, st.flac[fo[1] + 5] ^ 0x11), "OK")  # never checked (:407)
    out["bad_crc16_frame1"] = (patch(st.flac, fo[2] - 1, st.flac[fo[2] - 1] ^ 0x11), "OK")  # never checked (:548)
    b2 = st.flac[fo[2] + 2]
    out["rate_change_frame2"] = (patch(st.flac, fo[2] + 2, (b2 & 0xF0) | 10), "InconsistentParameters")  # :391
    b3 = st.flac[fo[2] + 3]
    out["channels_change_frame2"] = (patch(st.flac, fo[2] + 3, (b3 & 0x0F) | (0 << 4)), "InconsistentParameters")
    out["depth_code_change_frame2"] = (patch(st.flac, fo[2] + 3, (b3 & 0xF1) | (0 << 1)), "InconsistentParameters")
    out["assignment_change_frame2"] = (patch(st.flac, fo[2] + 3, (b3 & 0x0F) | (8 << 4)), "InvalidChecksum")
    out["reserved_channels_frame2"] = (patch(st.flac, fo[2] + 3, (b3 & 0x0F) | (11 << 4)), "InconsistentParameters")
    out["reserved_blocksize_frame2"] = (patch(st.flac, fo[2] + 2, b2 & 0x0F), "InvalidFrameHeader")  # :357
    out["forbidden_rate_frame2"] = (patch(st.flac, fo[2] + 2, (b2 & 0xF0) | 15), "InvalidFrameHeader")  # :372
    out["coded_number_ff_frame2"] = (patch(st.flac, fo[2] + 4, 0xFF), "InvalidCodedNumber")  # :206
    out["coded_number_10x_frame2"] = (patch(st.flac, fo[2] + 4, 0x80), "InvalidCodedNumber")
    b3f = st.flac[fo[0] + 3]
    out["reserved_depth_first_frame"] = (patch(st.flac, fo[0] + 3, (b3f & 0xF1) | (3 << 1)), "OutOfDomain")  # :143
    out["reserved_depth_frame2"] = (patch(st.flac, fo[2] + 3, (b3 & 0xF1) | (3 << 1)), "InconsistentParameters")
    out["trailing_garbage_known_total"] = (st.flac + b"\x12\x34\x56\x78\x9a" * 20, "OK")  # :341
    out["trailing_garbage_unknown_total"] = (_set_si_field(st.flac + b"\x12\x34\x56\x78\x9a" * 20, _si_total(0)),
                                             "InvalidFrameHeader")
    out["trailing_3_bytes_unknown_total"] = (_set_si_field(st.flac + b"\x01\x02\x03", _si_total(0)), "OK")
    out["no_frames_unknown_total"] = (_set_si_field(st.flac[: st.frames_begin], _si_total(0)), "InvalidChecksum")
    out["no_frames_known_total"] = (st.flac[: st.frames_begin], "EndOfStream")
    # encoder-level faults (synth fault_kind)
    out["reserved_subframe_type"] = (_base(fault_frame=2, fault_kind=1).flac, "InvalidSubframeHeader")  # :542
    out["residual_method_2"] = (_base(fault_frame=3, fault_kind=2).flac, "InvalidResidualCodingMethod")  # :618
    out["lpc_precision_15"] = (_base(fault_frame=1, fault_kind=3).flac, "OutOfDomain")  # :508 u4 overflow
    out["blocksize1_middle"] = (_base(fault_frame=2, fault_kind=4).flac, "InvalidFrameHeader")  # faulty/09, :405
    out["partition_order_not_dividing"] = (
        _base(fault_frame=1, fault_kind=5, block_size=4095, partition_order=0, n_samples=4095 * 4).flac,
        "OutOfDomain")
    # STREAMINFO max block size / max frame size are never used (faulty/01, faulty/02)
    def _si_max_block(v):
        def f(b, o):
            b[o + 2], b[o + 3] = (v >> 8) & 0xFF, v & 0xFF
        return f

    def _si_max_frame(v):
        def f(b, o):
            b[o + 7], b[o + 8], b[o + 9] = (v >> 16) & 0xFF, (v >> 8) & 0xFF, v & 0xFF
        return f

    out["wrong_max_blocksize"] = (_set_si_field(st.flac, _si_max_block(16)), "OK")  # faulty/01
    out["wrong_max_framesize"] = (_set_si_field(st.flac, _si_max_frame(1)), "OK")  # faulty/02
    # a PADDING block ahead of STREAMINFO (faulty/07): the metadata loop takes any order (:228-265)
    out["streaminfo_not_first"] = (b"fLaC" + bytes([0x01, 0, 0, 4, 0, 0, 0, 0]) + st.flac[4:], "OK")
    # a VORBIS_COMMENT block whose content is garbage is skipped unread (faulty/10, :248-250)
    si_end = streaminfo_offset(st.flac) + 34
    vc = bytes([0x04 | (st.flac[4] & 0x80), 0, 0, 9]) + b"\xff\xff\xff\x7fjunk\x00"
    out["invalid_vorbis_comment"] = (st.flac[:4] + bytes([st.flac[4] & 0x7F]) + st.flac[5:si_end] + vc
                                     + st.flac[si_end:], "OK")
    # uncommon 16-bit block size 0xFFFF -> 65536 is refused (faulty/08, :358-361); the CRC-8
    # byte is not rewritten (zflac never reads it back before failing)
    h = bytearray(st.flac[fo[2]:fo[2] + 5])
    h[2] = (7 << 4) | (h[2] & 0x0F)
    out["blocksize_65536_frame2"] = (st.flac[:fo[2]] + bytes(h) + b"\xff\xff" + st.flac[fo[2] + 5:],
                                     "InvalidFrameHeader")
    # a last frame of one sample is legal (:405)
    out["blocksize1_last"] = (_base(n_samples=4096 * 3 + 1).flac, "OK")
    del n
    return out
