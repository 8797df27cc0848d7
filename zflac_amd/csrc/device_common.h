// device_common.h -- device helpers shared by the scan and decode translation units:
// format tables, the exact frame-header parser (src/zflac.zig:343-407) and small utils.
#pragma once
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdint>
#include <utility>

#include "common.h"

namespace zflac {

// ----------------------------------------------------------------------------------
// small helpers
// ----------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

__device__ __forceinline__ int channels_count(uint32_t code) {  // Channels.count, src/zflac.zig:107-122
    return code <= 7 ? (int)code + 1 : (code <= 10 ? 2 : 0);
}
__device__ __forceinline__ uint32_t rate_table(uint32_t code) {  // SampleRate.hz, src/zflac.zig:75-90
    switch (code) {
        case 1: return 88200;
        case 2: return 176400;
        case 3: return 192000;
        case 4: return 8000;
        case 5: return 16000;
        case 6: return 22050;
        case 7: return 24000;
        case 8: return 32000;
        case 9: return 44100;
        case 10: return 48000;
        default: return 96000;
    }
}
__device__ __forceinline__ int depth_bits(uint32_t dcode, int si_bps) {  // BitDepth.bps, src/zflac.zig:135-145
    switch (dcode) {
        case 0: return si_bps;
        case 1: return 8;
        case 2: return 12;
        case 4: return 16;
        case 5: return 20;
        case 6: return 24;
        case 7: return 32;
        default: return -1;  // reserved: `unreachable` in zflac
    }
}

struct Crc8Table {
    uint8_t t[256];
};
constexpr Crc8Table make_crc8_table() {  // x^8 + x^2 + x + 1, init 0 (RFC 9639 frame header CRC)
    Crc8Table r{};
    for (int i = 0; i < 256; i++) {
        uint32_t c = (uint32_t)i;
        for (int k = 0; k < 8; k++) c = (c & 0x80) ? ((c << 1) ^ 0x07) & 0xFF : (c << 1) & 0xFF;
        r.t[i] = (uint8_t)c;
    }
    return r;
}
static __constant__ Crc8Table CRC8 = make_crc8_table();

// a (a polynomial of degree < 32 over GF(2)) mod x^8 + x^2 + x + 1. With x^8 = x^2 + x + 1,
// a = t x^8 + l reduces to t (x^2 + x + 1) + l: one fold lowers the degree by 6, four take
// 31 down to 7. Register-only: a table lookup is an LDS round trip per byte, and the bytes of
// a header are a dependent chain.
constexpr uint32_t crc8_reduce(uint32_t a) {
    for (int i = 0; i < 4; i++) {
        const uint32_t t = a >> 8;
        a = (t ^ (t << 1) ^ (t << 2)) ^ (a & 0xFFu);
    }
    return a;
}
// CRC-8 (init 0, MSB first) after three more bytes b0 b1 b2 (w = b0 << 16 | b1 << 8 | b2):
// the message (b0 ^ crc) x^16 + b1 x^8 + b2, times x^8, mod the polynomial
constexpr uint32_t crc8_3(uint32_t crc, uint32_t w) { return crc8_reduce((w ^ (crc << 16)) << 8); }
constexpr uint32_t crc8_1(uint32_t crc, uint32_t b) { return crc8_reduce((crc ^ b) << 8); }
constexpr bool crc8_fold_matches_table() {
    const Crc8Table t = make_crc8_table();
    for (uint32_t i = 0; i < 256; i++)
        if (crc8_1(0, i) != t.t[i]) return false;
    uint32_t a = 0, b = 0, x = 12345;  // 3-byte steps against byte steps over a pseudo-random message
    for (int k = 0; k < 300; k++) {
        uint32_t w = 0;
        for (int j = 0; j < 3; j++) {
            x = x * 1103515245u + 12345u;
            const uint32_t by = (x >> 16) & 0xFFu;
            a = t.t[a ^ by];
            w = (w << 8) | by;
        }
        b = crc8_3(b, w);
        if (a != b) return false;
    }
    return true;
}
static_assert(crc8_fold_matches_table(), "register CRC-8 = table CRC-8");

// ----------------------------------------------------------------------------------
// Frame header, exact zflac semantics (src/zflac.zig:343-375, 203-214, 407).
// `err` holds errors raised before the first-frame / consistency checks; a missing
// CRC-8 byte is reported separately because zflac reads it after those checks.
// ----------------------------------------------------------------------------------
struct FrameHdr {
    uint32_t bs, rate, hdr_len;
    uint32_t chan_code, dcode, byte1, zero_bit, bs_code;
    int err;
    bool crc_eof;
    bool crc_ok;
};

// `at(i)` returns header byte i (global memory, an LDS copy or registers). CRC: 0 skips the
// CRC-8 (the decode kernels only need the fields: candidates were filtered already), 1 looks
// it up in `crc_tab` (global memory, or an LDS copy), 2 computes it in registers (k_scan).
template <int CRC, typename At>
__device__ __forceinline__ FrameHdr parse_frame_header_t(At&& at, uint64_t avail, uint32_t si_rate,
                                                         const uint8_t* crc_tab) {
    FrameHdr h;
    h.bs = h.rate = h.hdr_len = 0;
    h.chan_code = h.dcode = h.byte1 = h.zero_bit = h.bs_code = 0;
    h.err = 0;
    h.crc_eof = false;
    h.crc_ok = false;
    if (avail < 4) { h.err = E_END_OF_STREAM; return h; }
    const uint32_t b0 = at(0), b1 = at(1), b2 = at(2), b3 = at(3);
    h.byte1 = b1;
    h.chan_code = b3 >> 4;
    h.dcode = (b3 >> 1) & 7;
    h.zero_bit = b3 & 1;
    h.bs_code = b2 >> 4;
    if (((b0 << 7) | (b1 >> 1)) != 0x7FFC) { h.err = E_INVALID_FRAME_HEADER; return h; }  // :351-352
    uint32_t idx = 4;
    // read_coded_number (:203-214)
    if (avail <= idx) { h.err = E_END_OF_STREAM; return h; }
    const uint32_t first = at(idx++);
    const uint32_t ones = __clz((~first & 0xFFu) << 24) > 8 ? 8 : __clz((~first & 0xFFu) << 24);
    if (first == 0xFF || ones == 1) { h.err = E_INVALID_CODED_NUMBER; return h; }
    if (ones >= 2) {
        if (avail < (uint64_t)idx + (ones - 1)) { h.err = E_END_OF_STREAM; return h; }
        idx += ones - 1;
    }
    // block size (:356-365)
    const uint32_t bc = b2 >> 4;
    if (bc == 0) { h.err = E_INVALID_FRAME_HEADER; return h; }
    if (bc == 6) {
        if (avail <= idx) { h.err = E_END_OF_STREAM; return h; }
        h.bs = (uint32_t)at(idx++) + 1;
    } else if (bc == 7) {
        if (avail < (uint64_t)idx + 2) { h.err = E_END_OF_STREAM; return h; }
        const uint32_t v = ((uint32_t)at(idx) << 8) | at(idx + 1);
        idx += 2;
        if (v == 0xFFFF) { h.err = E_INVALID_FRAME_HEADER; return h; }
        h.bs = v + 1;
    } else if (bc == 1) {
        h.bs = 192;
    } else if (bc <= 5) {
        h.bs = 144u << bc;
    } else {
        h.bs = 1u << bc;
    }
    // sample rate (:367-374); uncommon 8-bit rate is taken in Hz as zflac does (:369)
    const uint32_t rc = b2 & 15;
    if (rc == 0) {
        h.rate = si_rate;
    } else if (rc == 12) {
        if (avail <= idx) { h.err = E_END_OF_STREAM; return h; }
        h.rate = at(idx++);
    } else if (rc == 13 || rc == 14) {
        if (avail < (uint64_t)idx + 2) { h.err = E_END_OF_STREAM; return h; }
        h.rate = ((uint32_t)at(idx) << 8) | at(idx + 1);
        if (rc == 14) h.rate *= 10;
        idx += 2;
    } else if (rc == 15) {
        h.err = E_INVALID_FRAME_HEADER;
        return h;
    } else {
        h.rate = rate_table(rc);
    }
    // CRC-8 byte (:407): read, never checked by zflac; checked here only to filter
    // sync candidates.
    h.hdr_len = idx + 1;
    if (avail <= idx) {
        h.crc_eof = true;
        return h;
    }
    if constexpr (CRC == 1) {
        uint32_t crc = 0;
        for (uint32_t i = 0; i < idx; i++) crc = crc_tab[crc ^ at(i)];
        h.crc_ok = crc == at(idx);
    } else if constexpr (CRC == 2) {
        uint32_t crc = 0, i = 0;  // idx <= 15: up to five 3-byte steps, then up to two bytes
#pragma unroll
        for (int g = 0; g < 5; g++) {
            if (i + 3 <= idx) {
                crc = crc8_3(crc, (at(i) << 16) | (at(i + 1) << 8) | at(i + 2));
                i += 3;
            }
        }
#pragma unroll
        for (int g = 0; g < 2; g++) {
            if (i < idx) {
                crc = crc8_1(crc, at(i));
                i++;
            }
        }
        h.crc_ok = crc == at(idx);
    }
    return h;
}

__device__ __forceinline__ FrameHdr parse_frame_header(const uint8_t* p, uint64_t avail, uint32_t si_rate) {
    return parse_frame_header_t<1>([p](uint32_t i) -> uint32_t { return p[i]; }, avail, si_rate, CRC8.t);
}
__device__ __forceinline__ FrameHdr parse_frame_fields(const uint8_t* p, uint64_t avail, uint32_t si_rate) {
    return parse_frame_header_t<0>([p](uint32_t i) -> uint32_t { return p[i]; }, avail, si_rate, nullptr);
}



// Filter for sync candidates: a well-formed header consistent with the stream's first
// frame. Anything it rejects that zflac would still decode breaks the verified chain and
// sends the stream to the sequential planner, so the filter affects speed only.
__device__ __forceinline__ bool candidate_ok(const FrameHdr& h, const StreamDesc& S) {
    return h.err == 0 && !h.crc_eof && h.crc_ok && h.zero_bit == 0 && h.byte1 == S.byte1 &&
           channels_count(h.chan_code) == S.nch && h.dcode == S.dcode && h.rate == S.rate_hz;
}

}  // namespace zflac
