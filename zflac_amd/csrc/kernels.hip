// kernels.hip -- gfx950 kernels of the FLAC decode path.
//
//   k_scan      frame-sync scan: every input byte once, 16 B/lane coalesced loads;
//               candidates = 0xFF 0xF8|F9 + exact header parse + CRC-8 + the stream's
//               first-frame parameters. Up to CHUNK_CAP ordered candidates per 32 KiB chunk.
//   k_scan_chunks   exclusive scan of per-chunk candidate counts / sample units.
//   k_compact   ordered candidate table (position, stream, output offset).
//   k_decode    THE HOT PATH. One lane per subframe (64 subframes per wave: 32 stereo
//               frames, 64 mono frames, floor(64/C) frames otherwise). A walk phase finds
//               where subframe c+1 starts (subframe c's end), then every lane decodes its
//               subframe: header, warm-up, Rice/escape residuals, fixed/LPC rollback in
//               registers, wasted bits, stereo decorrelation through v_permlane32_swap,
//               left-justify and packed 16-byte PCM stores.
//   k_verify    checks that the candidate chain is exactly what zflac's sequential frame
//               loop (src/zflac.zig:340-581) would have walked; streams that fail it are
//               finished by the host's sequential planner.
//
// Reference semantics cited inline as src/zflac.zig:LINE.
#include <hip/hip_runtime.h>

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
__constant__ Crc8Table CRC8 = make_crc8_table();

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

__device__ inline FrameHdr parse_frame_header(const uint8_t* p, uint64_t avail, uint32_t si_rate) {
    FrameHdr h;
    h.bs = h.rate = h.hdr_len = 0;
    h.chan_code = h.dcode = h.byte1 = h.zero_bit = h.bs_code = 0;
    h.err = 0;
    h.crc_eof = false;
    h.crc_ok = false;
    if (avail < 4) { h.err = E_END_OF_STREAM; return h; }
    const uint32_t b0 = p[0], b1 = p[1], b2 = p[2], b3 = p[3];
    h.byte1 = b1;
    h.chan_code = b3 >> 4;
    h.dcode = (b3 >> 1) & 7;
    h.zero_bit = b3 & 1;
    h.bs_code = b2 >> 4;
    if (((b0 << 7) | (b1 >> 1)) != 0x7FFC) { h.err = E_INVALID_FRAME_HEADER; return h; }  // :351-352
    uint32_t idx = 4;
    // read_coded_number (:203-214)
    if (avail <= idx) { h.err = E_END_OF_STREAM; return h; }
    const uint32_t first = p[idx++];
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
        h.bs = (uint32_t)p[idx++] + 1;
    } else if (bc == 7) {
        if (avail < (uint64_t)idx + 2) { h.err = E_END_OF_STREAM; return h; }
        const uint32_t v = ((uint32_t)p[idx] << 8) | p[idx + 1];
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
        h.rate = p[idx++];
    } else if (rc == 13 || rc == 14) {
        if (avail < (uint64_t)idx + 2) { h.err = E_END_OF_STREAM; return h; }
        h.rate = ((uint32_t)p[idx] << 8) | p[idx + 1];
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
    uint32_t crc = 0;
    for (uint32_t i = 0; i < idx; i++) crc = CRC8.t[crc ^ p[i]];
    h.crc_ok = crc == p[idx];
    return h;
}

// Filter for sync candidates: a well-formed header consistent with the stream's first
// frame. Anything it rejects that zflac would still decode breaks the verified chain and
// sends the stream to the sequential planner, so the filter affects speed only.
__device__ inline bool candidate_ok(const FrameHdr& h, const StreamDesc& S) {
    return h.err == 0 && !h.crc_eof && h.crc_ok && h.zero_bit == 0 && h.byte1 == S.byte1 &&
           channels_count(h.chan_code) == S.nch && h.dcode == S.dcode && h.rate == S.rate_hz;
}

// ----------------------------------------------------------------------------------
// k_scan: frame-sync candidates per 32 KiB chunk
// ----------------------------------------------------------------------------------
__device__ inline uint32_t ff_mask(uint32_t d) { return ((d & 0x7F7F7F7Fu) + 0x01010101u) & d & 0x80808080u; }

// Calls fn(position) for every candidate in the 16-byte window at `ws` that lies in
// [lo, hi). Windows are 16-byte aligned.
template <typename Fn>
__device__ inline void scan_window(const uint8_t* in, uint64_t ws, uint64_t lo, uint64_t hi, Fn&& fn) {
    const uint4 v = *reinterpret_cast<const uint4*>(in + ws);
    const uint32_t d[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int k = 0; k < 4; k++) {
        uint32_t m = ff_mask(d[k]);
        while (m) {
            const int bit = __ffs(m) - 1;
            m &= m - 1;
            const int b = 4 * k + (bit >> 3);
            uint32_t nxt;
            if (b < 15) nxt = (d[(b + 1) >> 2] >> (8 * ((b + 1) & 3))) & 0xFF;
            else nxt = in[ws + 16];
            const uint64_t p = ws + b;
            if ((nxt & 0xFE) == 0xF8 && p >= lo && p < hi) fn(p);
        }
    }
}

__global__ __launch_bounds__(SCAN_THREADS) void k_scan(ScanArgs a) {
    const uint32_t chunk = blockIdx.x;
    if (chunk >= a.n_chunks) return;
    __shared__ uint32_t s_cnt;
    __shared__ unsigned long long s_units;
    __shared__ uint64_t s_pos[CHUNK_CAP];
    __shared__ uint32_t s_u[CHUNK_CAP];
    const ChunkDesc ch = a.chunks[chunk];
    const StreamDesc S = a.streams[ch.stream];
    if (threadIdx.x == 0) {
        s_cnt = 0;
        s_units = 0;
    }
    __syncthreads();
    const uint64_t abase = ch.begin & ~(uint64_t)15;
    for (int r = 0; r < SCAN_BYTES_PER_THREAD / 16; r++) {
        const uint64_t ws = abase + ((uint64_t)r * SCAN_THREADS + threadIdx.x) * 16;
        if (ws >= ch.end) break;
        scan_window(a.in, ws, ch.begin, ch.end, [&](uint64_t p) {
            const FrameHdr h = parse_frame_header(a.in + p, S.in_end - p, S.si_rate);
            if (!candidate_ok(h, S)) return;
            const uint32_t slot = atomicAdd(&s_cnt, 1u);
            const uint32_t units = h.bs * S.nch;
            atomicAdd(&s_units, (unsigned long long)units);
            if (slot < CHUNK_CAP) {
                s_pos[slot] = p;
                s_u[slot] = units;
            }
        });
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t n = s_cnt;
        const uint32_t m = n < CHUNK_CAP ? n : CHUNK_CAP;
        for (uint32_t i = 1; i < m; i++) {  // insertion sort by position (m is tiny)
            uint64_t p = s_pos[i];
            uint32_t u = s_u[i];
            int j = (int)i - 1;
            while (j >= 0 && s_pos[j] > p) {
                s_pos[j + 1] = s_pos[j];
                s_u[j + 1] = s_u[j];
                j--;
            }
            s_pos[j + 1] = p;
            s_u[j + 1] = u;
        }
        a.chunk_cnt[chunk] = n;
        a.chunk_units[chunk] = s_units;
    }
    __syncthreads();
    const uint32_t m = s_cnt < CHUNK_CAP ? s_cnt : CHUNK_CAP;
    if (threadIdx.x < m) {
        a.chunk_slots[(uint64_t)chunk * CHUNK_CAP + threadIdx.x] = s_pos[threadIdx.x];
        a.chunk_slot_units[(uint64_t)chunk * CHUNK_CAP + threadIdx.x] = s_u[threadIdx.x];
    }
}

// ----------------------------------------------------------------------------------
// k_scan_chunks: single-workgroup exclusive scans (n_chunks is ~input/32KiB)
// ----------------------------------------------------------------------------------
constexpr int SCANK_THREADS = 1024;

__global__ __launch_bounds__(SCANK_THREADS) void k_scan_chunks(const uint32_t* cnt, const unsigned long long* units,
                                                               uint32_t n, uint32_t* off,
                                                               unsigned long long* uoff, uint32_t* n_frames) {
    __shared__ uint32_t s_c[SCANK_THREADS];
    __shared__ unsigned long long s_u[SCANK_THREADS];
    const uint32_t t = threadIdx.x;
    const uint32_t per = (n + SCANK_THREADS - 1) / SCANK_THREADS;
    const uint32_t lo = t * per, hi = (lo + per < n) ? lo + per : n;
    uint32_t sc = 0;
    unsigned long long su = 0;
    for (uint32_t i = lo; i < hi; i++) {
        sc += cnt[i];
        su += units[i];
    }
    s_c[t] = sc;
    s_u[t] = su;
    __syncthreads();
    for (uint32_t d = 1; d < SCANK_THREADS; d <<= 1) {  // Hillis-Steele inclusive
        uint32_t vc = 0;
        unsigned long long vu = 0;
        if (t >= d) {
            vc = s_c[t - d];
            vu = s_u[t - d];
        }
        __syncthreads();
        s_c[t] += vc;
        s_u[t] += vu;
        __syncthreads();
    }
    uint32_t rc = t ? s_c[t - 1] : 0;
    unsigned long long ru = t ? s_u[t - 1] : 0;
    for (uint32_t i = lo; i < hi; i++) {
        off[i] = rc;
        uoff[i] = ru;
        rc += cnt[i];
        ru += units[i];
    }
    if (t == SCANK_THREADS - 1) {
        off[n] = s_c[t];
        uoff[n] = s_u[t];
        *n_frames = s_c[t];
    }
}

// ----------------------------------------------------------------------------------
// k_compact: ordered candidate table
// ----------------------------------------------------------------------------------
__global__ __launch_bounds__(SCAN_THREADS) void k_compact(CompactArgs a) {
    const uint32_t chunk = blockIdx.x;
    if (chunk >= a.n_chunks) return;
    const ChunkDesc ch = a.chunks[chunk];
    const StreamDesc S = a.streams[ch.stream];
    const uint32_t n = a.chunk_cnt[chunk];
    const uint32_t off = a.chunk_off[chunk];
    const unsigned long long ubase = a.chunk_uoff[S.first_chunk];
    const unsigned long long u0 = a.chunk_uoff[chunk];
    if (n <= CHUNK_CAP) {
        const uint32_t t = threadIdx.x;
        if (t < n) {
            unsigned long long pre = 0;
            for (uint32_t i = 0; i < t; i++) pre += a.chunk_slot_units[(uint64_t)chunk * CHUNK_CAP + i];
            const uint32_t idx = off + t;
            if (idx < a.cap) {
                a.c_pos[idx] = a.chunk_slots[(uint64_t)chunk * CHUNK_CAP + t];
                a.c_stream[idx] = ch.stream;
                a.c_out[idx] = S.out_base + (u0 - ubase + pre);
            } else {
                atomicOr(a.overflow, 1u);
            }
        }
        return;
    }
    // Overflowed chunk (more than CHUNK_CAP candidates): ordered two-pass rescan of each
    // 4 KiB sub-range with a block-wide exclusive scan.
    __shared__ uint32_t s_c[SCAN_THREADS];
    __shared__ unsigned long long s_u[SCAN_THREADS];
    __shared__ uint32_t s_base_c;
    __shared__ unsigned long long s_base_u;
    if (threadIdx.x == 0) {
        s_base_c = 0;
        s_base_u = 0;
    }
    __syncthreads();
    const uint64_t abase = ch.begin & ~(uint64_t)15;
    for (int r = 0; r < SCAN_BYTES_PER_THREAD / 16; r++) {
        const uint64_t ws = abase + ((uint64_t)r * SCAN_THREADS + threadIdx.x) * 16;
        uint32_t c = 0;
        unsigned long long u = 0;
        if (ws < ch.end) {
            scan_window(a.in, ws, ch.begin, ch.end, [&](uint64_t p) {
                const FrameHdr h = parse_frame_header(a.in + p, S.in_end - p, S.si_rate);
                if (!candidate_ok(h, S)) return;
                c++;
                u += h.bs * S.nch;
            });
        }
        s_c[threadIdx.x] = c;
        s_u[threadIdx.x] = u;
        __syncthreads();
        for (uint32_t d = 1; d < SCAN_THREADS; d <<= 1) {
            uint32_t vc = 0;
            unsigned long long vu = 0;
            if (threadIdx.x >= d) {
                vc = s_c[threadIdx.x - d];
                vu = s_u[threadIdx.x - d];
            }
            __syncthreads();
            s_c[threadIdx.x] += vc;
            s_u[threadIdx.x] += vu;
            __syncthreads();
        }
        uint32_t rc = s_base_c + s_c[threadIdx.x] - c;
        unsigned long long ru = s_base_u + s_u[threadIdx.x] - u;
        if (ws < ch.end && c) {
            scan_window(a.in, ws, ch.begin, ch.end, [&](uint64_t p) {
                const FrameHdr h = parse_frame_header(a.in + p, S.in_end - p, S.si_rate);
                if (!candidate_ok(h, S)) return;
                const uint32_t idx = off + rc;
                if (idx < a.cap) {
                    a.c_pos[idx] = p;
                    a.c_stream[idx] = ch.stream;
                    a.c_out[idx] = S.out_base + (u0 - ubase + ru);
                } else {
                    atomicOr(a.overflow, 1u);
                }
                rc++;
                ru += h.bs * S.nch;
            });
        }
        __syncthreads();
        if (threadIdx.x == SCAN_THREADS - 1) {
            s_base_c += s_c[threadIdx.x];
            s_base_u += s_u[threadIdx.x];
        }
        __syncthreads();
    }
}

// ----------------------------------------------------------------------------------
// Lane bit reader: MSB-first over 32-bit big-endian words, 64-bit window + one word
// prefetched (src/bit_reader.zig semantics; EOF is decided against `end` by callers).
// Positions are bit offsets from the lane's 4-byte aligned base. Word loads are clamped
// to the padded input, so garbage decodes never leave the buffer.
// ----------------------------------------------------------------------------------
struct BitReader {
    const uint32_t* base;
    uint64_t bb;       // valid bits MSB-aligned
    int32_t nb;        // number of valid bits (> 32 between operations)
    uint32_t w1;       // raw next word (index wnext)
    uint32_t wnext;
    uint32_t wmax;     // last loadable word index

    __device__ __forceinline__ void init(const uint32_t* b, uint32_t bitpos, uint32_t wmax_) {
        base = b;
        wmax = wmax_;
        uint32_t wi = bitpos >> 5;
        const uint32_t sh = bitpos & 31;
        const uint32_t w0 = bswap32(base[min(wi, wmax)]);
        const uint32_t wa = bswap32(base[min(wi + 1, wmax)]);
        bb = ((((uint64_t)w0) << 32) | wa) << sh;
        nb = 64 - (int32_t)sh;
        wnext = wi + 2;
        w1 = base[min(wnext, wmax)];
    }
    __device__ __forceinline__ uint32_t pos() const { return wnext * 32u - (uint32_t)nb; }
    __device__ __forceinline__ void refill() {
        if (nb <= 32) {
            bb |= ((uint64_t)bswap32(w1)) << (32 - nb);
            nb += 32;
            wnext++;
            w1 = base[min(wnext, wmax)];
        }
    }
    __device__ __forceinline__ uint32_t hi() const { return (uint32_t)(bb >> 32); }
    __device__ __forceinline__ void consume(uint32_t n) {  // n <= 32
        bb <<= n;
        nb -= (int32_t)n;
        refill();
    }
    // n in [0, 32]
    __device__ __forceinline__ uint32_t read(uint32_t n) {
        const uint32_t v = n ? (uint32_t)(bb >> (64 - n)) : 0u;
        consume(n);
        return v;
    }
    // n-bit two's complement, n in [1, 32] (read_signed_integer, src/zflac.zig:188-196)
    __device__ __forceinline__ int32_t read_signed(uint32_t n) {
        const uint32_t v = read(n);
        return n ? ((int32_t)(v << (32 - n)) >> (32 - n)) : 0;
    }
    // n in [1, 64]
    __device__ __forceinline__ int64_t read_signed_wide(uint32_t n) {
        if (n <= 32) return read_signed(n);
        const uint64_t hi_ = read(n - 32);
        const uint64_t lo_ = read(32);
        const uint64_t v = (hi_ << 32) | lo_;
        return (int64_t)(v << (64 - n)) >> (64 - n);
    }
    __device__ __forceinline__ void skip(uint64_t n) {
        if (n <= 32) {
            consume((uint32_t)n);
        } else {
            const uint64_t np = (uint64_t)pos() + n;
            init(base, np > 0xFFFFFF00ull ? 0xFFFFFF00u : (uint32_t)np, wmax);
        }
    }
    // readUnary (bit_reader.zig:95-120); stops at `end` with EndOfStream
    __device__ inline bool unary(uint32_t end, uint32_t& q) {
        q = 0;
        for (;;) {
            const uint32_t h = hi();
            if (h) {
                const uint32_t z = __clz(h);
                q += z;
                consume(z + 1);
                return pos() <= end;
            }
            q += 32;
            consume(32);
            if (pos() > end) return false;
        }
    }
};

// ----------------------------------------------------------------------------------
// Subframe decode, lane per subframe
// ----------------------------------------------------------------------------------
template <int KIND>
struct Kind;
template <>
struct Kind<0> {  // 8-bit container, InterType i16
    static constexpr int SB = 8, W = 16, ESZ = 1;
};
template <>
struct Kind<1> {  // 16-bit container, InterType i32
    static constexpr int SB = 16, W = 32, ESZ = 2;
};
template <>
struct Kind<2> {  // 32-bit container (17..32 bps), InterType i64
    static constexpr int SB = 32, W = 64, ESZ = 4;
};

enum Mode : int { M_NONE = 0, M_CONST = 1, M_VERB = 2, M_PRED = 3 };

// wrap to the SampleType width
template <int KIND>
__device__ __forceinline__ int32_t wrap_st(int64_t v) {
    if constexpr (Kind<KIND>::SB == 8) return (int32_t)(int8_t)v;
    else if constexpr (Kind<KIND>::SB == 16) return (int32_t)(int16_t)v;
    else return (int32_t)v;
}

struct LaneCtx {
    // frame
    uint32_t bs;
    int bps;          // frame bits per sample
    int ubps;         // + side bit for this lane's channel (src/zflac.zig:436-441)
    uint32_t chan_code;
    uint32_t end;     // stream end, bit offset from the lane base
    // subframe
    int mode;
    int wasted;
    int cbps;
    int order;
    int shift;
    int32_t cval;
    // residual partitions
    int method;
    uint32_t psize;
    uint32_t parts_left;
    uint32_t left;
    uint32_t k;
    uint32_t escw;
    bool esc;
    int err;
};

template <int KIND>
__device__ __forceinline__ void set_err(LaneCtx& L, const BitReader& br, int e) {
    if (!L.err) L.err = (br.pos() > L.end) ? E_END_OF_STREAM : e;
    L.mode = M_NONE;
}

// Partition header (src/zflac.zig:635-654)
template <int KIND>
__device__ inline void read_partition_header(LaneCtx& L, BitReader& br) {
    const uint32_t k = br.read(L.method ? 5 : 4);
    L.esc = k == (L.method ? 31u : 15u);
    L.k = k;
    L.escw = 0;
    if (L.esc) {
        L.escw = br.read(5);
        if (L.escw > (uint32_t)Kind<KIND>::W) set_err<KIND>(L, br, E_OUT_OF_DOMAIN);  // read_signed_integer assert
    } else if (k >= (uint32_t)Kind<KIND>::W) {
        set_err<KIND>(L, br, E_OUT_OF_DOMAIN);  // :656 unreachable
    }
    L.left = L.psize;
    L.parts_left--;
}

// Residual header (src/zflac.zig:614-633)
template <int KIND>
__device__ inline void read_residual_header(LaneCtx& L, BitReader& br) {
    const uint32_t method = br.read(2);
    if (method >= 2) { set_err<KIND>(L, br, E_INVALID_RESIDUAL_CODING); return; }
    L.method = (int)method;
    const uint32_t po = br.read(4);
    L.psize = L.bs >> po;
    // :626 `count -= order` underflow; :623-632 stale residuals when bs % 2^po != 0
    if (L.psize < (uint32_t)L.order || (L.psize << po) != L.bs) { set_err<KIND>(L, br, E_OUT_OF_DOMAIN); return; }
    L.parts_left = 1u << po;
    read_partition_header<KIND>(L, br);
    L.left = L.psize - (uint32_t)L.order;
}

// Rice code with the generic slow path (long unary / long code). Returns the residual
// in InterType arithmetic (src/zflac.zig:657-663).
template <int KIND>
__device__ inline int64_t rice_general(LaneCtx& L, BitReader& br) {
    uint32_t q;
    if (!br.unary(L.end, q)) { set_err<KIND>(L, br, E_END_OF_STREAM); return 0; }
    const uint32_t rem = br.read(L.k);
    if constexpr (Kind<KIND>::W == 64) {
        const uint64_t zz = ((uint64_t)q << L.k) + rem;
        return (int64_t)((zz >> 1) ^ (0 - (zz & 1)));
    } else if constexpr (Kind<KIND>::W == 32) {
        const uint32_t zz = (q << L.k) + rem;
        return (int32_t)((zz >> 1) ^ (0u - (zz & 1)));
    } else {
        if (q > 0xFFFFu) set_err<KIND>(L, br, E_OUT_OF_DOMAIN);  // @intCast to u16
        const uint32_t zz = ((q << L.k) + rem) & 0xFFFFu;
        return (int16_t)((zz >> 1) ^ (0u - (zz & 1)));
    }
}

// One residual in the lane's current partition (escape or Rice), generic path.
template <int KIND>
__device__ inline int64_t residual_general(LaneCtx& L, BitReader& br) {
    if (L.esc) {
        if (!L.escw) return 0;
        return br.read_signed(L.escw);
    }
    const uint32_t h = br.hi();
    const uint32_t q = __clz(h);
    const uint32_t len = q + 1 + L.k;
    if (len <= 32) {  // fast code
        const uint32_t rem = __builtin_amdgcn_ubfe(h, 32 - len, L.k);
        br.consume(len);
        const uint32_t zz = (q << L.k) | rem;
        if constexpr (Kind<KIND>::W == 16) return (int16_t)((zz >> 1) ^ (0u - (zz & 1)));
        else return (int32_t)((zz >> 1) ^ (0u - (zz & 1)));
    }
    return rice_general<KIND>(L, br);
}

// Walk one subframe without producing samples: returns its end (subframe c+1 start).
// Mirrors the reads of src/zflac.zig:426-541 and :614-666.
template <int KIND>
__device__ inline void walk_subframe(LaneCtx& L, BitReader& br) {
    const uint32_t h8 = br.read(8);
    if (h8 >> 7) { set_err<KIND>(L, br, E_INVALID_SUBFRAME_HEADER); return; }
    const uint32_t type = (h8 >> 1) & 63;
    int wasted = 0;
    if (h8 & 1) {
        uint32_t u;
        if (!br.unary(L.end, u)) { set_err<KIND>(L, br, E_END_OF_STREAM); return; }
        if (u + 1 >= 64) { set_err<KIND>(L, br, E_OUT_OF_DOMAIN); return; }
        wasted = (int)u + 1;
    }
    if (type == 0) {
        if (L.bps <= wasted) { set_err<KIND>(L, br, E_OUT_OF_DOMAIN); return; }
        br.skip((uint32_t)(L.bps - wasted));
        return;
    }
    if (L.ubps <= wasted) { set_err<KIND>(L, br, E_OUT_OF_DOMAIN); return; }
    const uint32_t cb = (uint32_t)(L.ubps - wasted);
    if (type == 1) {
        br.skip((uint64_t)L.bs * cb);
        return;
    }
    int order;
    if (type >= 8 && type <= 12) {
        order = (int)type - 8;
        br.skip((uint64_t)order * cb);
    } else if (type >= 32) {
        order = (int)type - 31;
        br.skip((uint64_t)order * cb);
        const uint32_t pc = br.read(4);
        if (pc == 15) { set_err<KIND>(L, br, E_OUT_OF_DOMAIN); return; }
        br.read(5);
        br.skip((uint64_t)order * (pc + 1));
    } else {
        set_err<KIND>(L, br, E_INVALID_SUBFRAME_HEADER);
        return;
    }
    L.order = order;
    read_residual_header<KIND>(L, br);
    if (L.err) return;
    for (;;) {
        uint32_t n = L.left;
        if (L.esc) {
            br.skip((uint64_t)n * L.escw);
        } else {
            const uint32_t k = L.k;
            for (uint32_t i = 0; i < n; i++) {
                const uint32_t h = br.hi();
                const uint32_t q = __clz(h);
                const uint32_t len = q + 1 + k;
                if (len <= 32) {
                    br.consume(len);
                } else {
                    uint32_t qq;
                    if (!br.unary(L.end, qq)) { set_err<KIND>(L, br, E_END_OF_STREAM); return; }
                    br.read(k);
                }
            }
        }
        if (br.pos() > L.end) { set_err<KIND>(L, br, E_END_OF_STREAM); return; }
        if (!L.parts_left) break;
        read_partition_header<KIND>(L, br);
        if (L.err) return;
    }
}

// Full subframe header for decoding (src/zflac.zig:426-520): warm-up samples go to
// ring[0..order-1] (ring slot = sample index mod M), coefficients to coef[j] which
// multiplies s[i-1-j] (zflac stores them reversed, :512-514; same products).
template <int KIND, int M>
__device__ inline void parse_subframe(LaneCtx& L, BitReader& br, int32_t (&ring)[M], int32_t (&coef)[M]) {
    L.mode = M_NONE;
    const uint32_t h8 = br.read(8);
    if (h8 >> 7) { set_err<KIND>(L, br, E_INVALID_SUBFRAME_HEADER); return; }  // :431
    const uint32_t type = (h8 >> 1) & 63;
    int wasted = 0;
    if (h8 & 1) {  // :433
        uint32_t u;
        if (!br.unary(L.end, u)) { set_err<KIND>(L, br, E_END_OF_STREAM); return; }
        if (u + 1 >= 64) { set_err<KIND>(L, br, E_OUT_OF_DOMAIN); return; }
        wasted = (int)u + 1;
    }
    L.wasted = wasted;
    if (type == 0) {  // constant: reads bits_per_sample, not the side depth (:447)
        if (L.bps <= wasted || L.bps - wasted > Kind<KIND>::W || wasted >= Kind<KIND>::SB) {
            set_err<KIND>(L, br, E_OUT_OF_DOMAIN);
            return;
        }
        const int64_t v = br.read_signed_wide((uint32_t)(L.bps - wasted));
        L.cval = wrap_st<KIND>((int64_t)((uint64_t)v << wasted));
        L.mode = M_CONST;
        return;
    }
    if (L.ubps <= wasted || L.ubps - wasted > Kind<KIND>::W || (wasted > 0 && wasted >= Kind<KIND>::SB)) {
        set_err<KIND>(L, br, E_OUT_OF_DOMAIN);
        return;
    }
    L.cbps = L.ubps - wasted;
    if (type == 1) {  // verbatim (:455-465)
        L.mode = M_VERB;
        return;
    }
#pragma unroll
    for (int j = 0; j < M; j++) {
        ring[j] = 0;
        coef[j] = 0;
    }
    int order;
    if (type >= 8 && type <= 12) {  // fixed (:466-490) as LPC with shift 0
        order = (int)type - 8;
#pragma unroll
        for (int j = 0; j < M; j++)
            if (j < order) ring[j] = (int32_t)br.read_signed_wide((uint32_t)L.cbps);
        if (order == 1) coef[0] = 1;
        if (order == 2) { coef[0] = 2; if (M > 1) coef[1] = -1; }
        if (order == 3) { coef[0] = 3; if (M > 2) { coef[1] = -3; coef[2] = 1; } }
        if (order == 4) { coef[0] = 4; if (M > 3) { coef[1] = -6; coef[2] = 4; coef[3] = -1; } }
        L.shift = 0;
    } else if (type >= 32) {  // LPC (:499-520)
        order = (int)type - 31;
#pragma unroll
        for (int j = 0; j < M; j++)
            if (j < order) ring[j] = (int32_t)br.read_signed_wide((uint32_t)L.cbps);
        const uint32_t pc = br.read(4);
        if (pc == 15) { set_err<KIND>(L, br, E_OUT_OF_DOMAIN); return; }  // u4 `+ 1` overflow (:508)
        const uint32_t prec = pc + 1;
        L.shift = (int)br.read(5);  // unsigned u5 (:510)
        if (L.shift >= Kind<KIND>::W) { set_err<KIND>(L, br, E_OUT_OF_DOMAIN); return; }
#pragma unroll
        for (int j = 0; j < M; j++)
            if (j < order) coef[j] = br.read_signed(prec);
    } else {
        set_err<KIND>(L, br, E_INVALID_SUBFRAME_HEADER);  // reserved (:542)
        return;
    }
    L.order = order;
    read_residual_header<KIND>(L, br);
    if (L.err) return;
    L.mode = M_PRED;
}

// Prediction from the ring: sum_j coef[j] * s[i-1-j], in InterType, then >> shift.
template <int KIND, int M, int U>
__device__ __forceinline__ int64_t predict(const int32_t (&ring)[M], const int32_t (&coef)[M], int shift) {
    if constexpr (Kind<KIND>::W == 64) {
        int64_t acc = 0;
#pragma unroll
        for (int j = 0; j < M; j++) acc += (int64_t)coef[j] * (int64_t)ring[((U - 1 - j) % M + M) % M];
        return acc >> shift;
    } else {
        int32_t acc = 0;
#pragma unroll
        for (int j = 0; j < M; j++) acc += __mul24(coef[j], ring[((U - 1 - j) % M + M) % M]);
        if constexpr (Kind<KIND>::W == 16) acc = (int16_t)acc;
        return acc >> shift;
    }
}

// Stereo decorrelation for lane c (0/1) of a pair, given x0 = channel-0 value and
// x1 = channel-1 value (src/zflac.zig:553-578).
template <int KIND>
__device__ __forceinline__ int32_t decorrelate(uint32_t code, int c, int32_t x0, int32_t x1) {
    if (code == 10) {  // mid/side in InterType
        if constexpr (KIND == 2) {
            const int64_t mid = ((int64_t)x0 * 2) | (x1 & 1);
            return (int32_t)((mid + (c ? -(int64_t)x1 : (int64_t)x1)) >> 1);
        } else {
            const int32_t mid = (x0 * 2) | (x1 & 1);
            return (mid + (c ? -x1 : x1)) >> 1;
        }
    }
    if (code == 8) return c ? x0 - x1 : x0;  // left/side: R = L - S
    if (code == 9) return c ? x1 : x0 + x1;  // side/right: L = S + R
    return c ? x1 : x0;
}

struct FrameCtx {
    uint64_t out_elem;   // absolute output element of sample 0, channel 0
    bool write;
    bool packed;         // 16-byte aligned, packed stores allowed
    uint32_t justify;
};

template <int KIND>
__device__ __forceinline__ void store_elem(void* out, uint64_t idx, int32_t v) {
    if constexpr (Kind<KIND>::ESZ == 1) reinterpret_cast<int8_t*>(out)[idx] = (int8_t)v;
    else if constexpr (Kind<KIND>::ESZ == 2) reinterpret_cast<int16_t*>(out)[idx] = (int16_t)v;
    else reinterpret_cast<int32_t*>(out)[idx] = v;
}

// exchange between lane l and l+32: returns (value of lanes 0-31 side, value of 32-63 side)
__device__ __forceinline__ void pair_values(int32_t v, int32_t& x0, int32_t& x1) {
    const auto r = __builtin_amdgcn_permlane32_swap((uint32_t)v, (uint32_t)v, false, false);
    x0 = (int32_t)r[0];
    x1 = (int32_t)r[1];
}

// Compile-time loop: f(std::integral_constant<int, I>) for I in [0, N).
template <typename F, int... Is>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, Is...>) {
    (f(std::integral_constant<int, Is>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
    static_for_impl(f, std::make_integer_sequence<int, N>{});
}

template <int KIND>
__device__ __forceinline__ int32_t add_inter(int64_t r, int64_t p) {
    if constexpr (Kind<KIND>::W == 16) return (int16_t)(r + p);
    else if constexpr (Kind<KIND>::W == 32) return (int32_t)((uint32_t)r + (uint32_t)p);
    else return (int32_t)(r + p);
}

// Generic (slow) chunk: per-sample handling of every mode, partition switches,
// warm-up and escapes; scalar stores. Called in wave-uniform control flow.
template <int KIND, int M, int L_>
__device__ inline void slow_chunk(LaneCtx& L, BitReader& br, int32_t (&ring)[M], const int32_t (&coef)[M],
                                  uint32_t base, const FrameCtx& fc, void* out, int nch, int c, bool stereo_pair) {
    static_for<L_>([&](auto uc) {
        constexpr int u = decltype(uc)::value;
        const uint32_t i = base + u;
        const bool act = L.mode != M_NONE && i < L.bs;
        int32_t val = 0;
        if (act) {
            if (L.mode == M_CONST) {
                val = L.cval;
            } else if (L.mode == M_VERB) {
                const int64_t v = br.read_signed_wide((uint32_t)L.cbps);
                val = wrap_st<KIND>((int64_t)((uint64_t)v << L.wasted));
            } else {
                int32_t s;
                if (i < (uint32_t)L.order) {
                    s = ring[u % M];
                } else {
                    if (L.left == 0) {
                        if (L.parts_left == 0) set_err<KIND>(L, br, E_OUT_OF_DOMAIN);
                        else read_partition_header<KIND>(L, br);
                    }
                    const int64_t r = residual_general<KIND>(L, br);
                    L.left--;
                    s = add_inter<KIND>(r, predict<KIND, M, u % M>(ring, coef, L.shift));
                }
                ring[u % M] = s;
                val = wrap_st<KIND>((int64_t)((uint64_t)(int64_t)s << L.wasted));
            }
        }
        int32_t o = val;
        if (stereo_pair) {
            int32_t x0, x1;
            pair_values(val, x0, x1);
            o = decorrelate<KIND>(L.chan_code, c, x0, x1);
        }
        if (act && fc.write) store_elem<KIND>(out, fc.out_elem + (uint64_t)nch * i + c, o << fc.justify);
    });
}

// Fast chunk: every active lane is a predicted subframe with >= L_ Rice codes left in
// its partition. Fully unrolled: ring slots and coefficient registers are static.
// Lanes that are not `lane_fast` run the same instruction stream on a forced 1-bit
// code and store nothing (the wave stays converged for the half-wave exchanges).
template <int KIND, int M, int L_>
__device__ inline void fast_chunk(LaneCtx& L, BitReader& br, int32_t (&ring)[M], const int32_t (&coef)[M],
                                  uint32_t base, const FrameCtx& fc, void* out, int nch, int c, bool stereo_pair,
                                  bool lane_fast) {
    const uint32_t inact = lane_fast ? 0u : 0x80000000u;
    const uint32_t k = lane_fast ? L.k : 0u;
    const int shift = L.shift;
    const int wasted = L.wasted;
    const bool do_store = lane_fast && fc.write;
    uint32_t pk[4] = {0, 0, 0, 0};  // own channel's 8 samples as 16-bit pairs (KIND 1)
    static_for<L_>([&](auto uc) {
        constexpr int u = decltype(uc)::value;
        const uint32_t i = base + u;
        // Rice code (src/zflac.zig:657-663) from one 32-bit peek
        const uint32_t h = br.hi() | inact;
        const uint32_t q = __clz(h);
        const uint32_t len = q + 1 + k;
        int64_t r;
        if (__builtin_expect(len > 32, 0)) {
            r = rice_general<KIND>(L, br);
        } else {
            const uint32_t rem = __builtin_amdgcn_ubfe(h, 32 - len, k);
            br.consume(len);
            const uint32_t zz = (q << k) | rem;
            if constexpr (Kind<KIND>::W == 16) r = (int16_t)((zz >> 1) ^ (0u - (zz & 1)));
            else r = (int32_t)((zz >> 1) ^ (0u - (zz & 1)));
        }
        const int32_t s = add_inter<KIND>(r, predict<KIND, M, u % M>(ring, coef, shift));
        ring[u % M] = s;
        const int32_t val = wrap_st<KIND>((int64_t)((uint64_t)(int64_t)s << wasted));
        int32_t o = val;
        if (stereo_pair) {
            int32_t x0, x1;
            pair_values(val, x0, x1);
            o = decorrelate<KIND>(L.chan_code, c, x0, x1);
        }
        o <<= fc.justify;
        if constexpr (KIND == 1) {
            if (nch <= 2) {  // launch-uniform
                if constexpr ((u & 1) == 0) pk[(u & 7) >> 1] = (uint32_t)o & 0xFFFFu;
                else pk[(u & 7) >> 1] |= (uint32_t)o << 16;
                if constexpr ((u & 7) == 7) {
                    const uint32_t i0 = i - 7;
                    if (stereo_pair) {
                        // lanes 0-31 hold L0..L7, lanes 32-63 R0..R7 of the same frames. After
                        // the swaps lanes 0-31 own pairs 0-3, lanes 32-63 pairs 4-7: a = L, b = R.
                        const auto s0 = __builtin_amdgcn_permlane32_swap(pk[0], pk[2], false, false);
                        const auto s1 = __builtin_amdgcn_permlane32_swap(pk[1], pk[3], false, false);
                        const uint32_t a0 = s0[0], b0 = s0[1], a1 = s1[0], b1 = s1[1];
                        uint4 v;
                        v.x = __builtin_amdgcn_perm(b0, a0, 0x05040100u);
                        v.y = __builtin_amdgcn_perm(b0, a0, 0x07060302u);
                        v.z = __builtin_amdgcn_perm(b1, a1, 0x05040100u);
                        v.w = __builtin_amdgcn_perm(b1, a1, 0x07060302u);
                        if (do_store) {
                            int16_t* dst = reinterpret_cast<int16_t*>(out) + fc.out_elem + 2ull * i0 + (c ? 8 : 0);
                            *reinterpret_cast<uint4*>(dst) = v;
                        }
                    } else if (do_store) {
                        int16_t* dst = reinterpret_cast<int16_t*>(out) + fc.out_elem + i0;
                        *reinterpret_cast<uint4*>(dst) = make_uint4(pk[0], pk[1], pk[2], pk[3]);
                    }
                }
                return;
            }
        }
        if (do_store) store_elem<KIND>(out, fc.out_elem + (uint64_t)nch * i + c, o);
    });
}

template <int KIND, int M>
__device__ inline void decode_subframe(LaneCtx& L, BitReader& br, const FrameCtx& fc, void* out, int nch, int c,
                                       bool stereo_pair, uint32_t bs_max) {
    constexpr int L_ = M < 8 ? 8 : M;
    int32_t ring[M];
    int32_t coef[M];
#pragma unroll
    for (int j = 0; j < M; j++) {
        ring[j] = 0;
        coef[j] = 0;
    }
    if (L.mode != M_NONE) parse_subframe<KIND, M>(L, br, ring, coef);
    const bool need_pack = KIND == 1 && nch <= 2;
    for (uint32_t base = 0; base < bs_max; base += L_) {
        if (L.mode == M_PRED && base < L.bs && base >= (uint32_t)L.order && L.left == 0 && L.parts_left > 0)
            read_partition_header<KIND>(L, br);
        if (L.mode != M_NONE && br.pos() > L.end) set_err<KIND>(L, br, E_END_OF_STREAM);
        const bool active = L.mode != M_NONE && base < L.bs;
        const bool lane_fast = active && base + L_ <= L.bs && L.mode == M_PRED && !L.esc &&
                               L.left >= (uint32_t)L_ && base >= (uint32_t)L.order && (!need_pack || fc.packed);
        const bool need_slow = active && !lane_fast;
        if (__builtin_amdgcn_ballot_w64(need_slow) == 0) {
            // lanes that are not fast (finished or idle) run the chunk on a scratch reader
            const BitReader keep = br;
            fast_chunk<KIND, M, L_>(L, br, ring, coef, base, fc, out, nch, c, stereo_pair, lane_fast);
            if (lane_fast) L.left -= L_;
            else br = keep;
        } else {
            slow_chunk<KIND, M, L_>(L, br, ring, coef, base, fc, out, nch, c, stereo_pair);
        }
    }
    if (L.mode != M_NONE && br.pos() > L.end) set_err<KIND>(L, br, E_END_OF_STREAM);
}

// ----------------------------------------------------------------------------------
// k_decode
// ----------------------------------------------------------------------------------
constexpr int DEC_THREADS = 256;

template <int KIND>
__global__ __launch_bounds__(DEC_THREADS) void k_decode(DecodeArgs a) {
    const int lane = threadIdx.x & 63;
    const uint32_t wave = (blockIdx.x * DEC_THREADS + threadIdx.x) >> 6;
    const uint32_t nwaves = (gridDim.x * DEC_THREADS) >> 6;
    const int nch = a.nch;
    const int F = 64 / nch;
    const int c = lane / F;
    const int j = lane - c * F;
    const bool lane_ok = c < nch;
    uint32_t nframes = a.n_frames ? *a.n_frames : a.n_frames_host;
    if (nframes > a.cap) nframes = a.cap;
    const bool stereo_pair = nch == 2;

    for (uint32_t g0 = wave * (uint32_t)F; g0 < nframes; g0 += nwaves * (uint32_t)F) {
        const uint32_t f = g0 + (uint32_t)j;
        const bool fvalid = lane_ok && f < nframes;
        LaneCtx L = {};
        FrameCtx fc = {};
        BitReader br;
        br.base = reinterpret_cast<const uint32_t*>(a.in);
        br.bb = 0;
        br.nb = 64;
        br.w1 = 0;
        br.wnext = 0;
        br.wmax = 0;
        uint64_t pos = 0;
        uint32_t hdr_info = 0, rate = 0, start = 0;
        bool frame_ok = false;  // header fine: this lane decodes its subframe
        if (fvalid) {
            pos = a.c_pos[f];
            const StreamDesc S = a.streams[a.c_stream[f]];
            const FrameHdr h = parse_frame_header(a.in + pos, S.in_end > pos ? S.in_end - pos : 0, S.si_rate);
            rate = h.rate;
            hdr_info = ((h.bs - 1) & 0xFFFFu) | (h.chan_code << 16) | (h.dcode << 20);
            L.bs = h.bs;
            L.chan_code = h.chan_code;
            L.bps = depth_bits(h.dcode, S.si_bps);
            if (h.err) {
                L.err = h.err;
                hdr_info |= INFO_PRE_ERR;
            } else if (h.crc_eof) {
                L.err = E_END_OF_STREAM;
                hdr_info |= INFO_CRC_EOF;
            } else if (channels_count(h.chan_code) != nch) {
                L.err = E_INCONSISTENT_PARAMETERS;
            } else if (L.bps < 0) {
                L.err = E_OUT_OF_DOMAIN;  // reserved depth code: `unreachable` (:143)
            } else {
                frame_ok = true;
            }
            const bool side = (h.chan_code == 8 && c == 1) || (h.chan_code == 9 && c == 0) ||
                              (h.chan_code == 10 && c == 1);
            L.ubps = L.bps + (side ? 1 : 0);
            const uint64_t abase = pos & ~(uint64_t)3;
            const uint64_t end_bytes = S.in_end > abase ? S.in_end - abase : 0;
            L.end = end_bytes * 8 > 0xFFFF0000ull ? 0xFFFF0000u : (uint32_t)(end_bytes * 8);
            const uint64_t words_avail = (S.in_end + INPUT_PAD - abase) / 4;
            br.base = reinterpret_cast<const uint32_t*>(a.in + abase);
            br.wmax = words_avail > 0x3FFFFFFFull ? 0x3FFFFFFFu : (uint32_t)words_avail - 1;
            start = ((uint32_t)(pos & 3) + h.hdr_len) * 8;
            const uint64_t rel = a.c_out[f] - S.out_base;
            const bool in_range = !S.valid_total || rel < S.total;
            fc.out_elem = a.c_out[f];
            fc.write = a.write && in_range && frame_ok && rel + (uint64_t)h.bs * nch <= S.out_cap;
            fc.packed = (fc.out_elem & 7) == 0;
            fc.justify = S.justify;
        }
        // ---- walk: subframe c+1 starts where subframe c ends --------------------------
        for (int r = 0; r + 1 < nch; r++) {
            uint32_t e = 0;
            if (c == r && frame_ok) {
                LaneCtx W = L;
                W.mode = M_PRED;
                br.init(br.base, start, br.wmax);
                walk_subframe<KIND>(W, br);
                e = br.pos();
            }
            const int src = lane - F;
            const uint32_t e_in = (uint32_t)__shfl((int)e, src < 0 ? 0 : src);
            if (c == r + 1) start = e_in;
        }
        // ---- decode ------------------------------------------------------------------
        if (frame_ok) {
            L.mode = M_PRED;  // active marker until the subframe header is parsed
            br.init(br.base, start, br.wmax);
        }
        uint32_t ord = 0, bs_act = 0;
        if (L.mode != M_NONE) {  // peek the subframe type (header bits 1..6) to size the ring
            const uint32_t t = (br.hi() >> 25) & 63;
            ord = (t >= 32) ? t - 31 : ((t >= 8 && t <= 12) ? t - 8 : 0);
            bs_act = L.bs;
        }
        for (int o = 32; o > 0; o >>= 1) {
            ord = max(ord, (uint32_t)__shfl_xor((int)ord, o));
            bs_act = max(bs_act, (uint32_t)__shfl_xor((int)bs_act, o));
        }
        if (ord <= 4) decode_subframe<KIND, 4>(L, br, fc, a.out, nch, c, stereo_pair, bs_act);
        else if (ord <= 8) decode_subframe<KIND, 8>(L, br, fc, a.out, nch, c, stereo_pair, bs_act);
        else if (ord <= 16) decode_subframe<KIND, 16>(L, br, fc, a.out, nch, c, stereo_pair, bs_act);
        else decode_subframe<KIND, 32>(L, br, fc, a.out, nch, c, stereo_pair, bs_act);

        // ---- frame end and record -------------------------------------------------------
        uint32_t endbits = (uint32_t)((br.pos() + 7) & ~7u);  // alignToByte (:546)
        if (frame_ok && !L.err && c == nch - 1 && endbits + 16 > L.end) L.err = E_END_OF_STREAM;  // CRC-16 (:548)
        int ferr = 0;  // first error in channel order
        for (int cc = nch - 1; cc >= 0; cc--) {
            const int e = __shfl(L.err, cc * F + j);
            if (e) ferr = e;
        }
        const uint32_t last_end = (uint32_t)__shfl((int)endbits, (nch - 1) * F + j);
        if (fvalid && c == 0) {
            a.c_err[f] = ferr;
            a.c_info[f] = hdr_info;
            a.c_rate[f] = rate;
            a.c_end[f] = (pos & ~(uint64_t)3) + last_end / 8 + 2;
        }
    }
}

// ----------------------------------------------------------------------------------
// k_verify: is the candidate chain what zflac's frame loop would walk? (see header)
// ----------------------------------------------------------------------------------
__global__ void k_verify(VerifyArgs a) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t nframes = *a.n_frames;
    if (nframes > a.cap) nframes = a.cap;
    if (t < a.n_streams) {
        const StreamDesc S = a.streams[t];
        const uint32_t f0 = a.chunk_off[S.first_chunk], f1 = a.chunk_off[S.end_chunk];
        if (f1 <= f0 || f1 > nframes || !S.valid_total || a.c_pos[f0] != S.in_begin) atomicOr(&a.status[t], 1u);
    }
    if (t >= nframes) return;
    const uint32_t s = a.c_stream[t];
    const StreamDesc S = a.streams[s];
    const uint32_t f1 = min(a.chunk_off[S.end_chunk], nframes);
    const uint64_t rel = a.c_out[t] - S.out_base;
    if (S.valid_total && rel >= S.total) return;  // past the last sample: never read (:341)
    bool bad = a.c_err[t] != 0;
    const uint32_t info = a.c_info[t];
    const uint32_t bs = (info & 0xFFFF) + 1;
    const uint32_t code = (info >> 16) & 15, dcode = (info >> 20) & 7;
    if ((uint32_t)channels_count(code) != S.nch || dcode != S.dcode || a.c_rate[t] != S.rate_hz) bad = true;
    const uint64_t units = (uint64_t)bs * S.nch;
    if (bs == 1 && rel + S.nch < S.total) bad = true;  // :405
    const uint64_t end_rel = rel + units;
    if (end_rel > S.total || end_rel > S.out_cap) bad = true;     // zflac would grow the buffer
    if (end_rel < S.total && (t + 1 >= f1 || a.c_pos[t + 1] != a.c_end[t])) bad = true;
    if (bad) atomicOr(&a.status[s], 1u);
}

// ----------------------------------------------------------------------------------
// launchers
// ----------------------------------------------------------------------------------
hipError_t launch_scan(const ScanArgs& a, hipStream_t st) {
    if (a.n_chunks == 0) return hipSuccess;
    hipLaunchKernelGGL(k_scan, dim3(a.n_chunks), dim3(SCAN_THREADS), 0, st, a);
    return hipGetLastError();
}
hipError_t launch_scan_chunks(const uint32_t* cnt, const unsigned long long* units, uint32_t n, uint32_t* off,
                              unsigned long long* uoff, uint32_t* n_frames, hipStream_t st) {
    hipLaunchKernelGGL(k_scan_chunks, dim3(1), dim3(SCANK_THREADS), 0, st, cnt, units, n, off, uoff, n_frames);
    return hipGetLastError();
}
hipError_t launch_compact(const CompactArgs& a, hipStream_t st) {
    if (a.n_chunks == 0) return hipSuccess;
    hipLaunchKernelGGL(k_compact, dim3(a.n_chunks), dim3(SCAN_THREADS), 0, st, a);
    return hipGetLastError();
}
hipError_t launch_decode(int kind, const DecodeArgs& a, uint32_t max_frames, hipStream_t st) {
    const uint32_t F = 64 / a.nch;
    uint32_t waves = (max_frames + F - 1) / F;
    uint32_t blocks = (waves + 3) / 4;
    if (blocks > 4096) blocks = 4096;
    if (blocks == 0) blocks = 1;
    if (kind == 0) hipLaunchKernelGGL(k_decode<0>, dim3(blocks), dim3(DEC_THREADS), 0, st, a);
    else if (kind == 1) hipLaunchKernelGGL(k_decode<1>, dim3(blocks), dim3(DEC_THREADS), 0, st, a);
    else hipLaunchKernelGGL(k_decode<2>, dim3(blocks), dim3(DEC_THREADS), 0, st, a);
    return hipGetLastError();
}
hipError_t launch_verify(const VerifyArgs& a, uint32_t max_items, hipStream_t st) {
    uint32_t n = max_items > a.n_streams ? max_items : a.n_streams;
    uint32_t blocks = (n + 255) / 256;
    if (blocks == 0) blocks = 1;
    hipLaunchKernelGGL(k_verify, dim3(blocks), dim3(256), 0, st, a);
    return hipGetLastError();
}

}  // namespace zflac
