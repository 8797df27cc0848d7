// walk_wave.hip -- k_walk_wave: where subframe c >= 1 of each frame starts, one WAVE per frame.
//
// Subframe c+1 starts where subframe c ends (src/zflac.zig:425-541 read order), so before
// subframe c >= 1 can be decoded the bit length of subframes 0..c-1 must be known. k_walk
// (decode.inc) gives each lane one frame: 64 independent serial chains per wave, the right
// shape when a launch has tens of thousands of frames. This kernel is the other shape: a
// whole wave walks one frame, so a launch with few frames (one stream of a few thousand
// frames, the sequential planner's probes) or with several subframes to walk per frame
// (3..8 channels) still fills the chip and each frame's walk is short.
//
// Subframe headers, warm-up / coefficient skips and partition headers are read
// wave-uniformly. The Rice codes of a partition (src/zflac.zig:655-664: unary q, a 1, k
// bits) are found by a wave-wide scan of the next 4096 bits: lane i takes words 2i, 2i+1 and, for
// an entry offset e, follows the codes through its two words (clz per code: ffs over the
// segment) to the offset x where the next code starts in lane i+1's segment, recording the
// set V of code starts it visited. Entries are guessed and corrected (Jacobi rounds with a ballot for
// convergence): lane i's entry is lane i-1's exit; if it is in V the lane's chain has
// already merged with the true one, otherwise the lane re-runs from it. Rice codes
// resynchronise within a few codes, so a few rounds settle all 64 lanes. The codes each lane
// completes are then summed by a wave prefix scan, which locates the partition's last code.
// Lane i scans two words (64 bits, ~7 codes at C3's k): a chain from a wrong entry merges
// with the true one within the segment ~70 % of the time, so ~4 rounds settle the wave, and
// one pass covers 4096 bits, a whole partition of C3.
#include "device_common.h"

namespace zflac {
namespace {

constexpr int WW_THREADS = 256;  // 4 waves (frames) per workgroup
constexpr int WBUFFER_RSRC_WORD3 = 0x00020000;  // raw buffer, 32-bit data format (as decode.inc)

template <int KIND>
struct WKind;
template <>
struct WKind<0> {
    static constexpr int W = 16;  // InterType bits (Rice k and escape width limits)
};
template <>
struct WKind<1> {
    static constexpr int W = 32;
};
template <>
struct WKind<2> {
    static constexpr int W = 64;
};

__device__ __forceinline__ uint32_t lane_id() { return threadIdx.x & 63u; }
__device__ __forceinline__ uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

// The frame's bytes as big-endian words, a 320-word window: lane i holds words wb + 64 m + i
// in r_m. Words wb .. wb + 191 are read (r0..r2); r3, r4 are in flight for the next 128
// words, so a pass that moves on by a whole 4096-bit scan finds them resident. Word indices
// count from the frame's 16-byte aligned base; loads past the input buffer read zeros
// (buffer range check).
struct WaveWin {
    __amdgpu_buffer_rsrc_t rs;
    uint32_t nwords;  // words inside the buffer resource
    uint32_t wb;      // wave-uniform
    uint32_t r0, r1, r2, r3, r4;

    __device__ __forceinline__ uint32_t load(uint32_t w) const {
        const uint32_t off = w < nwords ? w * 4u : 0x80000000u;
        return bswap32((uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rs, off, 0, 0));
    }
    __device__ __forceinline__ void init(uint32_t w0) {
        wb = uni(w0);
        r0 = load(wb + lane_id());
        r1 = load(wb + 64u + lane_id());
        r2 = load(wb + 128u + lane_id());
        r3 = load(wb + 192u + lane_id());
        r4 = load(wb + 256u + lane_id());
    }
    __device__ __forceinline__ void slide() {
        r0 = r1;
        r1 = r2;
        r2 = r3;
        r3 = r4;
        wb = uni(wb + 64u);
        r4 = load(wb + 256u + lane_id());
    }
    // make words w .. w + 127 readable: w - wb < 64 (w only grows)
    __device__ __forceinline__ void reach(uint32_t w) {
        for (int i = 0; i < 4 && w >= wb + 64u; i++) slide();
        if (w >= wb + 64u) init(w);
    }
    __device__ __forceinline__ uint32_t word(uint32_t w) const {  // wb <= w < wb + 192, uniform
        const uint32_t j = uni(w - wb);
        const uint32_t v = j < 64u ? r0 : (j < 128u ? r1 : r2);
        return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)(j & 63u));
    }
    __device__ __forceinline__ uint32_t byte(uint32_t b) const {  // byte b from the base, uniform
        return (word(wb + (b >> 2)) >> (24u - 8u * (b & 3u))) & 0xFFu;
    }
    // the 32 bits at bit position P (MSB first)
    __device__ __forceinline__ uint32_t peek(uint32_t P) {
        const uint32_t w = P >> 5, o = P & 31u;
        reach(w);
        const uint32_t hi = word(w), lo = word(w + 1u);
        return o ? (hi << o) | (lo >> (32u - o)) : hi;
    }
    __device__ __forceinline__ uint32_t bits(uint32_t& P, uint32_t n) {  // 0 <= n <= 32
        const uint32_t v = n ? peek(P) >> (32u - n) : 0u;
        P += n;
        return v;
    }
    __device__ __forceinline__ uint32_t at(uint32_t j) const {  // window word j (< 192) to this lane
        const int src = (int)(j & 63u);
        const uint32_t a = (uint32_t)__shfl((int)r0, src), b = (uint32_t)__shfl((int)r1, src),
                       c = (uint32_t)__shfl((int)r2, src);
        return j < 64u ? a : (j < 128u ? b : c);
    }
    // lane i gets words (P >> 5) + 2i and + 2i + 1: the 4096 bits from P's word on
    __device__ __forceinline__ void from(uint32_t P, uint32_t& hi, uint32_t& lo) {
        reach(P >> 5);
        const uint32_t j0 = uni((P >> 5) - wb);
        hi = at(j0 + 2u * lane_id());
        lo = at(j0 + 2u * lane_id() + 1u);
    }
};

// Codes through one 64-bit segment (hi, lo) from entry offset e (0..63): V = code starts
// visited (bit 63 - s for start s), x = start of the next code in the following segment
// (0..31: a code's k <= 30 remainder bits end at most 31 bits past the segment), un = the
// last start's unary run continues past the segment (its code is not counted here).
__device__ __forceinline__ void chain(uint64_t w, uint32_t e, uint32_t kp1, uint64_t& V, uint32_t& x, uint32_t& un) {
    V = 0;
    un = 0;
    x = 0;
    for (int it = 0; it < 65; it++) {
        V |= 0x8000000000000000ull >> e;
        const uint64_t m = w << e;
        if (m == 0) {
            un = 1;
            x = 0;
            break;
        }
        const uint32_t e2 = e + (uint32_t)__builtin_clzll(m) + kp1;  // terminator + 1 + k
        if (e2 >= 64u) {
            x = e2 - 64u;
            break;
        }
        e = e2;
    }
}

// Inclusive prefix sum over the wave (row scans by DPP, rows joined by readlane).
__device__ __forceinline__ uint32_t wave_scan(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, true);  // row_shr:1
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, true);  // row_shr:2
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, true);  // row_shr:4
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, true);  // row_shr:8
    const uint32_t t0 = (uint32_t)__builtin_amdgcn_readlane((int)v, 15);
    const uint32_t t1 = (uint32_t)__builtin_amdgcn_readlane((int)v, 31);
    const uint32_t t2 = (uint32_t)__builtin_amdgcn_readlane((int)v, 47);
    const uint32_t l = lane_id();
    return v + (l >= 16u ? t0 : 0u) + (l >= 32u ? t1 : 0u) + (l >= 48u ? t2 : 0u);
}

// x of the lane below (DPP wave_shr:1; lane 0 gets 0)
__device__ __forceinline__ uint32_t from_below(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x138, 0xf, 0xf, true);
}

// Skip n Rice codes of parameter k starting at bit P (src/zflac.zig:655-664). False when the
// scan runs past `end` (the frame's decode then fails at EndOfStream anyway).
__device__ bool skip_rice(WaveWin& W, uint32_t& P, uint32_t n, uint32_t k, uint32_t end) {
    const uint32_t lane = lane_id();
    const uint32_t kp1 = k + 1u;
    while (n) {
        if (P > end) return false;
        uint32_t hi, lo;
        W.from(P, hi, lo);
        const uint64_t w = ((uint64_t)hi << 32) | lo;
        const uint32_t e0 = P & 31u;
        const uint32_t wbase = P & ~31u;  // bit position of lane 0's segment
        uint64_t V;
        uint32_t x, un;
        chain(w, lane == 0 ? e0 : 0u, kp1, V, x, un);
        uint32_t want = e0;
        for (int round = 0; round < 64; round++) {
            const uint32_t px = from_below(x);
            want = lane == 0 ? e0 : px;
            const bool need = lane != 0 && ((V << want) >> 63) == 0;  // want not among the visited starts
            if (__builtin_amdgcn_ballot_w64(need) == 0) break;
            if (need) chain(w, want, kp1, V, x, un);
        }
        const uint64_t Vw = V & (~0ull >> want);  // starts on the true chain
        const uint32_t cnt = (uint32_t)__builtin_popcountll(Vw) - un;
        const uint32_t cum = wave_scan(cnt);
        const uint32_t total = uni((uint32_t)__builtin_amdgcn_readlane((int)cum, 63));
        if (total < n) {
            n -= total;
            P = wbase + 4096u + uni((uint32_t)__builtin_amdgcn_readlane((int)x, 63));
            continue;
        }
        const uint64_t hit = __builtin_amdgcn_ballot_w64(cum >= n);
        const uint32_t L = uni((uint32_t)__builtin_ctzll(hit));
        const uint32_t cumL = uni((uint32_t)__builtin_amdgcn_readlane((int)cum, (int)L));
        const uint32_t cntL = uni((uint32_t)__builtin_amdgcn_readlane((int)cnt, (int)L));
        const uint32_t vh = uni((uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(Vw >> 32), (int)L));
        const uint32_t vl = uni((uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)Vw, (int)L));
        uint64_t VL = ((uint64_t)vh << 32) | vl;
        const uint32_t xL = uni((uint32_t)__builtin_amdgcn_readlane((int)x, (int)L));
        // the last code is lane L's r-th counted one; it ends where the next start is
        const uint32_t r = n - (cumL - cntL);
        for (uint32_t i = 0; i < r; i++) VL &= ~(0x8000000000000000ull >> __builtin_clzll(VL));
        P = VL ? wbase + 64u * L + (uint32_t)__builtin_clzll(VL) : wbase + 64u * (L + 1u) + xL;
        n = 0;
    }
    return true;
}

// readUnary (bit_reader.zig:95-120), wave-uniform; false past `end`
__device__ bool unary_w(WaveWin& W, uint32_t& P, uint32_t end, uint32_t& q) {
    q = 0;
    for (;;) {
        if (P > end) return false;
        const uint32_t h = W.peek(P);
        if (h) {
            const uint32_t z = (uint32_t)__builtin_clz(h);
            q += z;
            P += z + 1u;
            return P <= end;
        }
        q += 32u;
        P += 32u;
    }
}

// One subframe, same reads as walk_subframe + the residual loop of run_subframe<WALK> in
// decode.inc (src/zflac.zig:426-541, 614-666); P moves to its end. False on any error: the
// frame's decode reports it (channel 0 fails at the same read), so the recorded starts of
// later subframes do not matter then.
template <int KIND>
__device__ bool walk_subframe_w(WaveWin& W, uint32_t& P, uint32_t bs, int bps, int ubps, uint32_t end) {
    constexpr int IW = WKind<KIND>::W;
    const uint32_t h8 = W.bits(P, 8);
    if (h8 >> 7) return false;  // :431
    const uint32_t type = (h8 >> 1) & 63u;
    int wasted = 0;
    if (h8 & 1u) {
        uint32_t u;
        if (!unary_w(W, P, end, u)) return false;
        if (u + 1u >= 64u) return false;
        wasted = (int)u + 1;
    }
    if (type == 0) {  // constant: bits_per_sample - wasted (:447)
        if (bps <= wasted) return false;
        P += (uint32_t)(bps - wasted);
        return P <= end;
    }
    if (ubps <= wasted) return false;
    const uint32_t cb = (uint32_t)(ubps - wasted);
    if (type == 1) {  // verbatim
        const uint64_t np = (uint64_t)P + (uint64_t)bs * cb;
        if (np > end) return false;
        P = (uint32_t)np;
        return true;
    }
    uint32_t order;
    if (type >= 8 && type <= 12) {
        order = type - 8u;
        P += order * cb;
    } else if (type >= 32) {
        order = type - 31u;
        P += order * cb;
        if (P > end) return false;
        const uint32_t pc = W.bits(P, 4);
        if (pc == 15) return false;
        P += 5u + order * (pc + 1u);
    } else {
        return false;  // reserved (:542)
    }
    if (P > end) return false;
    const uint32_t method = W.bits(P, 2);
    if (method >= 2) return false;  // :618
    const uint32_t po = W.bits(P, 4);
    const uint32_t psize = bs >> po;
    if (psize < order || (psize << po) != bs) return false;
    const uint32_t parts = 1u << po;
    for (uint32_t p = 0; p < parts; p++) {
        if (P > end) return false;
        const uint32_t k = W.bits(P, method ? 5 : 4);
        const uint32_t n = psize - (p == 0 ? order : 0u);
        if (k == (method ? 31u : 15u)) {  // escape: 5-bit width, n raw values
            const uint32_t escw = W.bits(P, 5);
            if (escw > (uint32_t)IW) return false;
            const uint64_t np = (uint64_t)P + (uint64_t)n * escw;
            if (np > end) return false;
            P = (uint32_t)np;
        } else {
            if (k >= (uint32_t)IW) return false;  // :656
            if (!skip_rice(W, P, n, k, end)) return false;
        }
    }
    return P <= end;
}

template <int KIND>
__global__ __launch_bounds__(WW_THREADS) void k_walk_wave(DecodeArgs a) {
    const uint32_t wave = (blockIdx.x * WW_THREADS + threadIdx.x) >> 6;
    const uint32_t nwaves = (gridDim.x * WW_THREADS) >> 6;
    const int nch = a.nch;
    uint32_t nframes = a.n_frames ? *a.n_frames : a.n_frames_host;
    if (nframes > a.cap) nframes = a.cap;
    for (uint32_t f = uni(wave); f < nframes; f += nwaves) {
        const uint64_t pos = a.c_pos[f];
        const StreamDesc S = a.streams[a.c_stream[f]];
        const uint64_t abase = pos & ~(uint64_t)15;
        WaveWin W;
        const uint64_t wlen = a.in_size > abase ? a.in_size - abase : 0;
        const uint32_t rbytes = (uint32_t)(wlen > 0x7FFFFFF0ull ? 0x7FFFFFF0ull : wlen);
        W.rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(a.in) + abase, (short)0, (int)rbytes,
                                                 WBUFFER_RSRC_WORD3);
        W.nwords = rbytes / 4u;
        W.init(0);
        // the frame header from the window (its at most 16 + 16 bytes are words 0..7)
        const uint32_t hb = (uint32_t)(pos & 15);
        const FrameHdr h = parse_frame_header_t<0>([&](uint32_t i) -> uint32_t { return W.byte(hb + i); },
                                                       S.in_end > pos ? S.in_end - pos : 0, S.si_rate, nullptr);
        const int bps = depth_bits(h.dcode, S.si_bps);
        // the frame decodes only with these (setup_frame in decode.inc)
        bool ok = !h.err && !h.crc_eof && channels_count(h.chan_code) == nch && bps >= 0;
        const uint64_t end_bytes = S.in_end > abase ? S.in_end - abase : 0;
        const uint32_t end = end_bytes * 8 > 0xFFFF0000ull ? 0xFFFF0000u : (uint32_t)(end_bytes * 8);
        uint32_t P = (hb + h.hdr_len) * 8u;
        for (int c = 0; c + 1 < nch; c++) {
            if (ok) {
                const bool side = (h.chan_code == 8 && c == 1) || (h.chan_code == 9 && c == 0) ||
                                  (h.chan_code == 10 && c == 1);  // src/zflac.zig:436-441
                ok = walk_subframe_w<KIND>(W, P, h.bs, bps, bps + (side ? 1 : 0), end);
            }
            const bool frame_ok = !h.err && !h.crc_eof && channels_count(h.chan_code) == nch && bps >= 0;
            if (lane_id() == 0) a.sub_start[(uint64_t)f * MAX_CH + c + 1] = frame_ok ? P : 0u;
        }
    }
}

template <int KIND>
hipError_t launch_walk_wave_kind(const DecodeArgs& a, uint32_t max_frames, hipStream_t st) {
    uint32_t blocks = (max_frames + WW_THREADS / 64 - 1) / (WW_THREADS / 64);
    if (blocks > 16384) blocks = 16384;
    if (blocks == 0) blocks = 1;
    hipLaunchKernelGGL((k_walk_wave<KIND>), dim3(blocks), dim3(WW_THREADS), 0, st, a);
    return hipGetLastError();
}

}  // namespace

hipError_t launch_walk_wave(int kind, const DecodeArgs& a, uint32_t max_frames, hipStream_t st) {
    if (kind == 0) return launch_walk_wave_kind<0>(a, max_frames, st);
    if (kind == 1) return launch_walk_wave_kind<1>(a, max_frames, st);
    return launch_walk_wave_kind<2>(a, max_frames, st);
}

}  // namespace zflac
