// scan.hip -- frame-sync scan, candidate compaction and chain verification kernels.
//
//   k_scan          frame-sync scan: every input byte once, 16 B/lane coalesced loads;
//                   candidates = 0xFF 0xF8|F9 + exact header parse + CRC-8 + the stream's
//                   first-frame parameters. Up to CHUNK_CAP ordered candidates per 32 KiB chunk.
//   k_scan_chunks   exclusive scan of per-chunk candidate counts / sample units.
//   k_compact       ordered candidate table (position, stream, output offset).
//   k_verify        is the candidate chain exactly what zflac's sequential frame loop
//                   (src/zflac.zig:340-581) would walk? Streams failing it are finished by
//                   the host's sequential planner.
#include "device_common.h"

#ifndef ZFLAC_SCAN_AUX
#define ZFLAC_SCAN_AUX 0  // cache policy bits of k_scan's loads (experiment: 2 = nontemporal)
#endif

namespace zflac {

// ----------------------------------------------------------------------------------
// k_scan: frame-sync candidates per 32 KiB chunk
// ----------------------------------------------------------------------------------
__device__ inline uint32_t ff_mask(uint32_t d) { return ((d & 0x7F7F7F7Fu) + 0x01010101u) & d & 0x80808080u; }

// Calls fn(position) for every candidate in the 16-byte window `v` at `ws` that lies in
// [lo, hi). Windows are 16-byte aligned.
template <typename Fn>
__device__ inline void scan_window_v(const uint4 v, const uint8_t* in, uint64_t ws, uint64_t lo, uint64_t hi, Fn&& fn) {
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
template <typename Fn>
__device__ inline void scan_window(const uint8_t* in, uint64_t ws, uint64_t lo, uint64_t hi, Fn&& fn) {
    scan_window_v(*reinterpret_cast<const uint4*>(in + ws), in, ws, lo, hi, fn);
}

// A wave's 16-byte windows are consecutive per lane, so the 16 bytes after a lane's window
// are the next lane's window (DPP wave_shl:1); lane 63, and a lane whose next window lies
// past the chunk (zeroed), read them from memory.
// Bit 7 of byte i set where byte i of d is 0xFF and the byte after it (byte i + 1, or the
// first byte of dn for i = 3) is 0xF8 or 0xF9: a frame sync code (src/zflac.zig:351-352).
// Exact per byte (no borrow between bytes).
__device__ __forceinline__ uint32_t sync_mask(uint32_t d, uint32_t dn) {
    const uint32_t nxt = __builtin_amdgcn_alignbyte(dn, d, 1);  // byte i = the byte after byte i of d
    const uint32_t y = (nxt & 0xFEFEFEFEu) ^ 0xF8F8F8F8u;        // zero bytes: next is 0xF8 / 0xF9
    const uint32_t zero = ~(((y & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | y | 0x7F7F7F7Fu);
    return ff_mask(d) & zero;
}

// Nonzero iff some byte i of d is 0xFF and the byte after it 0xF8 / 0xF9: the same test as
// sync_mask, as an existence test only. Byte i of t is zero exactly at a sync code, and
// (t - 0x01..01) & ~t & 0x80..80 is nonzero iff t has a zero byte (the borrows can mark a
// byte above a zero one, never create a mark without one). ~5 VALU per dword against
// sync_mask's ~10: k_scan runs it on every window and the exact masks only where it fires
// (a sync code, or a 0xFF 0xF8|F9 pair in the coded bits: ~1 in 7 wave-windows of 1 KiB).
__device__ __forceinline__ uint32_t sync_any(uint32_t d, uint32_t dn) {
    const uint32_t nxt = __builtin_amdgcn_alignbyte(dn, d, 1);
    const uint32_t t = ~d | ((nxt & 0xFEFEFEFEu) ^ 0xF8F8F8F8u);
    return (t - 0x01010101u) & ~t & 0x80808080u;
}

// (Call at wave-uniform points: DPP reads the neighbour lane's registers.)
__device__ __forceinline__ uint32_t lane_above(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x130, 0xf, 0xf, true);  // wave_shl:1
}

// k_scan: one workgroup per 32 KiB chunk. Every lane's 8 windows are loaded at once. Sync
// codes (0xFF then 0xF8 / 0xF9) are found with exact per-byte SWAR masks over the window's
// four dwords and the next window's first one (the next lane's, DPP wave_shl:1): ~40 VALU
// per 16 bytes, and the per-candidate loop only runs at real sync codes (~1 in 64 KiB of
// compressed data). A real candidate's header (at most 16 bytes) is parsed
// from its window and the next one staged in the lane's own 32-byte LDS slot: no chain of
// dependent global byte reads, which kept each workgroup alive for several memory round
// trips.
// LDS of one chunk's scan: the candidates found (positions sorted at the end), their count
// and units.
struct ScanLds {
    uint32_t cnt;
    unsigned long long units;
    uint64_t pos[CHUNK_CAP];
    uint32_t u[CHUNK_CAP];
};


// The candidates of chunk `chunk` into L (called by the whole workgroup; ends with a barrier,
// the first min(cnt, CHUNK_CAP) positions sorted).
__device__ __forceinline__ void scan_chunk(const ScanArgs& a, uint32_t chunk, ScanLds& L) {
    const ChunkDesc ch = a.chunks[chunk];
    const uint64_t abase = ch.begin & ~(uint64_t)15;
    // all of the thread's windows in flight at once (coalesced 4 KiB rows per round); the
    // buffer unit answers reads past the chunk end with zeros (no per-load branch)
    constexpr int R = SCAN_BYTES_PER_THREAD / 16;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint8_t*>(a.in) + abase, (short)0, (int)(ch.end - abase), 0x00020000);
    uint4 v[R];
#pragma unroll
    for (int r = 0; r < R; r++)
        v[r] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, threadIdx.x * 16u,
                                                                                 r * SCAN_THREADS * 16, ZFLAC_SCAN_AUX));
    const StreamDesc S = a.streams[ch.stream];
    if (threadIdx.x == 0) {
        L.cnt = 0;
        L.units = 0;
    }
    __syncthreads();
    const uint64_t lane_ws = abase + (uint64_t)threadIdx.x * 16;
#pragma unroll
    for (int r = 0; r < R; r++) {
        const uint64_t ws = lane_ws + (uint64_t)r * SCAN_THREADS * 16;
        // a wave's windows are contiguous: the next window's first dword is the next lane's
        // (DPP), except for lane 63 and past the chunk end (zeroed), where a sync code in
        // byte 15 reads its next byte from memory (rare)
        const uint32_t n0 = lane_above(v[r].x);
        const bool nx_mem = (threadIdx.x & 63u) == 63u || ws + 16 >= ch.end;
        // cheap existence test first: the exact masks below only run in waves where some lane
        // may hold a sync code in this window (its last byte is tested against memory there).
        // The skip is a ballot, i.e. a wave-uniform branch: a per-lane condition was
        // if-converted, so every wave computed both tests (k_scan VALU 22.4M -> 23.2M).
        const bool maybe = ((sync_any(v[r].x, v[r].y) | sync_any(v[r].y, v[r].z) | sync_any(v[r].z, v[r].w) |
                             sync_any(v[r].w, n0)) != 0 ||
                            (nx_mem && (v[r].w >> 24) == 0xFFu)) &&
                           ws < ch.end;
        if (__builtin_amdgcn_ballot_w64(maybe) == 0) continue;
#if defined(ZFLAC_SCAN_ABL) && ZFLAC_SCAN_ABL == 2  // timing ablation: the existence test only
        atomicAdd(&L.cnt, 1u);
        continue;
#endif
        // the next window (the header of a sync code in this one may run into it): the next
        // lane's registers (DPP, at this wave-uniform point), from memory only where that lane
        // does not hold it (lane 63; a next window past the chunk end, which read as zeros).
        // Round 5 loaded it from memory in every candidate lane: a dependent round trip in
        // most workgroups (~3.6 frames per 32 KiB chunk of C5 data).
        const uint4 vn = make_uint4(n0, lane_above(v[r].y), lane_above(v[r].z), lane_above(v[r].w));
        if (ws >= ch.end) continue;
        const uint32_t c0 = sync_mask(v[r].x, v[r].y), c1 = sync_mask(v[r].y, v[r].z),
                       c2 = sync_mask(v[r].z, v[r].w);
        uint32_t c3 = sync_mask(v[r].w, n0);
        if (nx_mem && (v[r].w >> 24) == 0xFFu)
            c3 = (c3 & 0x00808080u) | ((a.in[ws + 16] & 0xFEu) == 0xF8u ? 0x80000000u : 0u);
        if ((c0 | c1 | c2 | c3) == 0 || ws >= ch.end) continue;  // no sync code: the common case
#if defined(ZFLAC_SCAN_ABL) && ZFLAC_SCAN_ABL == 1  // timing ablation (tools/replay.py): no header parse
        atomicAdd(&L.cnt, (uint32_t)__builtin_popcount(c0 | c1 | c2 | c3));
        continue;
#endif
        uint32_t cand = (c0 * 0x00204081u) >> 28 & 15u;  // bit b: a sync code at byte b
        cand |= ((c1 * 0x00204081u) >> 28 & 15u) << 4;
        cand |= ((c2 * 0x00204081u) >> 28 & 15u) << 8;
        cand |= ((c3 * 0x00204081u) >> 28 & 15u) << 12;
        // the header (at most 16 bytes from p) lies in this window and the next
        const uint4 nx = nx_mem ? *reinterpret_cast<const uint4*>(a.in + ws + 16) : vn;
        while (cand) {
            const uint32_t b = (uint32_t)__ffs(cand) - 1u;
            cand &= cand - 1u;
            const uint64_t p = ws + b;
            if (p < ch.begin || p >= ch.end) continue;
            // header bytes b..b+15 into four registers (little-endian words): a two-stage
            // dword shift by b >> 2, then v_alignbyte by b & 3; parsed and CRC-checked there
            // (round 5 staged the windows in LDS and parsed byte by byte with table lookups:
            // ~16 dependent LDS round trips per candidate, 15 of k_scan's 83 us)
            // (named registers, no arrays: an indexed array here became scratch / LDS)
            const bool s8 = (b & 8u) != 0, s4 = (b & 4u) != 0;
            const uint32_t x0 = s8 ? v[r].z : v[r].x, x1 = s8 ? v[r].w : v[r].y, x2 = s8 ? nx.x : v[r].z,
                           x3 = s8 ? nx.y : v[r].w, x4 = s8 ? nx.z : nx.x, x5 = s8 ? nx.w : nx.y;
            const uint32_t y0 = s4 ? x1 : x0, y1 = s4 ? x2 : x1, y2 = s4 ? x3 : x2, y3 = s4 ? x4 : x3,
                           y4 = s4 ? x5 : x4;
            const uint32_t sb = b & 3u;
            const uint32_t h0 = __builtin_amdgcn_alignbyte(y1, y0, sb), h1 = __builtin_amdgcn_alignbyte(y2, y1, sb),
                           h2 = __builtin_amdgcn_alignbyte(y3, y2, sb), h3 = __builtin_amdgcn_alignbyte(y4, y3, sb);
            const FrameHdr h = parse_frame_header_t<2>(
                [h0, h1, h2, h3](uint32_t i) -> uint32_t {  // byte i: v_perm from 8 bytes, zeros above
                    const uint32_t sel = (i & 7u) | 0x0C0C0C00u;
                    return (i & 8u) ? __builtin_amdgcn_perm(h3, h2, sel) : __builtin_amdgcn_perm(h1, h0, sel);
                },
                S.in_end - p, S.si_rate, nullptr);
            if (!candidate_ok(h, S)) continue;
            const uint32_t slot = atomicAdd(&L.cnt, 1u);
            const uint32_t units = h.bs * S.nch;
            atomicAdd(&L.units, (unsigned long long)units);
            if (slot < CHUNK_CAP) {
                L.pos[slot] = p;
                L.u[slot] = units;
            }
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t n = L.cnt;
        const uint32_t m = n < CHUNK_CAP ? n : CHUNK_CAP;
        for (uint32_t i = 1; i < m; i++) {  // insertion sort by position (m is tiny)
            uint64_t p = L.pos[i];
            uint32_t u = L.u[i];
            int j = (int)i - 1;
            while (j >= 0 && L.pos[j] > p) {
                L.pos[j + 1] = L.pos[j];
                L.u[j + 1] = L.u[j];
                j--;
            }
            L.pos[j + 1] = p;
            L.u[j + 1] = u;
        }
    }
    __syncthreads();
}

// The run's status words and counters start at zero (read by kernels after this one).
__device__ __forceinline__ void zero_run_words(const ScanArgs& a, uint32_t chunk) {
    for (uint32_t i = chunk * SCAN_THREADS + threadIdx.x; i < a.n_status; i += a.n_chunks * SCAN_THREADS)
        a.status[i] = 0;
    if (chunk == 0 && threadIdx.x < 4) a.misc[threadIdx.x] = 0;
}

__global__ __launch_bounds__(SCAN_THREADS) void k_scan(ScanArgs a) {
    const uint32_t chunk = blockIdx.x;
    if (chunk >= a.n_chunks) return;
    zero_run_words(a, chunk);
    __shared__ ScanLds L;
    scan_chunk(a, chunk, L);
    if (threadIdx.x == 0) {
        a.chunk_cnt[chunk] = L.cnt;
        a.chunk_units[chunk] = L.units;
    }
    const uint32_t m = L.cnt < CHUNK_CAP ? L.cnt : CHUNK_CAP;
    if (threadIdx.x < m) {
        a.chunk_slots[(uint64_t)chunk * CHUNK_CAP + threadIdx.x] = L.pos[threadIdx.x];
        a.chunk_slot_units[(uint64_t)chunk * CHUNK_CAP + threadIdx.x] = L.u[threadIdx.x];
    }
}

// ----------------------------------------------------------------------------------
// wave-level scans (64 lanes, __shfl_up: no workgroup barrier)
// ----------------------------------------------------------------------------------
template <typename T>
__device__ __forceinline__ T wave_incl_sum(T v) {
    const uint32_t ln = threadIdx.x & 63u;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const T y = __shfl_up(v, d, 64);
        if (ln >= (uint32_t)d) v += y;
    }
    return v;
}

// ----------------------------------------------------------------------------------
// k_scan_chunks: single-workgroup exclusive scans (n_chunks is ~input/32KiB)
// ----------------------------------------------------------------------------------
constexpr int SCANK_THREADS = 1024;
constexpr int SCANK_WAVES = SCANK_THREADS / 64;
constexpr int SCANK_T = 4;  // chunks per thread per tile (16 contiguous bytes of counts)

// The chunks are scanned in tiles of 4,096: thread t owns chunks 4t..4t+3 of the tile, so a
// wave's loads and stores cover 1 KiB of counts (2 KiB of units) contiguously; per-thread
// sums are scanned in each wave (shuffles) and across the 16 wave totals (one barrier), and
// the tile's total carries into the next tile (the C5 shard: ~11k chunks, 3 tiles). (Round 2
// and v30: contiguous per-thread ranges of ~11 chunks, i.e. 44-byte lane strides.)
__global__ __launch_bounds__(SCANK_THREADS) void k_scan_chunks(const uint32_t* cnt, const unsigned long long* units,
                                                               uint32_t n, uint32_t* off,
                                                               unsigned long long* uoff, uint32_t* n_frames) {
    __shared__ uint32_t s_c[SCANK_WAVES];
    __shared__ unsigned long long s_u[SCANK_WAVES];
    const uint32_t t = threadIdx.x, wv = t >> 6;
    uint32_t carry_c = 0;
    unsigned long long carry_u = 0;
    for (uint32_t tb = 0; tb < n; tb += SCANK_THREADS * SCANK_T) {
        const uint32_t i0 = tb + t * SCANK_T;
        uint32_t c[SCANK_T];
        unsigned long long u[SCANK_T];
        uint32_t sc = 0;
        unsigned long long su = 0;
#pragma unroll
        for (int i = 0; i < SCANK_T; i++) {
            const bool in = i0 + i < n;
            c[i] = in ? cnt[i0 + i] : 0u;
            u[i] = in ? units[i0 + i] : 0ull;
            sc += c[i];
            su += u[i];
        }
        const uint32_t ic = wave_incl_sum(sc);
        const unsigned long long iu = wave_incl_sum(su);
        if ((t & 63u) == 63u) {
            s_c[wv] = ic;
            s_u[wv] = iu;
        }
        __syncthreads();
        uint32_t rc = carry_c + ic - sc;
        unsigned long long ru = carry_u + iu - su;
        uint32_t tc = 0;
        unsigned long long tu = 0;
#pragma unroll
        for (uint32_t w = 0; w < (uint32_t)SCANK_WAVES; w++) {  // LDS broadcasts
            if (w < wv) {
                rc += s_c[w];
                ru += s_u[w];
            }
            tc += s_c[w];
            tu += s_u[w];
        }
#pragma unroll
        for (int i = 0; i < SCANK_T; i++) {
            if (i0 + i < n) {
                off[i0 + i] = rc;
                uoff[i0 + i] = ru;
            }
            rc += c[i];
            ru += u[i];
        }
        carry_c += tc;
        carry_u += tu;
        __syncthreads();  // s_c / s_u are rewritten by the next tile
    }
    if (t == 0) {
        off[n] = carry_c;
        uoff[n] = carry_u;
        *n_frames = carry_c;
    }
}

// ----------------------------------------------------------------------------------
// k_compact: ordered candidate table
// ----------------------------------------------------------------------------------
constexpr int COMPACT_CHUNKS = SCAN_THREADS / 64;  // chunks per workgroup: one wave each

// Overflowed chunk (more than CHUNK_CAP candidates): ordered two-pass rescan of each 4 KiB
// sub-range with a workgroup-wide exclusive scan. Called at workgroup-uniform points.
// `off`: the chunk's first candidate index; `urel`: units of the stream before the chunk;
// `overflow` is set when the table is too small.
__device__ void compact_rescan_at(const uint8_t* in, const StreamDesc* streams, const ChunkDesc* chunks, uint32_t chunk,
                                  uint32_t off, unsigned long long urel, uint32_t cap, uint64_t* c_pos,
                                  uint32_t* c_stream, uint64_t* c_out, uint32_t* overflow) {
    const ChunkDesc ch = chunks[chunk];
    const StreamDesc S = streams[ch.stream];
    auto parse = [&](uint64_t, uint64_t p) -> FrameHdr { return parse_frame_header(in + p, S.in_end - p, S.si_rate); };
    __shared__ uint32_t s_c[SCAN_THREADS];
    __shared__ unsigned long long s_u[SCAN_THREADS];
    __shared__ uint32_t s_base_c;
    __shared__ unsigned long long s_base_u;
    __syncthreads();
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
            scan_window(in, ws, ch.begin, ch.end, [&](uint64_t p) {
                const FrameHdr h = parse(ws, p);
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
            scan_window(in, ws, ch.begin, ch.end, [&](uint64_t p) {
                const FrameHdr h = parse(ws, p);
                if (!candidate_ok(h, S)) return;
                const uint32_t idx = off + rc;
                if (idx < cap) {
                    c_pos[idx] = p;
                    c_stream[idx] = ch.stream;
                    c_out[idx] = S.out_base + (urel + ru);
                } else if (overflow) {
                    atomicOr(overflow, 1u);
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

// One wave per chunk: lane i < n writes the chunk's i-th candidate (in position order, as
// k_scan sorted them), its output offset = the stream's units before the chunk + the units
// of candidates 0..i-1 (a wave prefix sum). Four chunks per workgroup: a workgroup per chunk
// was ~40k mostly idle waves for the C5 shard's ~11k chunks. Overflowed chunks of the
// workgroup are then rescanned by the whole workgroup, in order.
__global__ __launch_bounds__(SCAN_THREADS) void k_compact(CompactArgs a) {
    const uint32_t c0 = blockIdx.x * COMPACT_CHUNKS;
    const uint32_t chunk = c0 + (threadIdx.x >> 6), ln = threadIdx.x & 63u;
    if (chunk < a.n_chunks) {
        const uint32_t n = a.chunk_cnt[chunk];
        if (n <= CHUNK_CAP) {  // wave-uniform
            const uint32_t stream = a.chunks[chunk].stream;
            const StreamDesc& S = a.streams[stream];
            const unsigned long long base = S.out_base + (a.chunk_uoff[chunk] - a.chunk_uoff[S.first_chunk]);
            const uint32_t u = ln < n ? a.chunk_slot_units[(uint64_t)chunk * CHUNK_CAP + ln] : 0u;
            const uint32_t pre = wave_incl_sum(u) - u;  // <= 64 frames x 65535 x 8 channels < 2^32
            if (ln < n) {
                const uint32_t idx = a.chunk_off[chunk] + ln;
                if (idx < a.cap) {
                    a.c_pos[idx] = a.chunk_slots[(uint64_t)chunk * CHUNK_CAP + ln];
                    a.c_stream[idx] = stream;
                    a.c_out[idx] = base + pre;
                } else {
                    atomicOr(a.overflow, 1u);
                }
            }
        }
    }
#pragma unroll 1
    for (uint32_t j = 0; j < (uint32_t)COMPACT_CHUNKS; j++) {  // workgroup-uniform
        const uint32_t cj = c0 + j;
        if (cj < a.n_chunks && a.chunk_cnt[cj] > CHUNK_CAP) {
            const StreamDesc& S = a.streams[a.chunks[cj].stream];
            compact_rescan_at(a.in, a.streams, a.chunks, cj, a.chunk_off[cj],
                              a.chunk_uoff[cj] - a.chunk_uoff[S.first_chunk], a.cap, a.c_pos, a.c_stream, a.c_out,
                              a.overflow);
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
        // (total unknown: certified only with room reserved for it, see alloc_class)
        if (f1 <= f0 || f1 > nframes || (!S.valid_total && !a.units) || a.c_pos[f0] != S.in_begin)
            atomicOr(&a.status[t], 1u);
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
    if (end_rel > S.out_cap) bad = true;
    if (S.valid_total) {
        if (end_rel > S.total) bad = true;  // zflac would grow the buffer and read on to EOF
        if (end_rel < S.total && (t + 1 >= f1 || a.c_pos[t + 1] != a.c_end[t])) bad = true;
    } else {
        // total unknown: frames until fewer than 4 bytes are left (:343-350 EndOfStream
        // break); the frame that ends there is the chain's last and holds its length
        const bool last = a.c_end[t] + 4 > S.in_end;
        if (!last && (t + 1 >= f1 || a.c_pos[t + 1] != a.c_end[t])) bad = true;
        if (last && t + 1 < f1) bad = true;  // a candidate in the last bytes: the planner decides
        if (last && a.units) a.units[s] = end_rel;
    }
    if (bad) atomicOr(&a.status[s], 1u);
}

// ----------------------------------------------------------------------------------
// k_sync_list: the sequential planner's batched probes. Every frame sync code in [lo, hi)
// whose header parses and matches the stream's channels, depth and rate: what zflac's
// frame loop checks (:343-392), without the fast path's CRC-8, reserved-bit and
// blocking-byte filters. Unordered (the host sorts).
// ----------------------------------------------------------------------------------
__global__ __launch_bounds__(SCAN_THREADS) void k_sync_list(SyncListArgs a) {
    const uint64_t abase = a.lo & ~(uint64_t)15;
    const uint64_t nwin = (a.hi - abase + 15) / 16;
    for (uint64_t w = (uint64_t)blockIdx.x * SCAN_THREADS + threadIdx.x; w < nwin;
         w += (uint64_t)gridDim.x * SCAN_THREADS) {
        scan_window(a.in, abase + w * 16, a.lo, a.hi, [&](uint64_t p) {
            const FrameHdr h = parse_frame_header(a.in + p, a.in_end - p, a.si_rate);
            if (h.err || h.crc_eof || channels_count(h.chan_code) != a.nch || h.dcode != a.dcode ||
                h.rate != a.rate_hz)
                return;
            const uint32_t slot = atomicAdd(a.count, 1u);
            if (slot < a.cap) a.pos[slot] = p;
        });
    }
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
    hipLaunchKernelGGL(k_compact, dim3((a.n_chunks + COMPACT_CHUNKS - 1) / COMPACT_CHUNKS), dim3(SCAN_THREADS), 0, st,
                       a);
    return hipGetLastError();
}
hipError_t launch_sync_list(const SyncListArgs& a, hipStream_t st) {
    if (a.hi <= a.lo) return hipSuccess;
    const uint64_t windows = (a.hi - (a.lo & ~(uint64_t)15) + 15) / 16;
    uint64_t blocks = (windows + SCAN_THREADS - 1) / SCAN_THREADS;
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(k_sync_list, dim3((uint32_t)blocks), dim3(SCAN_THREADS), 0, st, a);
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
