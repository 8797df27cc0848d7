// md5.hip -- batched STREAMINFO MD5 of decoded streams on the device.
//
// zflac hashes the decoded samples before left-justify (src/zflac.zig:267-280): the whole
// sample backing for 8/16/32-bit containers, 3 little-endian bytes per i32 for 24-bit
// containers. The device buffers hold the samples after left-justify (done at pack-out),
// so the message bytes are rebuilt on the fly: each sample is shifted back right by the
// stream's justify amount (arithmetic, as the values were sign-extended before it).
//
// MD5 (RFC 1321) is a chain over 64-byte blocks, so one stream is one lane: a batch of
// many streams fills waves, one long stream does not (the host keeps the CPU hash for
// that case, see host.cpp). Per block: 16 message words from HBM (loaded one unit ahead
// of the compression that uses them), 64 dependent rounds of ~5 VALU ops (gfx950's
// v_bitop3_b32 makes each round function one instruction).
//
// A lane's time is its stream's chain (~4 dependent VALU ops per round), so a batch's hash
// takes about as long as its longest stream, whatever the stream count. Runs are hashed by
// the device's md5 hub (host.cpp): one launch over the certified streams of several runs,
// on a stream of its own, while the runs of other batches decode. That launch is k_md5_coop
// (a wave reads its 64 streams' data cooperatively through LDS, hash_units_coop) when every
// job shares one mode and 16-byte alignment, else k_md5_multi (each lane its own loads).
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdlib>

#include "common.h"

namespace zflac {
namespace {

__device__ __forceinline__ uint32_t rotl(uint32_t x, int s) { return __builtin_amdgcn_alignbit(x, x, 32 - s); }

// The round functions as single v_bitop3_b32 (gfx950): truth tables over x = 0xF0,
// y = 0xCC, z = 0xAA. F = (x & y) | (~x & z), G = (x & z) | (y & ~z), H = x ^ y ^ z,
// I = y ^ (x | ~z) (RFC 1321 3.4). Left to the compiler, H took two v_xor per round.
#define MD_F(x, y, z) __builtin_amdgcn_bitop3_b32((x), (y), (z), 0xCA)
#define MD_G(x, y, z) __builtin_amdgcn_bitop3_b32((x), (y), (z), 0xE4)
#define MD_H(x, y, z) __builtin_amdgcn_bitop3_b32((x), (y), (z), 0x96)
#define MD_I(x, y, z) __builtin_amdgcn_bitop3_b32((x), (y), (z), 0x39)
#define MD_R(f, a, b, c, d, k, t, s) a = (b) + rotl((a) + f(b, c, d) + m[k] + (t), s)

__device__ __forceinline__ void compress(uint32_t st[4], const uint32_t m[16]) {
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3];
    MD_R(MD_F, a, b, c, d, 0, 0xd76aa478u, 7);  MD_R(MD_F, d, a, b, c, 1, 0xe8c7b756u, 12);
    MD_R(MD_F, c, d, a, b, 2, 0x242070dbu, 17); MD_R(MD_F, b, c, d, a, 3, 0xc1bdceeeu, 22);
    MD_R(MD_F, a, b, c, d, 4, 0xf57c0fafu, 7);  MD_R(MD_F, d, a, b, c, 5, 0x4787c62au, 12);
    MD_R(MD_F, c, d, a, b, 6, 0xa8304613u, 17); MD_R(MD_F, b, c, d, a, 7, 0xfd469501u, 22);
    MD_R(MD_F, a, b, c, d, 8, 0x698098d8u, 7);  MD_R(MD_F, d, a, b, c, 9, 0x8b44f7afu, 12);
    MD_R(MD_F, c, d, a, b, 10, 0xffff5bb1u, 17); MD_R(MD_F, b, c, d, a, 11, 0x895cd7beu, 22);
    MD_R(MD_F, a, b, c, d, 12, 0x6b901122u, 7); MD_R(MD_F, d, a, b, c, 13, 0xfd987193u, 12);
    MD_R(MD_F, c, d, a, b, 14, 0xa679438eu, 17); MD_R(MD_F, b, c, d, a, 15, 0x49b40821u, 22);
    MD_R(MD_G, a, b, c, d, 1, 0xf61e2562u, 5);  MD_R(MD_G, d, a, b, c, 6, 0xc040b340u, 9);
    MD_R(MD_G, c, d, a, b, 11, 0x265e5a51u, 14); MD_R(MD_G, b, c, d, a, 0, 0xe9b6c7aau, 20);
    MD_R(MD_G, a, b, c, d, 5, 0xd62f105du, 5);  MD_R(MD_G, d, a, b, c, 10, 0x02441453u, 9);
    MD_R(MD_G, c, d, a, b, 15, 0xd8a1e681u, 14); MD_R(MD_G, b, c, d, a, 4, 0xe7d3fbc8u, 20);
    MD_R(MD_G, a, b, c, d, 9, 0x21e1cde6u, 5);  MD_R(MD_G, d, a, b, c, 14, 0xc33707d6u, 9);
    MD_R(MD_G, c, d, a, b, 3, 0xf4d50d87u, 14); MD_R(MD_G, b, c, d, a, 8, 0x455a14edu, 20);
    MD_R(MD_G, a, b, c, d, 13, 0xa9e3e905u, 5); MD_R(MD_G, d, a, b, c, 2, 0xfcefa3f8u, 9);
    MD_R(MD_G, c, d, a, b, 7, 0x676f02d9u, 14); MD_R(MD_G, b, c, d, a, 12, 0x8d2a4c8au, 20);
    MD_R(MD_H, a, b, c, d, 5, 0xfffa3942u, 4);  MD_R(MD_H, d, a, b, c, 8, 0x8771f681u, 11);
    MD_R(MD_H, c, d, a, b, 11, 0x6d9d6122u, 16); MD_R(MD_H, b, c, d, a, 14, 0xfde5380cu, 23);
    MD_R(MD_H, a, b, c, d, 1, 0xa4beea44u, 4);  MD_R(MD_H, d, a, b, c, 4, 0x4bdecfa9u, 11);
    MD_R(MD_H, c, d, a, b, 7, 0xf6bb4b60u, 16); MD_R(MD_H, b, c, d, a, 10, 0xbebfbc70u, 23);
    MD_R(MD_H, a, b, c, d, 13, 0x289b7ec6u, 4); MD_R(MD_H, d, a, b, c, 0, 0xeaa127fau, 11);
    MD_R(MD_H, c, d, a, b, 3, 0xd4ef3085u, 16); MD_R(MD_H, b, c, d, a, 6, 0x04881d05u, 23);
    MD_R(MD_H, a, b, c, d, 9, 0xd9d4d039u, 4);  MD_R(MD_H, d, a, b, c, 12, 0xe6db99e5u, 11);
    MD_R(MD_H, c, d, a, b, 15, 0x1fa27cf8u, 16); MD_R(MD_H, b, c, d, a, 2, 0xc4ac5665u, 23);
    MD_R(MD_I, a, b, c, d, 0, 0xf4292244u, 6);  MD_R(MD_I, d, a, b, c, 7, 0x432aff97u, 10);
    MD_R(MD_I, c, d, a, b, 14, 0xab9423a7u, 15); MD_R(MD_I, b, c, d, a, 5, 0xfc93a039u, 21);
    MD_R(MD_I, a, b, c, d, 12, 0x655b59c3u, 6); MD_R(MD_I, d, a, b, c, 3, 0x8f0ccc92u, 10);
    MD_R(MD_I, c, d, a, b, 10, 0xffeff47du, 15); MD_R(MD_I, b, c, d, a, 1, 0x85845dd1u, 21);
    MD_R(MD_I, a, b, c, d, 8, 0x6fa87e4fu, 6);  MD_R(MD_I, d, a, b, c, 15, 0xfe2ce6e0u, 10);
    MD_R(MD_I, c, d, a, b, 6, 0xa3014314u, 15); MD_R(MD_I, b, c, d, a, 13, 0x4e0811a1u, 21);
    MD_R(MD_I, a, b, c, d, 4, 0xf7537e82u, 6);  MD_R(MD_I, d, a, b, c, 11, 0xbd3af235u, 10);
    MD_R(MD_I, c, d, a, b, 2, 0x2ad7d2bbu, 15); MD_R(MD_I, b, c, d, a, 9, 0xeb86d391u, 21);
    st[0] += a;
    st[1] += b;
    st[2] += c;
    st[3] += d;
}

// Message word from a raw little-endian word of the sample buffer (modes RAW, S16, S32).
template <int MODE>
__device__ __forceinline__ uint32_t unjustify_word(uint32_t r, uint32_t js) {
    if constexpr (MODE == MD5_S16_SHIFT) {
        const uint32_t lo = (uint32_t)((int32_t)(int16_t)(r & 0xffffu) >> js) & 0xffffu;
        const uint32_t hi = (uint32_t)(((int32_t)r >> 16) >> js);
        return lo | (hi << 16);
    } else if constexpr (MODE == MD5_S32_SHIFT) {
        return (uint32_t)((int32_t)r >> js);
    } else {
        return r;
    }
}

// Byte v of the hashed message (tail blocks only).
__device__ uint32_t message_byte(const Md5Job& j, uint64_t v) {
    switch (j.mode) {
        case MD5_RAW: return j.data[v];
        case MD5_S16_SHIFT: {
            const int16_t x = reinterpret_cast<const int16_t*>(j.data)[v >> 1];
            return ((uint32_t)((int32_t)x >> j.js) >> (8 * (v & 1))) & 0xffu;
        }
        case MD5_S32_SHIFT: {
            const int32_t x = reinterpret_cast<const int32_t*>(j.data)[v >> 2];
            return ((uint32_t)(x >> j.js) >> (8 * (v & 3))) & 0xffu;
        }
        default: {  // MD5_S24: 3 bytes per i32 sample
            const int32_t x = reinterpret_cast<const int32_t*>(j.data)[v / 3];
            return ((uint32_t)(x >> j.js) >> (8 * (uint32_t)(v % 3))) & 0xffu;
        }
    }
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// The wave's tile is its own (a workgroup holds several waves, each with a tile): the LDS
// writes of all its lanes before any lane's reads, and the reads before the next writes.
// LDS operations of one wave complete in order; the fence keeps the compiler's order and
// waits for the wave's outstanding LDS operations.
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
}
constexpr int UNIT_WORDS = 64;  // raw dwords per unit: 4 blocks, or 3 blocks of 24-bit samples

// Compress one unit (UNIT_WORDS raw dwords, plus the dword after it for unaligned bases).
template <int MODE>
__device__ __forceinline__ void hash_unit(const uint32_t* cur, uint32_t sh, uint32_t js, uint32_t st[4]) {
    uint32_t m[16];
    if constexpr (MODE == MD5_S24) {
#pragma unroll
        for (int blk = 0; blk < 3; blk++) {
#pragma unroll
            for (int w = 0; w < 16; w++) {
                // 4 samples -> 3 words: x0|x1<<24, x1>>8|x2<<16, x2>>16|x3<<8
                const int g = blk * 16 + w, ph = g % 3, s0 = (g / 3) * 4 + ph;
                const uint32_t x0 = (uint32_t)((int32_t)cur[s0] >> js) & 0xffffffu;
                const uint32_t x1 = (uint32_t)((int32_t)cur[s0 + 1] >> js) & 0xffffffu;
                m[w] = ph == 0 ? (x0 | (x1 << 24)) : ph == 1 ? ((x0 >> 8) | (x1 << 16)) : ((x0 >> 16) | (x1 << 8));
            }
            compress(st, m);
        }
    } else {
#pragma unroll
        for (int blk = 0; blk < 4; blk++) {
#pragma unroll
            for (int w = 0; w < 16; w++)
                m[w] = unjustify_word<MODE>(sh ? __builtin_amdgcn_alignbyte(cur[blk * 16 + w + 1], cur[blk * 16 + w], sh)
                                               : cur[blk * 16 + w],
                                            js);
            compress(st, m);
        }
    }
}

// The full units of one stream: 256 raw bytes each, loaded one unit (3-4 blocks of
// compression, several microseconds) ahead of their use, into two register sets used in
// turn (no copies between them). A 16-byte aligned stream (every certified stream: regions
// start on 32-byte boundaries) loads each unit with 16 dwordx4 loads; otherwise 65 dwords.
// Returns message bytes hashed.
template <int MODE, bool VEC>
__device__ __forceinline__ uint64_t hash_units(const Md5Job& j, uint32_t st[4]) {
    constexpr uint64_t MSG_PER_UNIT = MODE == MD5_S24 ? 192 : 256;
    const uint64_t L = j.n * (uint64_t)j.width;
    const uint64_t nu = L / MSG_PER_UNIT;
    const uint32_t sh = VEC ? 0u : (uint32_t)(reinterpret_cast<uintptr_t>(j.data) & 3);
    const uint32_t* p = reinterpret_cast<const uint32_t*>(reinterpret_cast<uintptr_t>(j.data) & ~(uintptr_t)3);
    uint32_t ba[UNIT_WORDS + 1], bb[UNIT_WORDS + 1];
    auto load = [&](uint64_t u, uint32_t* r) {
#if defined(ZFLAC_MD5_NOLOAD)  // (diagnostic) no memory reads: the chain alone; wrong digests
#pragma unroll
        for (int i = 0; i <= UNIT_WORDS; i++) r[i] = (uint32_t)u * 0x9e3779b9u + i;
        return;
#elif defined(ZFLAC_MD5_L2HIT)  // (diagnostic) every unit re-reads the stream's first 1 KiB; wrong digests
        u &= 3;
#endif
        const uint32_t* q = p + u * UNIT_WORDS;
        if constexpr (VEC) {
#pragma unroll
            for (int i = 0; i < UNIT_WORDS / 4; i++) {
                const u32x4 v = __builtin_nontemporal_load(
                    reinterpret_cast<const __attribute__((address_space(1))) u32x4*>(reinterpret_cast<uintptr_t>(q)) + i);
                r[4 * i] = v[0];
                r[4 * i + 1] = v[1];
                r[4 * i + 2] = v[2];
                r[4 * i + 3] = v[3];
            }
            r[UNIT_WORDS] = 0u;
        } else {
#pragma unroll
            for (int i = 0; i < UNIT_WORDS; i++) r[i] = __builtin_nontemporal_load(q + i);
            // the dword after the unit carries its last bytes when the base is unaligned
            r[UNIT_WORDS] = (MODE != MD5_S24 && sh) ? __builtin_nontemporal_load(q + UNIT_WORDS) : 0u;
        }
    };
    if (nu) load(0, ba);
    uint64_t u = 0;
    for (; u + 2 <= nu; u += 2) {
        load(u + 1, bb);
        hash_unit<MODE>(ba, sh, j.js, st);
        if (u + 2 < nu) load(u + 2, ba);
        hash_unit<MODE>(bb, sh, j.js, st);
    }
    if (u < nu) hash_unit<MODE>(ba, sh, j.js, st);
    return nu * MSG_PER_UNIT;
}

template <int MODE>
__device__ __forceinline__ uint64_t hash_units_any(const Md5Job& j, uint32_t st[4]) {
    return (reinterpret_cast<uintptr_t>(j.data) & 15) == 0 ? hash_units<MODE, true>(j, st)
                                                          : hash_units<MODE, false>(j, st);
}

// Wave-cooperative unit loop: every lane of the wave calls it (lanes with `act` false only
// help load). Lane-per-stream loads touch 64 streams' cache lines per wave-instruction; here
// wave-instruction i instead reads the 256-byte units of streams 4i..4i+3 (four 256-byte
// runs: the lane-per-stream form's 64 lines become 8), the wave's 64 units go through one
// 16 KiB LDS tile, and each lane then reads its own stream's unit from it. Row s of the tile
// is stream s (lane s); its piece pc (16 bytes) sits at slot (pc + s) & 15, so the 64 lanes'
// reads of one piece fall on different banks (a plain 256-byte row stride puts them on one).
// The next unit's loads are in flight in registers while the current one is compressed.
// Needs every active lane's samples 16-byte aligned (certified streams: see hash_units) and
// one MODE across the wave. Returns message bytes hashed.
template <int MODE>
__device__ __forceinline__ uint64_t hash_units_coop(const Md5Job& j, bool act, uint32_t st[4], u32x4* tile) {
    constexpr uint64_t MSG_PER_UNIT = MODE == MD5_S24 ? 192 : 256;
    const uint32_t L = threadIdx.x & 63u;
    const uint32_t nu = act ? (uint32_t)min(j.n * (uint64_t)j.width / MSG_PER_UNIT, (uint64_t)0xFFFFFFFFu) : 0u;
    const uint64_t base = reinterpret_cast<uintptr_t>(j.data);
    uint64_t src[16];  // this lane's 16 bytes of stream 4i + L/16's unit 0 (piece (L - s) & 15)
    uint32_t nus[16];
#pragma unroll
    for (int i = 0; i < 16; i++) {
        const int sl = 4 * i + (int)(L >> 4);
        const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)base, sl), hi = (uint32_t)__shfl((int)(uint32_t)(base >> 32), sl);
        src[i] = (((uint64_t)hi << 32) | lo) + ((L - (uint32_t)sl) & 15u) * 16u;
        nus[i] = (uint32_t)__shfl((int)nu, sl);
    }
    uint32_t maxu = nu;
#pragma unroll
    for (int o = 32; o; o >>= 1) maxu = max(maxu, (uint32_t)__shfl_xor((int)maxu, o));
    u32x4 R[16];
    auto load = [&](uint32_t u) {
#pragma unroll
        for (int i = 0; i < 16; i++)
            if (u < nus[i])  // global (not flat) loads: a flat load would also hold lgkmcnt, i.e. the tile reads
                R[i] = __builtin_nontemporal_load(
                    reinterpret_cast<const __attribute__((address_space(1))) u32x4*>(src[i] + (uint64_t)u * 256u));
    };
    if (maxu) load(0);
    const u32x4* row = tile + L * 16u;
    for (uint32_t u = 0; u < maxu; u++) {
#pragma unroll
        for (int i = 0; i < 16; i++) tile[i * 64 + L] = R[i];  // row 4i + L/16, slot L & 15
        wave_sync();
        if (u + 1 < maxu) load(u + 1);
        if (u < nu) {
            if constexpr (MODE == MD5_S24) {
                uint32_t cur[UNIT_WORDS + 1];
#pragma unroll
                for (int pc = 0; pc < 16; pc++) {
                    const u32x4 v = row[(pc + L) & 15u];
#pragma unroll
                    for (int e = 0; e < 4; e++) cur[4 * pc + e] = v[e];
                }
                cur[UNIT_WORDS] = 0u;
                hash_unit<MODE>(cur, 0u, j.js, st);
            } else {
#pragma unroll
                for (int blk = 0; blk < 4; blk++) {
                    uint32_t m[16];
#pragma unroll
                    for (int pc = 0; pc < 4; pc++) {
                        const u32x4 v = row[(blk * 4 + pc + L) & 15u];
#pragma unroll
                        for (int e = 0; e < 4; e++) m[4 * pc + e] = unjustify_word<MODE>(v[e], j.js);
                    }
                    compress(st, m);
                }
            }
        }
        wave_sync();  // every lane's reads of the tile before the next unit's writes
    }
    return (uint64_t)nu * MSG_PER_UNIT;
}

// The tail blocks of one stream (the message bytes after `done`, 0x80, zero fill, the
// 64-bit little-endian bit length) and its digest into out[0..3].
__device__ __forceinline__ void md5_tail(const Md5Job& j, uint64_t done, uint32_t st[4], uint32_t* __restrict__ out) {
    const uint64_t L = j.n * (uint64_t)j.width;  // message bytes
    uint32_t m[16];
    const uint64_t r = L - done;
    const uint32_t tb = (uint32_t)((r + 8) / 64 + 1);
    const uint64_t bits = L * 8;
    for (uint32_t b = 0; b < tb; b++) {
        for (int w = 0; w < 16; w++) {
            uint32_t word = 0;
            for (int q = 0; q < 4; q++) {
                const uint64_t o = (uint64_t)b * 64 + w * 4 + q;  // offset from `done`
                uint32_t byte;
                if (o < r) byte = message_byte(j, done + o);
                else if (o == r) byte = 0x80u;
                else if (b + 1 == tb && w >= 14) byte = (uint32_t)(bits >> (8 * ((w - 14) * 4 + q))) & 0xffu;
                else byte = 0;
                word |= byte << (8 * q);
            }
            m[w] = word;
        }
        compress(st, m);
    }
#pragma unroll
    for (int i = 0; i < 4; i++) out[i] = st[i];
}

__device__ __forceinline__ void md5_prio() {
#ifdef ZFLAC_MD5_PRIO
    // (experiment) the hash waves ahead of the decode waves they share SIMDs with: the
    // serial chains then run at the pace of a wave alone, but the decode waves slow down
    __builtin_amdgcn_s_setprio(ZFLAC_MD5_PRIO);
#endif
}

// One stream's digest into out[0..3], the lane's own loads (any mode and alignment).
__device__ __forceinline__ void md5_job(const Md5Job& j, uint32_t* __restrict__ out) {
    md5_prio();
    uint32_t st[4] = {0x67452301u, 0xefcdab89u, 0x98badcfeu, 0x10325476u};
    if (j.status && *j.status) {  // not certified by this run: the host hashes it after the planner
#pragma unroll
        for (int i = 0; i < 4; i++) out[i] = 0u;
        return;
    }
    uint64_t done;  // message bytes hashed by the unit loop
    switch (j.mode) {
        case MD5_RAW: done = hash_units_any<MD5_RAW>(j, st); break;
        case MD5_S16_SHIFT: done = hash_units_any<MD5_S16_SHIFT>(j, st); break;
        case MD5_S32_SHIFT: done = hash_units_any<MD5_S32_SHIFT>(j, st); break;
        default: done = hash_units_any<MD5_S24>(j, st); break;
    }
    md5_tail(j, done, st, out);
}

// The jobs of several runs (one segment each: several batches' runs hashed by one launch,
// md5 hub in host.cpp): lane t's job is job t - start[s] of the segment s holding t.
__device__ __forceinline__ const Md5Job* seg_job(const Md5Segs& sg, uint32_t t, uint32_t*& out) {
    if (t >= sg.start[sg.nseg]) return nullptr;
    uint32_t s = 0;
    while (s + 1 < sg.nseg && sg.start[s + 1] <= t) s++;
    const uint32_t k = t - sg.start[s];
    out = sg.dig[s] + (uint64_t)k * 4;
    return sg.jobs[s] + k;
}

__global__ __launch_bounds__(64) void k_md5(const Md5Job* __restrict__ jobs, uint32_t n_jobs,
                                            uint32_t* __restrict__ digests) {
    const uint32_t t = blockIdx.x * 64 + threadIdx.x;
    if (t >= n_jobs) return;
    md5_job(jobs[t], digests + (uint64_t)t * 4);
}

__global__ __launch_bounds__(64) void k_md5_multi(Md5Segs sg) {
    uint32_t* out = nullptr;
    const Md5Job* j = seg_job(sg, blockIdx.x * 64 + threadIdx.x, out);
    if (j) md5_job(*j, out);
}

// Every job of the launch in mode MODE with 16-byte aligned samples (the host checks):
// the wave's lanes load cooperatively (hash_units_coop); lanes past the job list, or whose
// stream this run did not certify, only help load.
// Workgroups of ZFLAC_MD5_WG_WAVES waves (1..8, default 4), one 16 KiB tile each: the
// workgroup's LDS decides how the hash shares CUs with k_decode, whose four 40 KiB
// workgroups fill a CU's 160 KiB. A one-wave hash workgroup (16 KiB) on a CU leaves room
// for three decode workgroups, so hash waves spread one per CU each cost that CU a quarter
// of its decode capacity; four waves (64 KiB: one per SIMD, beside two decode workgroups)
// put the same hash on a quarter as many CUs. Decode + MD5 on the C5 shard
// (profiles/r5_md5_wg_sweep.json): 1 wave 357k, 2 366k, 3 383k, 4 401-428k, 5-8 290-300k
// Msamples/s (five or more hash waves per CU starve the hash chains of issue slots).
constexpr int MD5_MAX_WG_WAVES = 8;
extern __shared__ u32x4 g_md5_tile[];
template <int MODE>
__global__ __launch_bounds__(64 * MD5_MAX_WG_WAVES) void k_md5_coop(Md5Segs sg) {
    u32x4* const tile = g_md5_tile + (threadIdx.x >> 6) * (64 * 16);
    md5_prio();
    uint32_t* out = nullptr;
    const Md5Job* jp = seg_job(sg, blockIdx.x * blockDim.x + threadIdx.x, out);
    Md5Job j{};
    if (jp) j = *jp;
    const bool act = jp && !(j.status && *j.status);
    uint32_t st[4] = {0x67452301u, 0xefcdab89u, 0x98badcfeu, 0x10325476u};
    const uint64_t done = hash_units_coop<MODE>(j, act, st, tile);
    if (act) {
        md5_tail(j, done, st, out);
    } else if (jp) {
#pragma unroll
        for (int i = 0; i < 4; i++) out[i] = 0u;
    }
}

}  // namespace

// waves per k_md5_coop workgroup (ZFLAC_MD5_WG_WAVES, default MD5_WG_WAVES_DEFAULT)
#ifndef MD5_WG_WAVES_DEFAULT
#define MD5_WG_WAVES_DEFAULT 4
#endif
int md5_wg_waves() {
    static const int w = [] {
        const char* e = std::getenv("ZFLAC_MD5_WG_WAVES");
        const int v = e ? atoi(e) : MD5_WG_WAVES_DEFAULT;
        return v < 1 ? 1 : (v > MD5_MAX_WG_WAVES ? MD5_MAX_WG_WAVES : v);
    }();
    return w;
}

// hipFuncSetAttribute(MaxDynamicSharedMemorySize) once per device and kernel (the attribute
// belongs to the kernel's instance on the current device)
template <int MODE>
hipError_t allow_md5_lds(size_t bytes) {
    static std::atomic<uint64_t> done{0};
    int dev = 0;
    if (const hipError_t e = hipGetDevice(&dev); e != hipSuccess) return e;
    const uint64_t bit = 1ull << (dev & 63);
    if (done.load(std::memory_order_acquire) & bit) return hipSuccess;
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_md5_coop<MODE>),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
    if (e == hipSuccess) done.fetch_or(bit, std::memory_order_acq_rel);
    return e;
}

// Waves per k_md5_coop workgroup on the current device: ZFLAC_MD5_WG_WAVES clamped to what
// the device's per-workgroup LDS limit holds (16 KiB of tile per wave), 0 if not even one.
uint32_t md5_wg_waves_dev() {
    static std::atomic<uint64_t> cache[64];  // per device: 1 + waves (0 = not yet queried)
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 0;
    const uint64_t c = cache[dev & 63].load(std::memory_order_acquire);
    if (c) return (uint32_t)(c - 1);
    int optin = 0, plain = 0;
    if (hipDeviceGetAttribute(&optin, hipDeviceAttributeSharedMemPerBlockOptin, dev) != hipSuccess) optin = 0;
    if (hipDeviceGetAttribute(&plain, hipDeviceAttributeMaxSharedMemoryPerBlock, dev) != hipSuccess) plain = 0;
    const size_t lim = (size_t)(optin > plain ? optin : plain);
    const size_t per = 64 * 16 * sizeof(u32x4);
    uint32_t w = (uint32_t)md5_wg_waves();
    if ((size_t)w * per > lim) w = (uint32_t)(lim / per);
    cache[dev & 63].store(1 + w, std::memory_order_release);
    return w;
}

template <int MODE>
hipError_t launch_coop(const Md5Segs& sg, uint32_t n, hipStream_t st) {
    const uint32_t w = md5_wg_waves_dev();
    if (w == 0) {  // no room for a tile: the lane-load kernel
        hipLaunchKernelGGL(k_md5_multi, dim3((n + 63) / 64), dim3(64), 0, st, sg);
        return hipGetLastError();
    }
    const size_t lds = (size_t)w * 64 * 16 * sizeof(u32x4);
    if (const hipError_t e = allow_md5_lds<MODE>(lds); e != hipSuccess) {
        (void)hipGetLastError();  // the attribute was refused: the lane-load kernel instead
        hipLaunchKernelGGL(k_md5_multi, dim3((n + 63) / 64), dim3(64), 0, st, sg);
        return hipGetLastError();
    }
    hipLaunchKernelGGL(k_md5_coop<MODE>, dim3((n + 64 * w - 1) / (64 * w)), dim3(64 * w), lds, st, sg);
    return hipGetLastError();
}

hipError_t launch_md5_multi(const Md5Segs& sg, hipStream_t st, int coop_mode) {
    const uint32_t n = sg.start[sg.nseg];
    if (!n) return hipSuccess;
    switch (coop_mode) {
        case MD5_RAW: return launch_coop<MD5_RAW>(sg, n, st);
        case MD5_S16_SHIFT: return launch_coop<MD5_S16_SHIFT>(sg, n, st);
        case MD5_S32_SHIFT: return launch_coop<MD5_S32_SHIFT>(sg, n, st);
        case MD5_S24: return launch_coop<MD5_S24>(sg, n, st);
        default: hipLaunchKernelGGL(k_md5_multi, dim3((n + 63) / 64), dim3(64), 0, st, sg); return hipGetLastError();
    }
}

hipError_t launch_md5(const Md5Job* jobs, uint32_t n_jobs, uint32_t* digests, hipStream_t st, int coop_mode) {
    if (!n_jobs) return hipSuccess;
    if (coop_mode >= 0) {
        Md5Segs sg;
        sg.jobs[0] = jobs;
        sg.dig[0] = digests;
        sg.start[0] = 0;
        sg.start[1] = n_jobs;
        sg.nseg = 1;
        return launch_md5_multi(sg, st, coop_mode);
    }
    hipLaunchKernelGGL(k_md5, dim3((n_jobs + 63) / 64), dim3(64), 0, st, jobs, n_jobs, digests);
    return hipGetLastError();
}

}  // namespace zflac
