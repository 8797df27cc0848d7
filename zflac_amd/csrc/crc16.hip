// crc16.hip -- optional frame CRC-16 check (ZFLAC_FLAG_CHECK_CRC16).
//
// zflac reads each frame's CRC-16 trailer and ignores it (src/zflac.zig:548-551 is a TODO);
// this check is therefore off by default and, when asked for, reports a mismatch as
// ZFLAC_E_FRAME_CRC. CRC-16 of FLAC frames: x^16 + x^15 + x^2 + 1, MSB first, init 0, over
// every frame byte from the sync code up to (not including) the trailer (RFC 9639 9.1.8).
//
// One wave per frame. The CRC with init 0 is linear, so CRC(A || B) = CRC(A) * x^(8|B|) mod P
// xor CRC(B): each lane hashes a contiguous 1/64 of the frame (whole aligned dwords,
// slice-by-4 tables in LDS), multiplies its remainder by x^(8 * bytes after its piece) and
// the wave xor-reduces. HBM-bound: each frame byte is read once.
#include "device_common.h"

namespace zflac {
namespace {

constexpr uint32_t CRC16_P = 0x18005;  // x^16 + x^15 + x^2 + 1

struct Crc16Tabs {
    uint16_t t[4][256];  // t[k][v] = v(x) * x^(8k + 16) mod P
};
constexpr Crc16Tabs make_crc16_tabs() {
    Crc16Tabs r{};
    for (uint32_t v = 0; v < 256; v++) {
        uint32_t c = v << 8;
        for (int i = 0; i < 8; i++) c = (c & 0x8000) ? ((c << 1) ^ CRC16_P) : (c << 1);
        r.t[0][v] = (uint16_t)c;
    }
    for (int k = 1; k < 4; k++)
        for (uint32_t v = 0; v < 256; v++) {
            const uint32_t c = r.t[k - 1][v];  // one more zero byte
            r.t[k][v] = (uint16_t)(r.t[0][c >> 8] ^ ((c << 8) & 0xFFFF));
        }
    return r;
}

// a(x) * b(x) mod P for 16-bit remainders (Horner over b's bits, most significant first)
__host__ __device__ constexpr uint32_t crc16_mulmod(uint32_t a, uint32_t b) {
    uint32_t r = 0;
    for (int i = 15; i >= 0; i--) {
        r <<= 1;
        if (r & 0x10000) r ^= CRC16_P;
        if ((b >> i) & 1) r ^= a;
    }
    return r;
}

struct Crc16Pow {
    uint16_t p[40];  // p[k] = x^(8 * 2^k) mod P
};
constexpr Crc16Pow make_crc16_pow() {
    Crc16Pow r{};
    r.p[0] = 0x100;  // x^8
    for (int k = 1; k < 40; k++) r.p[k] = (uint16_t)crc16_mulmod(r.p[k - 1], r.p[k - 1]);
    return r;
}

static __constant__ Crc16Tabs CRC16T = make_crc16_tabs();
static __constant__ Crc16Pow CRC16POW = make_crc16_pow();

constexpr int CRC_THREADS = 256;

__device__ __forceinline__ uint32_t crc16_byte(const uint32_t* t0, uint32_t crc, uint32_t b) {
    return t0[(crc >> 8) ^ b] ^ ((crc << 8) & 0xFFFFu);
}

__global__ __launch_bounds__(CRC_THREADS) void k_crc16(Crc16Args a) {
    __shared__ uint32_t T[4][256];
    for (uint32_t i = threadIdx.x; i < 4 * 256; i += CRC_THREADS) T[i >> 8][i & 255] = CRC16T.t[i >> 8][i & 255];
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = (blockIdx.x * CRC_THREADS + threadIdx.x) >> 6;
    const uint32_t nwaves = (gridDim.x * CRC_THREADS) >> 6;
    uint32_t n = a.n_frames ? *a.n_frames : a.n_frames_host;
    if (n > a.cap) n = a.cap;
    const uint32_t* in32 = reinterpret_cast<const uint32_t*>(a.in);
    for (uint32_t f = wave; f < n; f += nwaves) {
        const uint64_t pos = a.pos[f], end = a.end[f];
        // frames that failed to decode have no trailer to check (their error stands), and
        // candidates at or past their stream's STREAMINFO total are never read by zflac
        // (src/zflac.zig:341): false syncs in the last frame or trailing bytes, extra frames
        bool past = false;
        if (a.streams) {
            const StreamDesc& S = a.streams[a.c_stream[f]];
            past = S.valid_total && a.c_out[f] - S.out_base >= S.total;
        }
        const bool ok = !past && (!a.err || a.err[f] == 0) && end >= pos + 3 && end <= a.in_size;
        if (!ok) {
            if (lane == 0) a.bad[f] = 0;
            continue;
        }
        const uint64_t lo = pos, hi = end - 2;  // hashed bytes [lo, hi); trailer at hi
        const uint64_t d0 = lo >> 2, d1 = (hi + 3) >> 2;
        const uint64_t per = (d1 - d0 + 63) >> 6;  // dwords per lane
        const uint64_t my0 = d0 + lane * per;
        const uint64_t my1 = my0 + per < d1 ? my0 + per : d1;
        uint32_t crc = 0;
        for (uint64_t d = my0; d < my1; d++) {
            const uint32_t w = in32[d];  // the input buffer is 16-B aligned and zero-padded
            const uint32_t b0 = w & 255u, b1 = (w >> 8) & 255u, b2 = (w >> 16) & 255u, b3 = w >> 24;
            const uint64_t base = d << 2;
            if (base >= lo && base + 4 <= hi) {  // slice-by-4
                const uint32_t hi8 = (crc >> 8) ^ b0, lo8 = (crc & 255u) ^ b1;
                crc = T[3][hi8] ^ T[2][lo8] ^ T[1][b2] ^ T[0][b3];
            } else {  // the frame's first / last dword: only its bytes
                if (base >= lo && base < hi) crc = crc16_byte(T[0], crc, b0);
                if (base + 1 >= lo && base + 1 < hi) crc = crc16_byte(T[0], crc, b1);
                if (base + 2 >= lo && base + 2 < hi) crc = crc16_byte(T[0], crc, b2);
                if (base + 3 >= lo && base + 3 < hi) crc = crc16_byte(T[0], crc, b3);
            }
        }
        // shift by the bytes after this lane's piece: x^(8 * rem) by squares
        const uint64_t piece_end = my1 > my0 ? ((my1 << 2) < hi ? (my1 << 2) : hi) : hi;
        uint64_t rem = hi - piece_end;
        for (int k = 0; rem && k < 40; k++, rem >>= 1)
            if (rem & 1) crc = crc16_mulmod(crc, CRC16POW.p[k]);
        for (int o = 32; o > 0; o >>= 1) crc ^= (uint32_t)__shfl_xor((int)crc, o);
        if (lane == 0) {
            const uint32_t stored = ((uint32_t)a.in[hi] << 8) | a.in[hi + 1];
            a.bad[f] = crc != stored ? 1u : 0u;
        }
    }
}

}  // namespace

hipError_t launch_crc16(const Crc16Args& a, uint32_t max_frames, hipStream_t st) {
    uint32_t blocks = (max_frames + CRC_THREADS / 64 - 1) / (CRC_THREADS / 64);
    if (blocks > 8192) blocks = 8192;
    if (blocks == 0) blocks = 1;
    hipLaunchKernelGGL(k_crc16, dim3(blocks), dim3(CRC_THREADS), 0, st, a);
    return hipGetLastError();
}

}  // namespace zflac
