// md5.hpp -- RFC 1321 MD5 for the host side of the product (STREAMINFO check of
// decode(), src/zflac.zig:267-280). Header-only so the synthetic writer can reuse it.
#pragma once
#include <cstddef>
#include <cstdint>
#include <cstring>

namespace zflac {

class Md5 {
public:
    Md5() { reset(); }
    void reset() {
        s_[0] = 0x67452301u;
        s_[1] = 0xefcdab89u;
        s_[2] = 0x98badcfeu;
        s_[3] = 0x10325476u;
        len_ = 0;
        fill_ = 0;
    }
    void update(const void* data, size_t n) {
        const uint8_t* p = static_cast<const uint8_t*>(data);
        len_ += n;
        if (fill_) {
            size_t t = 64 - fill_;
            if (t > n) t = n;
            std::memcpy(blk_ + fill_, p, t);
            fill_ += t;
            p += t;
            n -= t;
            if (fill_ < 64) return;
            compress(blk_);
            fill_ = 0;
        }
        for (; n >= 64; n -= 64, p += 64) compress(p);
        if (n) {
            std::memcpy(blk_, p, n);
            fill_ = n;
        }
    }
    void finish(uint8_t out[16]) {
        const uint64_t bits = len_ * 8;
        uint8_t tail[72] = {0x80};
        size_t padn = (fill_ < 56) ? (56 - fill_) : (120 - fill_);
        for (int i = 0; i < 8; i++) tail[padn + i] = static_cast<uint8_t>(bits >> (8 * i));
        update(tail, padn + 8);
        for (int i = 0; i < 4; i++)
            for (int j = 0; j < 4; j++) out[4 * i + j] = static_cast<uint8_t>(s_[i] >> (8 * j));
    }

private:
    static inline uint32_t rol(uint32_t x, int c) { return (x << c) | (x >> (32 - c)); }
    void compress(const uint8_t* p) {
        uint32_t m[16];
        std::memcpy(m, p, 64);  // little-endian host
        uint32_t a = s_[0], b = s_[1], c = s_[2], d = s_[3];
#define ZF_STEP(f, w, x, y, z, k, t, r) w = rol(w + f(x, y, z) + m[k] + t, r) + x
#define ZF_F(x, y, z) (z ^ (x & (y ^ z)))
#define ZF_G(x, y, z) (y ^ (z & (x ^ y)))
#define ZF_H(x, y, z) (x ^ y ^ z)
#define ZF_I(x, y, z) (y ^ (x | ~z))
        ZF_STEP(ZF_F, a, b, c, d, 0, 0xd76aa478u, 7);   ZF_STEP(ZF_F, d, a, b, c, 1, 0xe8c7b756u, 12);
        ZF_STEP(ZF_F, c, d, a, b, 2, 0x242070dbu, 17);  ZF_STEP(ZF_F, b, c, d, a, 3, 0xc1bdceeeu, 22);
        ZF_STEP(ZF_F, a, b, c, d, 4, 0xf57c0fafu, 7);   ZF_STEP(ZF_F, d, a, b, c, 5, 0x4787c62au, 12);
        ZF_STEP(ZF_F, c, d, a, b, 6, 0xa8304613u, 17);  ZF_STEP(ZF_F, b, c, d, a, 7, 0xfd469501u, 22);
        ZF_STEP(ZF_F, a, b, c, d, 8, 0x698098d8u, 7);   ZF_STEP(ZF_F, d, a, b, c, 9, 0x8b44f7afu, 12);
        ZF_STEP(ZF_F, c, d, a, b, 10, 0xffff5bb1u, 17); ZF_STEP(ZF_F, b, c, d, a, 11, 0x895cd7beu, 22);
        ZF_STEP(ZF_F, a, b, c, d, 12, 0x6b901122u, 7);  ZF_STEP(ZF_F, d, a, b, c, 13, 0xfd987193u, 12);
        ZF_STEP(ZF_F, c, d, a, b, 14, 0xa679438eu, 17); ZF_STEP(ZF_F, b, c, d, a, 15, 0x49b40821u, 22);
        ZF_STEP(ZF_G, a, b, c, d, 1, 0xf61e2562u, 5);   ZF_STEP(ZF_G, d, a, b, c, 6, 0xc040b340u, 9);
        ZF_STEP(ZF_G, c, d, a, b, 11, 0x265e5a51u, 14); ZF_STEP(ZF_G, b, c, d, a, 0, 0xe9b6c7aau, 20);
        ZF_STEP(ZF_G, a, b, c, d, 5, 0xd62f105du, 5);   ZF_STEP(ZF_G, d, a, b, c, 10, 0x02441453u, 9);
        ZF_STEP(ZF_G, c, d, a, b, 15, 0xd8a1e681u, 14); ZF_STEP(ZF_G, b, c, d, a, 4, 0xe7d3fbc8u, 20);
        ZF_STEP(ZF_G, a, b, c, d, 9, 0x21e1cde6u, 5);   ZF_STEP(ZF_G, d, a, b, c, 14, 0xc33707d6u, 9);
        ZF_STEP(ZF_G, c, d, a, b, 3, 0xf4d50d87u, 14);  ZF_STEP(ZF_G, b, c, d, a, 8, 0x455a14edu, 20);
        ZF_STEP(ZF_G, a, b, c, d, 13, 0xa9e3e905u, 5);  ZF_STEP(ZF_G, d, a, b, c, 2, 0xfcefa3f8u, 9);
        ZF_STEP(ZF_G, c, d, a, b, 7, 0x676f02d9u, 14);  ZF_STEP(ZF_G, b, c, d, a, 12, 0x8d2a4c8au, 20);
        ZF_STEP(ZF_H, a, b, c, d, 5, 0xfffa3942u, 4);   ZF_STEP(ZF_H, d, a, b, c, 8, 0x8771f681u, 11);
        ZF_STEP(ZF_H, c, d, a, b, 11, 0x6d9d6122u, 16); ZF_STEP(ZF_H, b, c, d, a, 14, 0xfde5380cu, 23);
        ZF_STEP(ZF_H, a, b, c, d, 1, 0xa4beea44u, 4);   ZF_STEP(ZF_H, d, a, b, c, 4, 0x4bdecfa9u, 11);
        ZF_STEP(ZF_H, c, d, a, b, 7, 0xf6bb4b60u, 16);  ZF_STEP(ZF_H, b, c, d, a, 10, 0xbebfbc70u, 23);
        ZF_STEP(ZF_H, a, b, c, d, 13, 0x289b7ec6u, 4);  ZF_STEP(ZF_H, d, a, b, c, 0, 0xeaa127fau, 11);
        ZF_STEP(ZF_H, c, d, a, b, 3, 0xd4ef3085u, 16);  ZF_STEP(ZF_H, b, c, d, a, 6, 0x04881d05u, 23);
        ZF_STEP(ZF_H, a, b, c, d, 9, 0xd9d4d039u, 4);   ZF_STEP(ZF_H, d, a, b, c, 12, 0xe6db99e5u, 11);
        ZF_STEP(ZF_H, c, d, a, b, 15, 0x1fa27cf8u, 16); ZF_STEP(ZF_H, b, c, d, a, 2, 0xc4ac5665u, 23);
        ZF_STEP(ZF_I, a, b, c, d, 0, 0xf4292244u, 6);   ZF_STEP(ZF_I, d, a, b, c, 7, 0x432aff97u, 10);
        ZF_STEP(ZF_I, c, d, a, b, 14, 0xab9423a7u, 15); ZF_STEP(ZF_I, b, c, d, a, 5, 0xfc93a039u, 21);
        ZF_STEP(ZF_I, a, b, c, d, 12, 0x655b59c3u, 6);  ZF_STEP(ZF_I, d, a, b, c, 3, 0x8f0ccc92u, 10);
        ZF_STEP(ZF_I, c, d, a, b, 10, 0xffeff47du, 15); ZF_STEP(ZF_I, b, c, d, a, 1, 0x85845dd1u, 21);
        ZF_STEP(ZF_I, a, b, c, d, 8, 0x6fa87e4fu, 6);   ZF_STEP(ZF_I, d, a, b, c, 15, 0xfe2ce6e0u, 10);
        ZF_STEP(ZF_I, c, d, a, b, 6, 0xa3014314u, 15);  ZF_STEP(ZF_I, b, c, d, a, 13, 0x4e0811a1u, 21);
        ZF_STEP(ZF_I, a, b, c, d, 4, 0xf7537e82u, 6);   ZF_STEP(ZF_I, d, a, b, c, 11, 0xbd3af235u, 10);
        ZF_STEP(ZF_I, c, d, a, b, 2, 0x2ad7d2bbu, 15);  ZF_STEP(ZF_I, b, c, d, a, 9, 0xeb86d391u, 21);
#undef ZF_STEP
#undef ZF_F
#undef ZF_G
#undef ZF_H
#undef ZF_I
        s_[0] += a;
        s_[1] += b;
        s_[2] += c;
        s_[3] += d;
    }
    uint32_t s_[4];
    uint64_t len_;
    uint8_t blk_[64];
    size_t fill_;
};

}  // namespace zflac
