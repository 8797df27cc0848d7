/*
 * zflac_oracle.c -- TEST INFRASTRUCTURE ONLY (see zflac_oracle.h).
 *
 * A plain-C restatement of the decode semantics of Senryoku/zflac @ 2025-08-08:
 *   src/zflac.zig      (666 lines)  -- format parse, subframes, residuals, MD5, justify
 *   src/bit_reader.zig (126 lines)  -- MSB-first bit reader
 * Each function below cites the reference lines whose behaviour it restates.
 * It is not a translation: the bit reader is a 64-bit window over an in-memory
 * buffer (same bits, same EOF points as the byte-at-a-time Zig reader), arithmetic
 * is done in int64 and wrapped to the reference's InterType/SampleType widths.
 *
 * Domain: zflac CI runs Debug (.github/workflows/tests.yml:22-23); Debug traps on
 * integer overflow, out-of-range @intCast and `unreachable`. Inputs that would trap
 * are reported as ZFO_E_OUT_OF_DOMAIN. Built with
 * -DZFO_RELEASE_FAST the checks are compiled out (used only to time a ReleaseFast-like
 * CPU baseline on in-domain inputs, whose output must equal the checked build's).
 */
#include "zflac_oracle.h"

#include <stdlib.h>
#include <string.h>

#ifdef ZFO_RELEASE_FAST
#define DOMAIN(c) ((void)0)
#else
#define DOMAIN(c)                                  \
    do {                                           \
        if (!(c)) return ZFO_E_OUT_OF_DOMAIN;      \
    } while (0)
#endif
#define TRY(x)                 \
    do {                       \
        int e_ = (x);          \
        if (e_) return e_;     \
    } while (0)

int zfo_is_release_fast(void) {
#ifdef ZFO_RELEASE_FAST
    return 1;
#else
    return 0;
#endif
}

const char *zfo_error_name(int code) {
    switch (code) {
        case ZFO_OK: return "OK";
        case ZFO_E_INVALID_SIGNATURE: return "InvalidSignature";
        case ZFO_E_INVALID_METADATA_HEADER: return "InvalidMetadataHeader";
        case ZFO_E_MISSING_STREAMINFO: return "MissingStreaminfo";
        case ZFO_E_UNIMPLEMENTED: return "Unimplemented";
        case ZFO_E_INVALID_CHECKSUM: return "InvalidChecksum";
        case ZFO_E_INVALID_FRAME_HEADER: return "InvalidFrameHeader";
        case ZFO_E_INCONSISTENT_PARAMETERS: return "InconsistentParameters";
        case ZFO_E_INVALID_CODED_NUMBER: return "InvalidCodedNumber";
        case ZFO_E_INVALID_SUBFRAME_HEADER: return "InvalidSubframeHeader";
        case ZFO_E_INVALID_RESIDUAL_CODING: return "InvalidResidualCodingMethod";
        case ZFO_E_END_OF_STREAM: return "EndOfStream";
        case ZFO_E_OUT_OF_MEMORY: return "OutOfMemory";
        case ZFO_E_DEVICE: return "DeviceError";
        case ZFO_E_INVALID_ARGUMENT: return "InvalidArgument";
        case ZFO_E_OUT_OF_DOMAIN: return "OutOfDomain";
        default: return "Unknown";
    }
}

/* ------------------------------------------------------------------------- */
/* MD5, RFC 1321 (zflac uses std.crypto.hash.Md5: src/zflac.zig:267-280).     */
/* ------------------------------------------------------------------------- */
typedef struct {
    uint32_t h[4];
    uint64_t total;
    uint8_t buf[64];
    size_t nbuf;
} md5_ctx;

static const uint32_t MD5_K[64] = {
    0xd76aa478, 0xe8c7b756, 0x242070db, 0xc1bdceee, 0xf57c0faf, 0x4787c62a, 0xa8304613, 0xfd469501,
    0x698098d8, 0x8b44f7af, 0xffff5bb1, 0x895cd7be, 0x6b901122, 0xfd987193, 0xa679438e, 0x49b40821,
    0xf61e2562, 0xc040b340, 0x265e5a51, 0xe9b6c7aa, 0xd62f105d, 0x02441453, 0xd8a1e681, 0xe7d3fbc8,
    0x21e1cde6, 0xc33707d6, 0xf4d50d87, 0x455a14ed, 0xa9e3e905, 0xfcefa3f8, 0x676f02d9, 0x8d2a4c8a,
    0xfffa3942, 0x8771f681, 0x6d9d6122, 0xfde5380c, 0xa4beea44, 0x4bdecfa9, 0xf6bb4b60, 0xbebfbc70,
    0x289b7ec6, 0xeaa127fa, 0xd4ef3085, 0x04881d05, 0xd9d4d039, 0xe6db99e5, 0x1fa27cf8, 0xc4ac5665,
    0xf4292244, 0x432aff97, 0xab9423a7, 0xfc93a039, 0x655b59c3, 0x8f0ccc92, 0xffeff47d, 0x85845dd1,
    0x6fa87e4f, 0xfe2ce6e0, 0xa3014314, 0x4e0811a1, 0xf7537e82, 0xbd3af235, 0x2ad7d2bb, 0xeb86d391};
static const uint8_t MD5_R[64] = {7, 12, 17, 22, 7, 12, 17, 22, 7, 12, 17, 22, 7, 12, 17, 22,
                                  5, 9,  14, 20, 5, 9,  14, 20, 5, 9,  14, 20, 5, 9,  14, 20,
                                  4, 11, 16, 23, 4, 11, 16, 23, 4, 11, 16, 23, 4, 11, 16, 23,
                                  6, 10, 15, 21, 6, 10, 15, 21, 6, 10, 15, 21, 6, 10, 15, 21};

static void md5_block(uint32_t h[4], const uint8_t *p) {
    uint32_t m[16];
    for (int i = 0; i < 16; i++)
        m[i] = (uint32_t)p[4 * i] | ((uint32_t)p[4 * i + 1] << 8) | ((uint32_t)p[4 * i + 2] << 16) |
               ((uint32_t)p[4 * i + 3] << 24);
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3];
    for (int i = 0; i < 64; i++) {
        uint32_t f;
        int g;
        if (i < 16) { f = (b & c) | (~b & d); g = i; }
        else if (i < 32) { f = (d & b) | (~d & c); g = (5 * i + 1) & 15; }
        else if (i < 48) { f = b ^ c ^ d; g = (3 * i + 5) & 15; }
        else { f = c ^ (b | ~d); g = (7 * i) & 15; }
        uint32_t t = d;
        d = c;
        c = b;
        uint32_t x = a + f + MD5_K[i] + m[g];
        b = b + ((x << MD5_R[i]) | (x >> (32 - MD5_R[i])));
        a = t;
    }
    h[0] += a; h[1] += b; h[2] += c; h[3] += d;
}

static void md5_init(md5_ctx *c) {
    c->h[0] = 0x67452301; c->h[1] = 0xefcdab89; c->h[2] = 0x98badcfe; c->h[3] = 0x10325476;
    c->total = 0; c->nbuf = 0;
}
static void md5_update(md5_ctx *c, const uint8_t *p, size_t n) {
    c->total += n;
    if (c->nbuf) {
        size_t t = 64 - c->nbuf;
        if (t > n) t = n;
        memcpy(c->buf + c->nbuf, p, t);
        c->nbuf += t; p += t; n -= t;
        if (c->nbuf == 64) { md5_block(c->h, c->buf); c->nbuf = 0; }
    }
    while (n >= 64) { md5_block(c->h, p); p += 64; n -= 64; }
    if (n) { memcpy(c->buf, p, n); c->nbuf = n; }
}
static void md5_final(md5_ctx *c, uint8_t out[16]) {
    uint64_t bits = c->total * 8;
    uint8_t pad = 0x80;
    md5_update(c, &pad, 1);
    uint8_t z = 0;
    while (c->nbuf != 56) md5_update(c, &z, 1);
    uint8_t len[8];
    for (int i = 0; i < 8; i++) len[i] = (uint8_t)(bits >> (8 * i));
    md5_update(c, len, 8);
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++) out[4 * i + j] = (uint8_t)(c->h[i] >> (8 * j));
}
void zfo_md5(const uint8_t *data, size_t len, uint8_t digest[16]) {
    md5_ctx c;
    md5_init(&c);
    md5_update(&c, data, len);
    md5_final(&c, digest);
}

/* ------------------------------------------------------------------------- */
/* L0/L1: byte reader + MSB-first bit reader.                                 */
/* Restates the observable behaviour of std.io's readInt/readByte/skipBytes and */
/* src/bit_reader.zig:25-120: bits are consumed MSB first; a read fails with  */
/* EndOfStream exactly when it needs a byte past the end; alignToByte          */
/* (bit_reader.zig:90-93) drops the rest of the current byte.                 */
/* ------------------------------------------------------------------------- */
typedef struct {
    const uint8_t *d;
    size_t n;      /* bytes */
    uint64_t bp;   /* bit position; byte-reader position is bp/8 when aligned */
    uint64_t end;  /* n*8 */
} rd;

static inline uint64_t peek64(const rd *r) {
    size_t i = (size_t)(r->bp >> 3);
    unsigned s = (unsigned)(r->bp & 7);
    uint64_t v;
    uint8_t nx;
    if (i + 9 <= r->n) {
        memcpy(&v, r->d + i, 8);
        v = __builtin_bswap64(v);
        nx = r->d[i + 8];
    } else {
        uint8_t t[9] = {0};
        if (i < r->n) memcpy(t, r->d + i, (r->n - i) < 9 ? (r->n - i) : 9);
        memcpy(&v, t, 8);
        v = __builtin_bswap64(v);
        nx = t[8];
    }
    if (s) v = (v << s) | (uint64_t)(nx >> (8 - s));
    return v;
}

/* readBitsNoEof (bit_reader.zig:25-70), n in [0,64] */
static inline int rd_bits(rd *r, unsigned n, uint64_t *out) {
    if (r->bp + n > r->end) return ZFO_E_END_OF_STREAM;
    uint64_t v = peek64(r);
    *out = n ? (v >> (64 - n)) : 0;
    r->bp += n;
    return 0;
}

/* readUnary (bit_reader.zig:95-120): number of 0 bits before the next 1 bit. */
static inline int rd_unary(rd *r, uint64_t *out) {
    uint64_t q = 0;
    for (;;) {
        if (r->bp >= r->end) return ZFO_E_END_OF_STREAM;
        uint64_t v = peek64(r);
        if (v) {
            unsigned z = (unsigned)__builtin_clzll(v);
            if (r->bp + z + 1 > r->end) return ZFO_E_END_OF_STREAM;
            r->bp += z + 1;
            *out = q + z;
            return 0;
        }
        if (r->end - r->bp <= 64) return ZFO_E_END_OF_STREAM;
        r->bp += 64;
        q += 64;
    }
}

static inline void rd_align(rd *r) { r->bp = (r->bp + 7) & ~(uint64_t)7; }

/* std.io readInt(uN, .big) on a byte-aligned reader */
static inline int rd_be(rd *r, unsigned nbytes, uint64_t *out) { return rd_bits(r, 8 * nbytes, out); }

/* read_signed_integer (src/zflac.zig:188-196): n-bit two's complement, sign-extended.
 * The Zig assert `bit_depth > 0 and bit_depth <= @bitSizeOf(T)` is the DOMAIN check
 * done by callers. */
static inline int rd_signed(rd *r, unsigned n, int64_t *out) {
    uint64_t v;
    TRY(rd_bits(r, n, &v));
    *out = n ? (int64_t)(v << (64 - n)) >> (64 - n) : 0;
    return 0;
}

/* ------------------------------------------------------------------------- */
/* Integer width helpers: InterType/SampleType emulation.                     */
/* ------------------------------------------------------------------------- */
static inline int64_t wrap_bits(int64_t v, unsigned bits) {
    if (bits >= 64) return v;
    return (int64_t)((uint64_t)v << (64 - bits)) >> (64 - bits);
}
static inline int fits_bits(int64_t v, unsigned bits) {
    if (bits >= 64) return 1;
    int64_t lo = -((int64_t)1 << (bits - 1)), hi = ((int64_t)1 << (bits - 1)) - 1;
    return v >= lo && v <= hi;
}

typedef struct {
    unsigned sbits; /* SampleType width: 8 / 16 / 32 */
    unsigned ibits; /* InterType width: 16 / 32 / 64 (src/zflac.zig:314-319) */
} widths;

/* read_unencoded_sample (src/zflac.zig:198-201): reads bps-wasted bits into the
 * next-wider InterType, then @intCast to SampleType. */
static inline int rd_unencoded(rd *r, const widths *w, unsigned wasted, unsigned bps, int64_t *out) {
    (void)w;
    DOMAIN(bps >= wasted);             /* u6 subtraction underflow */
    unsigned n = bps - wasted;
    DOMAIN(n > 0 && n <= w->ibits);    /* read_signed_integer assert */
    int64_t v;
    TRY(rd_signed(r, n, &v));
    DOMAIN(fits_bits(v, w->sbits));    /* @intCast(.., SampleType) */
    *out = v;
    return 0;
}

/* ------------------------------------------------------------------------- */
/* Residuals: decode_residuals / decode_residual_partition                    */
/* (src/zflac.zig:614-666).                                                   */
/* ------------------------------------------------------------------------- */
static int decode_residuals(rd *r, const widths *w, int64_t *res, unsigned bs, unsigned order) {
    uint64_t method, po;
    TRY(rd_bits(r, 2, &method));                           /* :617 */
    if (method >= 2) return ZFO_E_INVALID_RESIDUAL_CODING; /* :618 */
    TRY(rd_bits(r, 4, &po));                               /* :619 */
    unsigned psize = bs >> po;
    DOMAIN(psize >= order);                 /* :626 u16 `count -= order` underflow */
    DOMAIN(((uint64_t)psize << po) == bs);  /* residuals past the last partition would keep
                                               stale working-buffer values (:623-632) */
    const unsigned kbits = method ? 5 : 4;  /* :637-640 */
    const unsigned escape = method ? 31 : 15;
    const unsigned W = w->ibits;
    const uint64_t wmask = (W >= 64) ? ~(uint64_t)0 : (((uint64_t)1 << W) - 1);
    unsigned idx = 0;
    for (unsigned p = 0; p < (1u << po); p++) {
        unsigned count = psize - (p == 0 ? order : 0); /* :625-626 */
        uint64_t k;
        TRY(rd_bits(r, kbits, &k)); /* :642 */
        if (k == escape) {          /* :646-654 escape: raw signed residuals */
            uint64_t bd;
            TRY(rd_bits(r, 5, &bd));
            if (bd == 0) {
                memset(res + idx, 0, sizeof(int64_t) * count);
            } else {
                DOMAIN(bd <= W);
                for (unsigned i = 0; i < count; i++) TRY(rd_signed(r, (unsigned)bd, &res[idx + i]));
            }
        } else {                       /* :655-664 Rice */
            DOMAIN(k < W);             /* :656 unreachable */
            for (unsigned i = 0; i < count; i++) {
                uint64_t q, rem;
                TRY(rd_unary(r, &q));
                DOMAIN(W >= 64 || q <= wmask); /* @intCast(readUnary()) to UnsignedResidualType */
                TRY(rd_bits(r, (unsigned)k, &rem));
                uint64_t zz = ((q << k) & wmask) + rem; /* `<<` discards, `+` cannot carry */
                uint64_t u = (zz >> 1) ^ (0 - (zz & 1));
                res[idx + i] = wrap_bits((int64_t)(u & wmask), W);
            }
        }
        idx += count;
    }
    return 0;
}

/* Checked InterType arithmetic (Debug overflow traps). */
static inline int chk_add(int64_t a, int64_t b, unsigned W, int64_t *out) {
    int64_t s;
#ifndef ZFO_RELEASE_FAST
    if (__builtin_add_overflow(a, b, &s)) return ZFO_E_OUT_OF_DOMAIN;
    if (!fits_bits(s, W)) return ZFO_E_OUT_OF_DOMAIN;
#else
    s = (int64_t)((uint64_t)a + (uint64_t)b);
    s = wrap_bits(s, W);
#endif
    *out = s;
    return 0;
}

/* LPC / fixed recurrence. zflac: fixed (:481-490), LPC orders 1..31 unrolled (:526-533),
 * order 32 via @Vector + @reduce (:525, linear_predictor :604-612). All three compute
 * s[i] += (sum_{o<order} s[i-order+o]*coef[o]) >> shift in InterType. coef[] is stored
 * in bitstream-reversed order as in :512-514. */
static int run_predictor(const widths *w, int64_t *s, unsigned bs, unsigned order, const int64_t *coef,
                         unsigned shift) {
    const unsigned W = w->ibits;
#ifdef ZFO_RELEASE_FAST
    /* ReleaseFast-like: wrapping arithmetic, no checks. Unrolled per order class. */
#define PRED_LOOP(N)                                                          \
    for (unsigned i = (N); i < bs; i++) {                                     \
        uint64_t p = 0;                                                       \
        for (unsigned o = 0; o < (N); o++) p += (uint64_t)(s[i - (N) + o] * coef[o]); \
        int64_t pw = wrap_bits((int64_t)p, W);                                \
        s[i] = wrap_bits((int64_t)((uint64_t)s[i] + (uint64_t)(pw >> shift)), W); \
    }
    switch (order) {
        case 1: PRED_LOOP(1) break;
        case 2: PRED_LOOP(2) break;
        case 3: PRED_LOOP(3) break;
        case 4: PRED_LOOP(4) break;
        case 8: PRED_LOOP(8) break;
        case 12: PRED_LOOP(12) break;
        case 16: PRED_LOOP(16) break;
        case 32: PRED_LOOP(32) break;
        default: {
            for (unsigned i = order; i < bs; i++) {
                uint64_t p = 0;
                for (unsigned o = 0; o < order; o++) p += (uint64_t)(s[i - order + o] * coef[o]);
                int64_t pw = wrap_bits((int64_t)p, W);
                s[i] = wrap_bits((int64_t)((uint64_t)s[i] + (uint64_t)(pw >> shift)), W);
            }
        }
    }
#undef PRED_LOOP
#else
    for (unsigned i = order; i < bs; i++) {
        int64_t p = 0;
        for (unsigned o = 0; o < order; o++) {
            int64_t prod;
            if (__builtin_mul_overflow(s[i - order + o], coef[o], &prod)) return ZFO_E_OUT_OF_DOMAIN;
            DOMAIN(fits_bits(prod, W));
            TRY(chk_add(p, prod, W, &p));
        }
        TRY(chk_add(s[i], p >> shift, W, &s[i]));
    }
#endif
    return 0;
}

/* ------------------------------------------------------------------------- */
/* Frame header helpers (src/zflac.zig:57-173, 203-214).                      */
/* ------------------------------------------------------------------------- */
/* read_coded_number (src/zflac.zig:203-214) */
static int read_coded_number(rd *r, uint64_t *out) {
    uint64_t b;
    TRY(rd_be(r, 1, &b));
    unsigned ones = 0;
    while (ones < 8 && (b & (0x80u >> ones))) ones++; /* @clz(first_byte ^ 0xFF) */
    if (b == 0xFF || ones == 1) return ZFO_E_INVALID_CODED_NUMBER;
    if (ones == 0) { *out = b; return 0; }
    uint64_t v = b & (0x7Fu >> ones);
    for (unsigned i = 0; i + 1 < ones; i++) {
        uint64_t c;
        TRY(rd_be(r, 1, &c));
        v = (v << 6) | (c & 0x3F); /* continuation bytes are not validated (:209-212) */
    }
    *out = v;
    return 0;
}

/* Channels.count (src/zflac.zig:107-122) */
static unsigned channels_count(unsigned code) {
    if (code <= 7) return code + 1;
    if (code <= 10) return 2;
    return 0;
}
/* SampleRate.hz (src/zflac.zig:75-90) for table codes 1..11 */
static uint32_t rate_hz(unsigned code) {
    static const uint32_t t[12] = {0, 88200, 176400, 192000, 8000, 16000, 22050, 24000, 32000, 44100, 48000, 96000};
    return t[code];
}

typedef struct {
    uint16_t min_block, max_block;
    uint32_t min_frame, max_frame, sample_rate;
    uint8_t channel_count; /* minus 1 */
    uint8_t sample_bit_depth; /* minus 1 */
    uint64_t number_of_samples;
    uint8_t md5[16];
} streaminfo;

/* One subframe: src/zflac.zig:425-544. `sub` points at out[frame_offset + channel]. */
static int decode_subframe(rd *r, const widths *w, unsigned channel, unsigned chan_code, unsigned nch,
                           unsigned bps, unsigned bs, int32_t *sub, int64_t *wbuf) {
    uint64_t zero, type, wflag;
    TRY(rd_bits(r, 1, &zero));
    TRY(rd_bits(r, 6, &type));
    TRY(rd_bits(r, 1, &wflag));
    if (zero != 0) return ZFO_E_INVALID_SUBFRAME_HEADER; /* :431 */
    unsigned wasted = 0;
    if (wflag) { /* :433 */
        uint64_t u;
        TRY(rd_unary(r, &u));
        DOMAIN(u + 1 < 64); /* @intCast to u6 */
        wasted = (unsigned)u + 1;
    }
    /* side channel carries one extra bit (:436-441) */
    unsigned ubps = bps;
    if ((chan_code == 8 && channel == 1) || (chan_code == 9 && channel == 0) || (chan_code == 10 && channel == 1))
        ubps = bps + 1;
    const unsigned SB = w->sbits;

    if (type == 0) { /* constant (:445-454); reads bits_per_sample, not the side depth */
        int64_t v;
        TRY(rd_unencoded(r, w, wasted, bps, &v));
        DOMAIN(wasted < SB); /* @intCast(wasted_bits) to Log2Int(SampleType) */
        int32_t sv = (int32_t)wrap_bits((int64_t)((uint64_t)v << wasted), SB);
        for (unsigned i = 0; i < bs; i++) sub[(size_t)nch * i] = sv;
        return 0;
    }
    if (type == 1) { /* verbatim (:455-465) */
        if (wasted > 0) DOMAIN(wasted < SB);
        for (unsigned i = 0; i < bs; i++) {
            int64_t v;
            TRY(rd_unencoded(r, w, wasted, ubps, &v));
            if (wasted > 0) v = wrap_bits((int64_t)((uint64_t)v << wasted), SB);
            sub[(size_t)nch * i] = (int32_t)v;
        }
        return 0;
    }
    unsigned order;
    int64_t coef[32];
    unsigned shift = 0;
    if (type >= 8 && type <= 12) { /* fixed predictor (:466-498) */
        order = (unsigned)(type & 7);
        /* (order > 4) -> InvalidSubframeHeader at :471 cannot trigger for 8..12 */
        for (unsigned i = 0; i < order; i++) TRY(rd_unencoded(r, w, wasted, ubps, &wbuf[i]));
        /* The fixed polynomials of :481-490, written as reversed LPC coefficients
         * with shift 0 (same InterType arithmetic). */
        static const int64_t F[5][4] = {{0}, {1}, {-1, 2}, {1, -3, 3}, {-1, 4, -6, 4}};
        for (unsigned o = 0; o < order; o++) coef[o] = F[order][o];
    } else if (type >= 32) { /* LPC (:499-541) */
        order = (unsigned)type - 31;
        for (unsigned i = 0; i < order; i++) TRY(rd_unencoded(r, w, wasted, ubps, &wbuf[i]));
        uint64_t pc, sh;
        TRY(rd_bits(r, 4, &pc));
        DOMAIN(pc != 15); /* `readBitsNoEof(u4,4) + 1` overflows u4 (:508) */
        unsigned prec = (unsigned)pc + 1;
        TRY(rd_bits(r, 5, &sh)); /* unsigned u5 shift (:510) */
        shift = (unsigned)sh;
        DOMAIN(shift < w->ibits); /* @intCast(shift) to Log2Int(InterType) (:531) */
        for (unsigned i = 0; i < order; i++) { /* stored reversed (:512-514) */
            int64_t c;
            TRY(rd_signed(r, prec, &c));
            coef[order - 1 - i] = c;
        }
    } else {
        return ZFO_E_INVALID_SUBFRAME_HEADER; /* reserved types (:542) */
    }
    TRY(decode_residuals(r, w, wbuf + order, bs, order));
    if (order > 0) TRY(run_predictor(w, wbuf, bs, order, coef, shift));
    /* interleave + wasted shift (:492-497, :535-540) */
    if (wasted > 0) DOMAIN(wasted < SB);
    for (unsigned i = 0; i < bs; i++) {
        int64_t v = wbuf[i];
        DOMAIN(fits_bits(v, SB)); /* @intCast(samples_working_buffer[i]) */
        if (wasted > 0) v = wrap_bits((int64_t)((uint64_t)v << wasted), SB);
        sub[(size_t)nch * i] = (int32_t)v;
    }
    return 0;
}

/* Stereo decorrelation (src/zflac.zig:553-578) on one interleaved frame. */
static int decorrelate(const widths *w, unsigned chan_code, int32_t *f, unsigned bs) {
    const unsigned SB = w->sbits, W = w->ibits;
    if (chan_code == 8) { /* left/side: R = L - S in SampleType (:555-560) */
        for (unsigned i = 0; i < bs; i++) {
            int64_t v = (int64_t)f[2 * i] - f[2 * i + 1];
            DOMAIN(fits_bits(v, SB));
            f[2 * i + 1] = (int32_t)wrap_bits(v, SB);
        }
    } else if (chan_code == 9) { /* side/right: L = S + R (:561-566) */
        for (unsigned i = 0; i < bs; i++) {
            int64_t v = (int64_t)f[2 * i] + f[2 * i + 1];
            DOMAIN(fits_bits(v, SB));
            f[2 * i] = (int32_t)wrap_bits(v, SB);
        }
    } else if (chan_code == 10) { /* mid/side in InterType (:567-576) */
        for (unsigned i = 0; i < bs; i++) {
            int64_t mid = wrap_bits((int64_t)((uint64_t)(int64_t)f[2 * i] << 1), W);
            int64_t side = f[2 * i + 1];
            mid += side & 1;
            int64_t l = (mid + side) >> 1, rr = (mid - side) >> 1;
            DOMAIN(fits_bits(mid + side, W) && fits_bits(mid - side, W));
            DOMAIN(fits_bits(l, SB) && fits_bits(rr, SB));
            f[2 * i] = (int32_t)wrap_bits(l, SB);
            f[2 * i + 1] = (int32_t)wrap_bits(rr, SB);
        }
    }
    return 0;
}

/* decode_frames (src/zflac.zig:312-602). Output: int32 interleaved values already
 * wrapped to SampleType width. */
static int decode_frames(rd *r, const widths *w, const streaminfo *si, int32_t **out_samples, uint64_t *out_len,
                         uint8_t *out_ch, uint32_t *out_rate, uint8_t *out_bps) {
    int first = 1;
    uint32_t sample_rate = 0;
    unsigned channel_count = 0, depth_code = 0, bps = 0;
    int valid_total = si->number_of_samples > 0; /* :327 */
    const uint64_t expected_ch = (uint64_t)si->channel_count + 1;
    const uint64_t total = expected_ch * (valid_total ? si->number_of_samples : 4096); /* :330 */
    uint64_t cap = total;
    int32_t *samples = (int32_t *)malloc((cap ? cap : 1) * sizeof(int32_t));
    if (!samples) return ZFO_E_OUT_OF_MEMORY;
    size_t wcap = si->max_block ? si->max_block : 4096; /* :336 */
    int64_t *wbuf = (int64_t *)malloc(wcap * sizeof(int64_t));
    if (!wbuf) { free(samples); return ZFO_E_OUT_OF_MEMORY; }
    uint64_t offset = 0;
    int err = 0;

    for (;;) {
        if (valid_total && offset >= total) break; /* :341 */
        uint64_t hdr;
        if (r->bp + 32 > r->end) { /* readInt(u32) at EOF (:343-350) */
            if (valid_total) { err = ZFO_E_END_OF_STREAM; goto fail; }
            break;
        }
        rd_be(r, 4, &hdr);
        const unsigned b1 = (hdr >> 16) & 0xFF, b2 = (hdr >> 8) & 0xFF, b3 = hdr & 0xFF;
        if ((hdr >> 17) != (0xFFF8 >> 1)) { err = ZFO_E_INVALID_FRAME_HEADER; goto fail; } /* :351-352 */
        (void)b1;
        uint64_t coded;
        if ((err = read_coded_number(r, &coded))) goto fail; /* :354 */
        const unsigned bs_code = b2 >> 4, rate_code = b2 & 15, ch_code = b3 >> 4, dcode = (b3 >> 1) & 7;
        unsigned bs; /* :356-365 */
        if (bs_code == 0) { err = ZFO_E_INVALID_FRAME_HEADER; goto fail; }
        else if (bs_code == 6) { uint64_t v; if ((err = rd_be(r, 1, &v))) goto fail; bs = (unsigned)v + 1; }
        else if (bs_code == 7) {
            uint64_t v;
            if ((err = rd_be(r, 2, &v))) goto fail;
            if (v == 0xFFFF) { err = ZFO_E_INVALID_FRAME_HEADER; goto fail; }
            bs = (unsigned)v + 1;
        } else if (bs_code == 1) bs = 192;
        else if (bs_code <= 5) bs = 144u << bs_code;
        else bs = 1u << bs_code;
        uint32_t frate; /* :367-374 */
        if (rate_code == 0) frate = si->sample_rate;
        else if (rate_code == 12) { uint64_t v; if ((err = rd_be(r, 1, &v))) goto fail; frate = (uint32_t)v; } /* Hz, not kHz */
        else if (rate_code == 13) { uint64_t v; if ((err = rd_be(r, 2, &v))) goto fail; frate = (uint32_t)v; }
        else if (rate_code == 14) { uint64_t v; if ((err = rd_be(r, 2, &v))) goto fail; frate = 10u * (uint32_t)v; }
        else if (rate_code == 15) { err = ZFO_E_INVALID_FRAME_HEADER; goto fail; }
        else frate = rate_hz(rate_code);

        if (first) { /* :376-388 */
            sample_rate = frate;
            channel_count = channels_count(ch_code);
            depth_code = dcode;
            if (dcode == 0) bps = (unsigned)si->sample_bit_depth + 1;
            else {
                static const unsigned B[8] = {0, 8, 12, 0, 16, 20, 24, 32};
                if (dcode == 3) { err = ZFO_E_OUT_OF_DOMAIN; goto fail; } /* BitDepth.bps unreachable :143 */
                bps = B[dcode];
            }
            if (channel_count != expected_ch) { err = ZFO_E_INCONSISTENT_PARAMETERS; goto fail; }
            first = 0;
        } else if (sample_rate != frate || channel_count != channels_count(ch_code) || depth_code != dcode) {
            err = ZFO_E_INCONSISTENT_PARAMETERS; /* :391 (compares the depth CODE) */
            goto fail;
        }
        const uint64_t expected = offset + (uint64_t)bs * channel_count; /* :394-402 */
        if (cap < expected) {
            uint64_t ncap = 2 * cap > expected ? 2 * cap : expected;
            int32_t *ns = (int32_t *)realloc(samples, ncap * sizeof(int32_t));
            if (!ns) { err = ZFO_E_OUT_OF_MEMORY; goto fail; }
            samples = ns;
            cap = ncap;
            valid_total = 0;
        }
        if (bs == 1 && valid_total && offset + channel_count * (uint64_t)bs < total) { /* :405 */
            err = ZFO_E_INVALID_FRAME_HEADER;
            goto fail;
        }
        uint64_t crc8;
        if ((err = rd_be(r, 1, &crc8))) goto fail; /* :407, not checked */
        if (wcap < bs) {
            int64_t *nw = (int64_t *)realloc(wbuf, bs * sizeof(int64_t));
            if (!nw) { err = ZFO_E_OUT_OF_MEMORY; goto fail; }
            wbuf = nw;
            wcap = bs;
        }
        for (unsigned c = 0; c < channel_count; c++) /* :425-544 */
            if ((err = decode_subframe(r, w, c, ch_code, channel_count, bps, bs, samples + offset + c, wbuf))) goto fail;
        rd_align(r); /* :546 */
        uint64_t crc16;
        if ((err = rd_be(r, 2, &crc16))) goto fail; /* :548, not checked */
        if ((err = decorrelate(w, ch_code, samples + offset, bs))) goto fail;
        offset += (uint64_t)channel_count * bs; /* :580 */
    }
    free(wbuf);
    *out_samples = samples;
    *out_len = offset; /* trim (:583-588) */
    *out_ch = (uint8_t)channel_count;
    *out_rate = sample_rate;
    *out_bps = (uint8_t)bps;
    return 0;
fail:
    free(wbuf);
    free(samples);
    return err;
}

/* decode (src/zflac.zig:217-310) */
int zfo_decode(const uint8_t *buf, size_t len, zfo_result *res) { return zfo_decode_ex(buf, len, 0, res); }

int zfo_decode_ex(const uint8_t *buf, size_t len, int flags, zfo_result *res) {
    memset(res, 0, sizeof(*res));
    rd r = {buf, len, 0, (uint64_t)len * 8};
    uint64_t sig;
    int err = rd_be(&r, 4, &sig);
    if (err) return res->err = err;
    if (sig != 0x664C6143) return res->err = ZFO_E_INVALID_SIGNATURE; /* :218-220 */

    int have_si = 0;
    streaminfo si;
    memset(&si, 0, sizeof si);
    for (;;) { /* :223-253 */
        uint64_t h;
        if ((err = rd_be(&r, 4, &h))) return res->err = err;
        const unsigned info = (unsigned)(h >> 24) & 0x7F, last = (unsigned)(h >> 31) & 1;
        const uint64_t length = h & 0xFFFFFF;
        if (info == 0) { /* STREAMINFO: always 34 bytes, whatever `length` says (:228-240) */
            static const unsigned FW[8] = {16, 16, 24, 24, 20, 3, 5, 36};
            uint64_t f[8], v;
            for (int i = 0; i < 8; i++)
                if ((err = rd_bits(&r, FW[i], &f[i]))) return res->err = err;
            si.min_block = (uint16_t)f[0];
            si.max_block = (uint16_t)f[1];
            si.min_frame = (uint32_t)f[2];
            si.max_frame = (uint32_t)f[3];
            si.sample_rate = (uint32_t)f[4];
            si.channel_count = (uint8_t)f[5];    /* channels - 1 */
            si.sample_bit_depth = (uint8_t)f[6]; /* bits per sample - 1 */
            si.number_of_samples = f[7];
            for (int i = 0; i < 16; i++) {
                if ((err = rd_bits(&r, 8, &v))) return res->err = err;
                si.md5[i] = (uint8_t)v;
            }
            have_si = 1;
        } else if (info >= 1 && info <= 6) { /* skipped (:243-247) */
            if (r.bp + length * 8 > r.end) return res->err = ZFO_E_END_OF_STREAM;
            r.bp += length * 8;
        } else {
            return res->err = ZFO_E_INVALID_METADATA_HEADER; /* :248 */
        }
        if (last) break;
    }
    if (!have_si) return res->err = ZFO_E_MISSING_STREAMINFO; /* :309 */

    const unsigned depth = (unsigned)si.sample_bit_depth + 1; /* :256-264 */
    const unsigned aligned = (depth + 7) & ~7u;
    widths w;
    if (aligned == 8) { w.sbits = 8; w.ibits = 16; res->sample_kind = ZFO_S8; }
    else if (aligned == 16) { w.sbits = 16; w.ibits = 32; res->sample_kind = ZFO_S16; }
    else if (aligned == 24 || aligned == 32) { w.sbits = 32; w.ibits = 64; res->sample_kind = ZFO_S32; }
    else return res->err = ZFO_E_UNIMPLEMENTED;

    int32_t *s32 = NULL;
    uint64_t n = 0;
    if ((err = decode_frames(&r, &w, &si, &s32, &n, &res->channels, &res->sample_rate, &res->bits_per_sample)))
        return res->err = err;

    /* pack to the SampleType container */
    size_t esz = w.sbits / 8;
    uint8_t *out = (uint8_t *)malloc(n ? n * esz : 1);
    if (!out) { free(s32); return res->err = ZFO_E_OUT_OF_MEMORY; }
    if (esz == 1) for (uint64_t i = 0; i < n; i++) ((int8_t *)out)[i] = (int8_t)s32[i];
    else if (esz == 2) for (uint64_t i = 0; i < n; i++) ((int16_t *)out)[i] = (int16_t)s32[i];
    else memcpy(out, s32, n * 4);
    free(s32);

    /* MD5 over the output bytes; 24-bit containers hash 3 bytes per sample (:267-280).
     * ZFO_NO_MD5 skips it (timing of the decode alone; not zflac's behaviour). */
    int md5_bad = 0;
    if (!(flags & ZFO_NO_MD5)) {
        uint8_t md5[16];
        md5_ctx c;
        md5_init(&c);
        if (aligned == 24) {
            for (uint64_t i = 0; i < n; i++) md5_update(&c, out + 4 * i, 3);
        } else {
            md5_update(&c, out, n * esz);
        }
        md5_final(&c, md5);
        /* decode() fails with InvalidChecksum (:279-280); the samples are still handed back
         * (justified) so tests can compare what both decoders produced for such a stream */
        md5_bad = memcmp(md5, si.md5, 16) != 0;
    }

    /* left-justify AFTER the MD5 (:287-306) */
    if (depth >= 9 && depth <= 15) {
        for (uint64_t i = 0; i < n; i++) {
            int16_t *p = (int16_t *)out + i;
            *p = (int16_t)(uint16_t)((uint16_t)*p << (16 - depth));
        }
    } else if (depth >= 17 && depth <= 31) {
        for (uint64_t i = 0; i < n; i++) {
            int32_t *p = (int32_t *)out + i;
            *p = (int32_t)(uint32_t)((uint32_t)*p << (32 - depth));
        }
    }
    res->samples = out;
    res->n_samples = n;
    res->err = md5_bad ? ZFO_E_INVALID_CHECKSUM : 0;
    return res->err;
}

void zfo_free(zfo_result *r) {
    if (r && r->samples) {
        free(r->samples);
        r->samples = NULL;
    }
}
