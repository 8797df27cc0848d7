/*
 * zflac_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of Senryoku/zflac `decode()` (reference snapshot 2025-08-08,
 * src/zflac.zig + src/bit_reader.zig). It exists to CHECK the HIP product path
 * (libzflac_hip.so) and to time a CPU baseline. Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it. The product never links or calls it.
 *
 * Parity pinning: the restatement is pinned by the three known-answer streams of
 * tests/basic.zig:4-95 (committed as data in tests/golden/basic_kat.json) and by
 * RFC 1321 MD5 vectors. The reference itself (Zig 0.14.1) cannot be built here
 * (no zig toolchain), see DESIGN.md "Oracle".
 */
#ifndef ZFLAC_ORACLE_H
#define ZFLAC_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Error codes: 1:1 with the zflac error set. The numeric
 * values are shared with include/zflac_hip.h so tests can compare codes directly. */
enum {
    ZFO_OK = 0,
    ZFO_E_INVALID_SIGNATURE = 1,          /* src/zflac.zig:220 */
    ZFO_E_INVALID_METADATA_HEADER = 2,    /* src/zflac.zig:248 */
    ZFO_E_MISSING_STREAMINFO = 3,         /* src/zflac.zig:309 */
    ZFO_E_UNIMPLEMENTED = 4,              /* src/zflac.zig:263 */
    ZFO_E_INVALID_CHECKSUM = 5,           /* src/zflac.zig:280 */
    ZFO_E_INVALID_FRAME_HEADER = 6,       /* src/zflac.zig:352,357,361,372,405 */
    ZFO_E_INCONSISTENT_PARAMETERS = 7,    /* src/zflac.zig:386,391 */
    ZFO_E_INVALID_CODED_NUMBER = 8,       /* src/zflac.zig:206 */
    ZFO_E_INVALID_SUBFRAME_HEADER = 9,    /* src/zflac.zig:431,471,542 */
    ZFO_E_INVALID_RESIDUAL_CODING = 10,   /* src/zflac.zig:618 */
    ZFO_E_END_OF_STREAM = 11,             /* std.io reader */
    ZFO_E_OUT_OF_MEMORY = 12,             /* allocator */
    ZFO_E_DEVICE = 13,                    /* product only */
    ZFO_E_INVALID_ARGUMENT = 14,          /* product only */
    ZFO_E_OUT_OF_DOMAIN = 15              /* input where Debug zflac would trap (Appendix A) */
};

/* sample_kind: which arm of the zflac `Samples` union (src/zflac.zig:12-16) */
enum { ZFO_S8 = 0, ZFO_S16 = 1, ZFO_S32 = 2 };

typedef struct zfo_result {
    int err;
    uint8_t channels;         /* DecodedFLAC.channels        src/zflac.zig:19 */
    uint8_t bits_per_sample;  /* DecodedFLAC.bits_per_sample src/zflac.zig:21 */
    uint8_t sample_kind;      /* ZFO_S8 / ZFO_S16 / ZFO_S32 */
    uint8_t _pad;
    uint32_t sample_rate;     /* DecodedFLAC.sample_rate     src/zflac.zig:20 */
    uint64_t n_samples;       /* samples.len (channel-samples, interleaved) */
    void *samples;            /* malloc'd (kept on InvalidChecksum too); free with zfo_free */
} zfo_result;

/* Full decode() semantics: signature, metadata walk, frames, MD5 verification,
 * left-justify (src/zflac.zig:217-310). */
int zfo_decode(const uint8_t *buf, size_t len, zfo_result *out);
/* zfo_decode with options: ZFO_NO_MD5 skips the STREAMINFO MD5 (CPU timing of the decode
 * alone, beside the device decode that `bench.py`'s headline excludes MD5 from). */
#define ZFO_NO_MD5 1
int zfo_decode_ex(const uint8_t *buf, size_t len, int flags, zfo_result *out);
void zfo_free(zfo_result *r);
const char *zfo_error_name(int code);

/* RFC 1321 MD5 (stands in for Zig std.crypto.hash.Md5, not vendored). */
void zfo_md5(const uint8_t *data, size_t len, uint8_t digest[16]);

/* 1 when built with ZFO_RELEASE_FAST (Debug domain checks compiled out). */
int zfo_is_release_fast(void);

#ifdef __cplusplus
}
#endif
#endif
