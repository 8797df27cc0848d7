/*
 * abi_consumer.c -- the C twin of zig/zflac_hip.zig: a consumer of include/zflac_hip.h
 * written against the header alone, compiled with `gcc -std=c11 -Wall -Wextra -Werror
 * -pedantic` (tests/test_c_consumer.py).
 *
 * It checks what the Zig shim relies on:
 *  - the layout of zflac_info / zflac_stream as a Zig `extern struct` (C layout) sees it:
 *    the offsets and sizes the shim's comptime block asserts;
 *  - the error mapping: shim_error_name() is the shim's `check` switch, one case per
 *    ZFLAC_E_* code, and must agree with zflac_hip_error_name() for every code;
 *  - the two-phase contract with caller memory: zflac_hip_open -> aligned_alloc(32, ...)
 *    (src/zflac.zig:331 allocates the backing 32-byte aligned) -> zflac_hip_read ->
 *    zflac_hip_close, the samples handed back in the caller's buffer.
 *
 * Usage:
 *   abi_consumer names                      every code: shim switch vs library name
 *   abi_consumer decode IN OUT [IN OUT...]  decode each stream, write its samples, print
 *                                           one JSON line {rc, error, channels, ...} each
 *                                           (one process: the device context is made once)
 */
#include <stdalign.h>
#include <stddef.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "zflac_hip.h"

/* zig/zflac_hip.zig comptime block: the same numbers */
_Static_assert(sizeof(zflac_info) == 24, "zflac_info size");
_Static_assert(offsetof(zflac_info, channels) == 0, "channels");
_Static_assert(offsetof(zflac_info, bits_per_sample) == 1, "bits_per_sample");
_Static_assert(offsetof(zflac_info, sample_kind) == 2, "sample_kind");
_Static_assert(offsetof(zflac_info, reserved) == 3, "reserved");
_Static_assert(offsetof(zflac_info, sample_rate) == 4, "sample_rate");
_Static_assert(offsetof(zflac_info, n_samples) == 8, "n_samples");
_Static_assert(offsetof(zflac_info, samples_bytes) == 16, "samples_bytes");
_Static_assert(alignof(zflac_info) == 8, "zflac_info alignment");
_Static_assert(sizeof(zflac_stream) == 2 * sizeof(size_t), "zflac_stream size");
_Static_assert(offsetof(zflac_stream, data) == 0, "zflac_stream.data");
_Static_assert(offsetof(zflac_stream, len) == sizeof(void *), "zflac_stream.len");
_Static_assert(ZFLAC_S8 == 0 && ZFLAC_S16 == 1 && ZFLAC_S32 == 2, "Samples arms");

/* zig/zflac_hip.zig `check`: ZFLAC_E_* -> the Zig error name (DeviceError for unknown codes) */
static const char *shim_error_name(int rc) {
    switch (rc) {
        case ZFLAC_OK: return "OK";
        case ZFLAC_E_INVALID_SIGNATURE: return "InvalidSignature";
        case ZFLAC_E_INVALID_METADATA_HEADER: return "InvalidMetadataHeader";
        case ZFLAC_E_MISSING_STREAMINFO: return "MissingStreaminfo";
        case ZFLAC_E_UNIMPLEMENTED: return "Unimplemented";
        case ZFLAC_E_INVALID_CHECKSUM: return "InvalidChecksum";
        case ZFLAC_E_INVALID_FRAME_HEADER: return "InvalidFrameHeader";
        case ZFLAC_E_INCONSISTENT_PARAMETERS: return "InconsistentParameters";
        case ZFLAC_E_INVALID_CODED_NUMBER: return "InvalidCodedNumber";
        case ZFLAC_E_INVALID_SUBFRAME_HEADER: return "InvalidSubframeHeader";
        case ZFLAC_E_INVALID_RESIDUAL_CODING: return "InvalidResidualCodingMethod";
        case ZFLAC_E_END_OF_STREAM: return "EndOfStream";
        case ZFLAC_E_OUT_OF_MEMORY: return "OutOfMemory";
        case ZFLAC_E_DEVICE: return "DeviceError";
        case ZFLAC_E_INVALID_ARGUMENT: return "InvalidArgument";
        case ZFLAC_E_OUT_OF_DOMAIN: return "OutOfDomain";
        case ZFLAC_E_FRAME_CRC: return "FrameCrcMismatch";
        default: return "DeviceError";
    }
}

static int names(void) {
    int bad = 0;
    for (int rc = 0; rc <= 16; rc++) {
        const char *lib = zflac_hip_error_name(rc);
        if (strcmp(lib, shim_error_name(rc)) != 0) {
            printf("code %d: shim %s, library %s\n", rc, shim_error_name(rc), lib);
            bad = 1;
        }
    }
    printf("{\"names\": %s, \"abi\": %d}\n", bad ? "false" : "true", zflac_hip_abi_version());
    return bad || zflac_hip_abi_version() != ZFLAC_HIP_ABI_VERSION;
}

static unsigned char *slurp(const char *path, size_t *len) {
    FILE *f = fopen(path, "rb");
    if (!f) return NULL;
    if (fseek(f, 0, SEEK_END) != 0) { fclose(f); return NULL; }
    const long n = ftell(f);
    if (n < 0 || fseek(f, 0, SEEK_SET) != 0) { fclose(f); return NULL; }
    unsigned char *buf = malloc(n > 0 ? (size_t)n : 1);
    if (buf && n > 0 && fread(buf, 1, (size_t)n, f) != (size_t)n) { free(buf); buf = NULL; }
    fclose(f);
    *len = (size_t)n;
    return buf;
}

static int decode(const char *in, const char *out) {
    size_t len = 0;
    unsigned char *bytes = slurp(in, &len);
    if (!bytes) { fprintf(stderr, "cannot read %s\n", in); return 2; }

    zflac_info info;
    memset(&info, 0, sizeof info);
    zflac_batch *h = NULL;
    int rc = zflac_hip_open(bytes, len, 0, &h, &info);
    void *backing = NULL;
    if (rc == ZFLAC_OK) {
        /* aligned_alloc wants a size that is a multiple of the alignment */
        const size_t cap = (size_t)((info.samples_bytes + 31u) & ~(uint64_t)31u);
        backing = aligned_alloc(32, cap ? cap : 32);
        if (!backing) {
            rc = ZFLAC_E_OUT_OF_MEMORY;
        } else if (((uintptr_t)backing & 31u) != 0) {
            fprintf(stderr, "aligned_alloc(32) returned a misaligned pointer\n");
            rc = ZFLAC_E_INVALID_ARGUMENT;
        } else {
            rc = zflac_hip_read(h, backing, (size_t)info.samples_bytes);
        }
    }
    zflac_hip_close(h);
    free(bytes);

    if (rc == ZFLAC_OK) {
        FILE *f = fopen(out, "wb");
        if (!f || fwrite(backing, 1, (size_t)info.samples_bytes, f) != (size_t)info.samples_bytes) {
            fprintf(stderr, "cannot write %s\n", out);
            if (f) fclose(f);
            free(backing);
            return 2;
        }
        fclose(f);
    }
    free(backing);
    printf("{\"rc\": %d, \"error\": \"%s\", \"library_name\": \"%s\", \"channels\": %u, \"bits_per_sample\": %u, "
           "\"sample_kind\": %u, \"sample_rate\": %u, \"n_samples\": %llu, \"samples_bytes\": %llu}\n",
           rc, shim_error_name(rc), zflac_hip_error_name(rc), (unsigned)info.channels, (unsigned)info.bits_per_sample,
           (unsigned)info.sample_kind, (unsigned)info.sample_rate, (unsigned long long)info.n_samples,
           (unsigned long long)info.samples_bytes);
    return 0;
}

int main(int argc, char **argv) {
    if (argc == 2 && strcmp(argv[1], "names") == 0) return names();
    if (argc >= 4 && argc % 2 == 0 && strcmp(argv[1], "decode") == 0) {
        for (int i = 2; i < argc; i += 2)
            if (decode(argv[i], argv[i + 1]) != 0) return 2;
        return 0;
    }
    fprintf(stderr, "usage: %s names | decode IN.flac OUT.raw [IN.flac OUT.raw ...]\n", argv[0]);
    return 2;
}
