/*
 * zflac_hip.h -- C ABI of the MI355X FLAC decode path (libzflac_hip.so).
 *
 * Drop-in boundary for Senryoku/zflac `pub fn decode(allocator, reader) !DecodedFLAC`
 * (src/zflac.zig:216-217). zflac's only entry point reads a whole stream through a
 * std reader and returns caller-owned samples; here the caller hands over the stream
 * bytes and receives the samples in memory it allocated itself (two-phase: open ->
 * size -> read), so a Zig shim can keep `DecodedFLAC` and its allocator contract
 * (src/zflac.zig:18-28, :331). See INTEGRATION.md for the shim.
 *
 * All decode work (frame sync scan, subframe decode, fixed/LPC rollback, wasted bits,
 * stereo decorrelation, left-justify, PCM pack-out) runs in HIP kernels on gfx950.
 * MD5 verification (src/zflac.zig:267-280) runs on the host over the PCM copied back,
 * or, for batches created with ZFLAC_FLAG_DEVICE_MD5, in a HIP kernel (k_md5).
 * There is no CPU decode fallback: without a usable GPU every call returns
 * ZFLAC_E_DEVICE.
 *
 * Thread safety: handles are independent; a handle must not be used by two threads
 * at once. No global mutable state besides a lazily initialised per-device context.
 */
#ifndef ZFLAC_HIP_H
#define ZFLAC_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Error codes, 1:1 with zflac's error set. */
#define ZFLAC_OK 0
#define ZFLAC_E_INVALID_SIGNATURE 1         /* src/zflac.zig:220 */
#define ZFLAC_E_INVALID_METADATA_HEADER 2   /* src/zflac.zig:248 */
#define ZFLAC_E_MISSING_STREAMINFO 3        /* src/zflac.zig:309 */
#define ZFLAC_E_UNIMPLEMENTED 4             /* src/zflac.zig:263 */
#define ZFLAC_E_INVALID_CHECKSUM 5          /* src/zflac.zig:280 */
#define ZFLAC_E_INVALID_FRAME_HEADER 6      /* src/zflac.zig:352,357,361,372,405 */
#define ZFLAC_E_INCONSISTENT_PARAMETERS 7   /* src/zflac.zig:386,391 */
#define ZFLAC_E_INVALID_CODED_NUMBER 8      /* src/zflac.zig:206 */
#define ZFLAC_E_INVALID_SUBFRAME_HEADER 9   /* src/zflac.zig:431,471,542 */
#define ZFLAC_E_INVALID_RESIDUAL_CODING 10  /* src/zflac.zig:618 */
#define ZFLAC_E_END_OF_STREAM 11            /* std.io reader EndOfStream */
#define ZFLAC_E_OUT_OF_MEMORY 12            /* allocator OutOfMemory */
#define ZFLAC_E_DEVICE 13                   /* HIP runtime failure / no GPU (no zflac equivalent) */
#define ZFLAC_E_INVALID_ARGUMENT 14         /* bad handle, index or buffer size */
#define ZFLAC_E_OUT_OF_DOMAIN 15            /* input on which Debug zflac traps */
#define ZFLAC_E_FRAME_CRC 16                /* frame CRC-16 mismatch, only with ZFLAC_FLAG_CHECK_CRC16 */

/* Arm of zflac's `Samples` union (src/zflac.zig:12-16). */
#define ZFLAC_S8 0
#define ZFLAC_S16 1
#define ZFLAC_S32 2

/* Mirrors the scalar fields of zflac.DecodedFLAC (src/zflac.zig:18-23). */
typedef struct zflac_info {
    uint8_t channels;        /* DecodedFLAC.channels */
    uint8_t bits_per_sample; /* DecodedFLAC.bits_per_sample */
    uint8_t sample_kind;     /* ZFLAC_S8 / ZFLAC_S16 / ZFLAC_S32 */
    uint8_t reserved;
    uint32_t sample_rate;    /* DecodedFLAC.sample_rate (u24 in zflac) */
    uint64_t n_samples;      /* samples.len: interleaved channel-samples */
    uint64_t samples_bytes;  /* n_samples * sizeof(SampleType) */
} zflac_info;

/* One input stream: a complete FLAC byte stream in host memory. */
typedef struct zflac_stream {
    const uint8_t *data;
    size_t len;
} zflac_stream;

/* Per-kernel device time of the last zflac_hip_batch_run (HIP events on the
 * library's stream). */
typedef struct zflac_timings {
    double scan_ms;     /* frame-sync scan + candidate compaction */
    double decode_ms;   /* subframe decode kernel k_decode (the hot path) */
    double verify_ms;   /* chain verification */
    double total_ms;    /* first launch -> last event */
    uint64_t frames;        /* frames decoded */
    uint64_t input_bytes;   /* compressed frame bytes of decoded frames */
    uint64_t output_bytes;  /* PCM bytes written */
    uint64_t samples;       /* channel-samples written */
    double walk_ms;     /* subframe-start walk k_walk (2+ channels; runs before k_decode) */
    double md5_ms;      /* batched STREAMINFO MD5 k_md5 (ZFLAC_FLAG_DEVICE_MD5), else 0 */
    /* host wall-clock times (steady clock), recorded whether or not ZFLAC_FLAG_TIMING is set */
    double plan_ms;     /* batch_create / open: metadata and first-frame parse */
    double upload_ms;   /* batch_create / open: staging + H2D of the compressed bytes, allocations */
    double run_wall_ms; /* last batch_run, launch to results (kernels + read-backs) */
    double read_ms;     /* last batch_read / read: D2H of the samples (+ MD5 overlapped) */
    double host_md5_ms; /* last batch_read / read: host STREAMINFO MD5 (overlapped with the D2H) */
    double crc16_ms;    /* k_crc16 of the last run (ZFLAC_FLAG_CHECK_CRC16 with ZFLAC_FLAG_TIMING), else 0 */
    /* (ABI 4) synchronous `rest` decode launches of the last run: frame groups of a k_decode
     * history bucket the batch's launch plan had not predicted; the bucket is then added to
     * the plan, so a later run of the same batch has none */
    uint32_t rest_launches;
    /* (ABI 5) streams of the last run finished by the sequential chain planner (the chain
     * check did not certify them: false syncs, a broken frame, a wrong STREAMINFO, a total
     * unknown without a minimum frame size); 0 when the parallel pass certified every one */
    uint32_t sequential_streams;
} zflac_timings;

typedef struct zflac_batch zflac_batch;

/* ---- single stream: the decode(allocator, reader) replacement --------------- */
/* Decode `buf` on `device`. On success *out_batch holds the decoded stream and
 * *info its shape (allocate info->samples_bytes, 32-byte aligned as zflac does,
 * then call zflac_hip_read). The returned code is the zflac error of the stream
 * (MD5 is checked by zflac_hip_read). */
int zflac_hip_open(const uint8_t *buf, size_t len, int device, zflac_batch **out_batch, zflac_info *info);
/* zflac_hip_open with batch flags (ZFLAC_FLAG_CHECK_CRC16, ZFLAC_FLAG_TIMING). */
int zflac_hip_open_ex(const uint8_t *buf, size_t len, int device, int flags, zflac_batch **out_batch,
                      zflac_info *info);
/* Copy the samples into caller memory, verify the STREAMINFO MD5
 * (ZFLAC_E_INVALID_CHECKSUM on mismatch, as src/zflac.zig:279-280), left-justify is
 * already applied on the device (src/zflac.zig:287-306). Long streams are copied back in
 * chunks while a host thread hashes the chunks already landed (MD5 is one serial chain per
 * stream, so it bounds this call). */
int zflac_hip_read(zflac_batch *b, void *out_samples, size_t out_bytes);
void zflac_hip_close(zflac_batch *b);

/* ---- batches of independent streams (C5 shard) ------------------------------- */
/* Parse metadata on the host, upload all compressed bytes to HBM and allocate the
 * device output. Streams are referenced, not copied, until this call returns. */
int zflac_hip_batch_create(const zflac_stream *streams, size_t n, int device, int flags, zflac_batch **out);
/* One device-resident decode of every stream of the batch (inputs already in HBM,
 * outputs left in HBM). Synchronous. Returns ZFLAC_OK or ZFLAC_E_DEVICE; per-stream
 * zflac errors are reported by zflac_hip_batch_info. */
int zflac_hip_batch_run(zflac_batch *b);
/* zflac_hip_batch_run in two halves, so that runs of different batches overlap on the
 * device: _submit enqueues the run's kernels on the next of the device's run streams
 * (ZFLAC_RUN_STREAMS, default 3) and returns; with ZFLAC_FLAG_DEVICE_MD5 the run's hash
 * goes to the device's md5 hub (one launch over several runs, streams of its own);
 * _wait blocks until they finish and produces the per-stream results (the sequential
 * planner, CRC-16 and MD5 legs run here). A batch has at most one run in flight: _submit
 * on a submitted batch and _wait without one return ZFLAC_E_INVALID_ARGUMENT, and results
 * (_info, _read, ...) are unavailable between the two. Destroying a submitted batch waits
 * for its kernels. */
/* With ZFLAC_FLAG_DEVICE_MD5, _wait of a run whose hash is still queued in the md5 hub
 * flushes the hub: one launch hashes every pending run (up to ZFLAC_MD5_RUNS) and waits on
 * each of their decodes, so the digests of the waited run arrive with the slowest of those
 * runs, and md5_ms reports that shared launch's time. */
int zflac_hip_batch_submit(zflac_batch *b);
int zflac_hip_batch_wait(zflac_batch *b);
/* (ABI 4) Non-blocking: 1 when the device work of the submitted run has finished (so
 * _wait returns without waiting on the GPU), 0 while it runs, -ZFLAC_E_INVALID_ARGUMENT
 * without a submitted run, -ZFLAC_E_DEVICE on a device error. With ZFLAC_FLAG_DEVICE_MD5
 * the run's hash counts as device work (a pending md5 hub launch is flushed when the hub is
 * idle). A caller with several batches
 * in flight waits for whichever is ready instead of the oldest. */
int zflac_hip_batch_ready(zflac_batch *b);
/* Per-stream result of the last run: zflac error code, and shape when OK.
 * Before the first completed run: ZFLAC_E_INVALID_ARGUMENT (as for _read, _md5 and
 * _device_samples, which returns NULL). */
int zflac_hip_batch_info(zflac_batch *b, size_t i, zflac_info *info);
/* Copy stream i's samples to host memory; verify_md5 != 0 checks STREAMINFO MD5. */
int zflac_hip_batch_read(zflac_batch *b, size_t i, void *out, size_t out_bytes, int verify_md5);
/* Device MD5 digest of stream i's samples as zflac hashes them (before left-justify,
 * src/zflac.zig:267-277), computed by the last run when the batch was created with
 * ZFLAC_FLAG_DEVICE_MD5; ZFLAC_E_INVALID_ARGUMENT otherwise. */
int zflac_hip_batch_md5(zflac_batch *b, size_t i, uint8_t *digest16);
/* Device pointer of stream i's samples (valid until the next run / destroy). */
const void *zflac_hip_batch_device_samples(zflac_batch *b, size_t i);
/* Timings of the last run / read. ZFLAC_OK when device timings were recorded
 * (ZFLAC_FLAG_TIMING); the host wall-clock fields are filled either way.
 * _ex copies min(size, sizeof(zflac_timings)) bytes (pass sizeof *t) and zero-fills the
 * rest of a longer struct, so callers built against another version of this header stay
 * within their struct. The legacy entry point writes only the first-version layout
 * (ZFLAC_TIMINGS_V1_SIZE bytes: scan_ms .. md5_ms). */
int zflac_hip_batch_timings(zflac_batch *b, zflac_timings *t);
int zflac_hip_batch_timings_ex(zflac_batch *b, zflac_timings *t, size_t size);
#define ZFLAC_TIMINGS_V1_SIZE 80
size_t zflac_hip_batch_size(zflac_batch *b);
void zflac_hip_batch_destroy(zflac_batch *b);

/* Flags for zflac_hip_batch_create */
#define ZFLAC_FLAG_TIMING 1        /* record HIP events around each kernel */
#define ZFLAC_FLAG_FORCE_SLOW 2    /* skip the parallel fast path (testing the sequential path) */
/* Verify every stream's STREAMINFO MD5 on the device after each run (one lane per
 * stream: pays off for batches of many streams; a single long stream hashes faster on
 * the host, which zflac_hip_read / zflac_hip_batch_read do without this flag). A
 * mismatch makes the stream's result ZFLAC_E_INVALID_CHECKSUM (src/zflac.zig:279-280).
 * The hash of the streams a run certifies is enqueued by zflac_hip_batch_submit right
 * behind that run's kernels (so it overlaps other batches' runs in flight); streams the
 * sequential planner finishes are hashed by zflac_hip_batch_wait. */
#define ZFLAC_FLAG_DEVICE_MD5 4
/* Check every decoded frame's CRC-16 trailer on the device (k_crc16). zflac reads the
 * trailer and ignores it (src/zflac.zig:548-551), so this is off by default; with it, the
 * first frame in stream order whose trailer differs makes the stream ZFLAC_E_FRAME_CRC
 * (ahead of a later frame's error and of the MD5 check, which come after it in zflac's
 * read order). */
#define ZFLAC_FLAG_CHECK_CRC16 8
/* Subframe-start walk of 2+ channel streams: by default the library picks k_walk (a lane per
 * frame) for launches of many frames and k_walk_wave (a wave per frame, wave-wide bit scan)
 * otherwise. These force one (testing, timing); results are identical. */
#define ZFLAC_FLAG_WALK_LANE 16
#define ZFLAC_FLAG_WALK_WAVE 32

const char *zflac_hip_error_name(int code);
/* Number of HIP devices visible; 0 means every decode will fail with ZFLAC_E_DEVICE. */
int zflac_hip_device_count(void);
/* Library build tag, e.g. "zflac_hip gfx950 r3". */
const char *zflac_hip_version(void);
/* Identity of the compiled library: "src=<sha256 of its sources, headers, target, flags and
 * -D defines>" (zflac_amd/build.py source_fingerprint). hipcc output is not bit-reproducible,
 * so this, not a hash of the .so, says which kernels a measurement ran. */
const char *zflac_hip_build_id(void);
/* ABI revision of this header; bumped whenever a struct or a signature changes.
 * 3: zflac_hip_batch_timings_ex, zflac_hip_abi_version; device MD5 pipelined into submit.
 * 4: zflac_timings.rest_launches; zflac_hip_build_id; zflac_hip_batch_ready.
 * 5: zflac_timings.sequential_streams (was reserved0); total-unknown streams certified by the
 *    parallel pass. */
#define ZFLAC_HIP_ABI_VERSION 5
int zflac_hip_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif
