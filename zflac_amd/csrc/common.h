// common.h -- descriptors shared by the host planner (host.cpp) and the HIP kernels
// (kernels.hip). Plain structs, identical layout on both sides.
#pragma once
#include <cstdint>

namespace zflac {

enum Err : int {
    E_OK = 0,
    E_INVALID_SIGNATURE = 1,
    E_INVALID_METADATA_HEADER = 2,
    E_MISSING_STREAMINFO = 3,
    E_UNIMPLEMENTED = 4,
    E_INVALID_CHECKSUM = 5,
    E_INVALID_FRAME_HEADER = 6,
    E_INCONSISTENT_PARAMETERS = 7,
    E_INVALID_CODED_NUMBER = 8,
    E_INVALID_SUBFRAME_HEADER = 9,
    E_INVALID_RESIDUAL_CODING = 10,
    E_END_OF_STREAM = 11,
    E_OUT_OF_MEMORY = 12,
    E_DEVICE = 13,
    E_INVALID_ARGUMENT = 14,
    E_OUT_OF_DOMAIN = 15,
    E_FRAME_CRC = 16,  // frame CRC-16 mismatch: only with ZFLAC_FLAG_CHECK_CRC16 (zflac never checks it)
};

// One stream of a batch, as the kernels see it. Byte offsets are absolute in the
// batch's input buffer; sample offsets are absolute element indices in the batch's
// output buffer (one SampleType per element).
struct StreamDesc {
    uint64_t in_begin;     // first frame header (right after the metadata blocks)
    uint64_t in_end;       // end of the stream bytes
    uint64_t out_base;     // first output element of this stream
    uint64_t out_cap;      // output elements reserved for this stream
    uint64_t total;        // STREAMINFO total samples * channels (0 when unknown)
    uint32_t rate_hz;      // sample rate of the first frame (consistency filter)
    uint32_t si_rate;      // STREAMINFO sample rate (frame rate code 0)
    uint32_t first_chunk;  // chunk range of this stream in the sync-scan chunk table
    uint32_t end_chunk;    // one past the last chunk
    uint8_t byte1;         // 0xF8 / 0xF9 of the first frame (blocking strategy)
    uint8_t nch;           // channel count of the first frame (== STREAMINFO)
    uint8_t dcode;         // bit-depth code of the first frame
    uint8_t si_bps;        // STREAMINFO bits per sample
    uint8_t valid_total;   // STREAMINFO total samples > 0
    uint8_t justify;       // left-justify shift applied at pack-out (src/zflac.zig:287-306)
    uint8_t pad_[2];
};

struct ChunkDesc {
    uint64_t begin;   // absolute byte range scanned for frame-sync candidates
    uint64_t end;
    uint32_t stream;
    uint32_t pad_;
};

// c_info packing for a decoded candidate frame
//   bits  0..15  block size - 1
//   bits 16..19  channel assignment code
//   bits 20..22  bit-depth code
//   bit  28      the frame error arose in the header before the consistency checks
//   bit  29      the header's CRC-8 byte is missing (EndOfStream after the checks)
constexpr uint32_t INFO_PRE_ERR = 1u << 28;
constexpr uint32_t INFO_CRC_EOF = 1u << 29;

constexpr int SCAN_THREADS = 256;
#ifndef ZFLAC_SCAN_BPT
#define ZFLAC_SCAN_BPT 128
#endif
constexpr int SCAN_BYTES_PER_THREAD = ZFLAC_SCAN_BPT;
constexpr uint64_t CHUNK_BYTES = (uint64_t)SCAN_THREADS * SCAN_BYTES_PER_THREAD;  // 32 KiB by default
constexpr int CHUNK_CAP = 64;           // candidates kept per chunk by the scan pass
constexpr uint64_t INPUT_PAD = 4096;    // zero bytes after the last stream
constexpr int MAX_CH = 8;               // FLAC channel limit; k_walk's per-frame record stride
// Launches walking fewer (frames x leading subframes) than this use k_walk_wave (a wave per
// frame) instead of k_walk (a lane per frame): below it k_walk leaves most SIMDs idle.
#ifndef ZFLAC_WAVE_WALK_MAX_FRAMES
#define ZFLAC_WAVE_WALK_MAX_FRAMES 16384
#endif
constexpr uint64_t WAVE_WALK_MAX_FRAMES = ZFLAC_WAVE_WALK_MAX_FRAMES;
constexpr uint64_t DUMMY_BYTES = 64 * 64 * 32;  // 64 wave slots x 64 lanes x 2 quads
constexpr uint64_t PROBE_BYTES = 256;           // after the dummy region: timing-probe builds only

struct ScanArgs {
    const uint8_t* in;
    const StreamDesc* streams;
    const ChunkDesc* chunks;
    uint32_t n_chunks;
    uint32_t* chunk_cnt;        // candidates per chunk (exact)
    unsigned long long* chunk_units;  // sum of block_size*channels per chunk
    uint64_t* chunk_slots;      // CHUNK_CAP positions per chunk
    uint32_t* chunk_slot_units; // CHUNK_CAP units per chunk
    // the run's per-stream status words and its 4 counters, zeroed by k_scan (instead of two
    // fill launches per run); k_verify and later kernels of the run accumulate into them
    uint32_t* status;
    uint32_t n_status;
    uint32_t* misc;
};

struct CompactArgs {
    const uint8_t* in;
    const StreamDesc* streams;
    const ChunkDesc* chunks;
    uint32_t n_chunks;
    const uint32_t* chunk_cnt;
    const uint64_t* chunk_slots;
    const uint32_t* chunk_slot_units;
    const uint32_t* chunk_off;             // exclusive scan of chunk_cnt (n_chunks + 1)
    const unsigned long long* chunk_uoff;  // exclusive scan of chunk_units (n_chunks + 1)
    uint32_t cap;                          // candidate table capacity
    uint64_t* c_pos;
    uint32_t* c_stream;
    uint64_t* c_out;
    uint32_t* overflow;                    // set when the table is too small
};

struct DecodeArgs {
    const uint8_t* in;
    uint64_t in_size;          // bytes of `in`, INPUT_PAD included
    void* out;
    const StreamDesc* streams;
    const uint64_t* c_pos;
    const uint32_t* c_stream;
    const uint64_t* c_out;
    const uint32_t* n_frames;  // device count (fast path) ...
    uint32_t n_frames_host;    // ... or host count when n_frames == nullptr
    uint32_t cap;
    uint64_t* c_end;
    int32_t* c_err;
    uint32_t* c_info;
    uint32_t* c_rate;
    int nch;
    int write;
    void* dummy;  // DUMMY_BYTES: target of masked-off / pending-less packed stores
    uint32_t* sub_start;  // [frame][MAX_CH]: bit offset of subframe c >= 1 (k_walk -> k_decode)
    uint32_t* group_mb;   // [frame group of a k_decode wave]: its history bucket, written by the
                          // first bucket launch so the later launches skip other groups cheaply
    uint32_t* bucket_used;  // optional: the first bucket launch ORs in bucket_bit() of every group
    uint32_t full_mask;     // host only: bucket_bit()s that get their own launch, with a grid
                            // covering every frame group (the order-8 launch, which classifies
                            // every group, and the buckets the host predicts from the input
                            // bytes); 0 = every bucket
    uint32_t rest;          // set on the `rest` launch (of the most general kernel, order 32 with
                            // constant / verbatim lanes) that decodes the frame groups of every
                            // bucket outside full_mask
    uint32_t rest_only;     // host only: launch nothing but the rest kernel (no walk, no bucket
                            // kernels). The normal launch never includes it: the host issues it
                            // after a run whose order-8 launch reported a bucket outside
                            // full_mask (bucket_used), so a correct prediction costs no launch
};

// Grid (workgroups) of the `rest` launch: a few waves striding over the frame groups (the
// groups of unpredicted buckets; a misprediction costs time, never correctness).
constexpr uint32_t SPARSE_DECODE_BLOCKS = 256;

// Bit of a k_decode launch (history bucket MB, MIX kernels) in DecodeArgs::bucket_used /
// full_mask: 8 -> 1, 4 -> 2, 16 -> 4, 32 -> 8, MIX 8 -> 16, MIX 32 -> 32, 12 -> 64. The order-8 launch
// always runs (it classifies every wave).
__host__ __device__ inline constexpr uint32_t bucket_bit(uint32_t mb, bool mix) {
    return mix ? (mb <= 8 ? 16u : 32u)
               : (mb == 8 ? 1u : (mb == 4 ? 2u : (mb == 16 ? 4u : (mb == 12 ? 64u : 8u))));
}
constexpr uint32_t BUCKET_MASK_ALL = 127u;

// One stream for k_md5 (md5.hip): the message is the decoded samples before left-justify,
// rebuilt from the justified device samples (src/zflac.zig:267-280).
enum Md5Mode : uint32_t {
    MD5_RAW = 0,        // bytes as stored (8-bit, 16-bit, 32-bit containers with no justify)
    MD5_S16_SHIFT = 1,  // i16 samples >> js (9..15-bit)
    MD5_S32_SHIFT = 2,  // i32 samples >> js, 4 bytes each (25..31-bit)
    MD5_S24 = 3,        // i32 samples >> js, 3 low bytes each (17..24-bit)
};

struct Md5Job {
    const uint8_t* data;     // device samples of the stream
    uint64_t n;              // samples
    uint32_t mode;           // Md5Mode
    uint32_t js;             // justify shift to undo
    uint32_t width;          // message bytes per sample (1, 2, 3 or 4)
    uint32_t pad_;
    const uint32_t* status;  // optional: the stream's k_verify status; nonzero = not certified by
                             // this run (the sequential planner decodes it later), no hash
};

// Jobs of several runs for one k_md5_multi launch (the md5 hub, host.cpp): segment s is
// jobs[s][0 .. start[s+1] - start[s]), its digests go to dig[s].
constexpr int MD5_MAX_SEGS = 16;
struct Md5Segs {
    const Md5Job* jobs[MD5_MAX_SEGS];
    uint32_t* dig[MD5_MAX_SEGS];
    uint32_t start[MD5_MAX_SEGS + 1];
    uint32_t nseg;
};

struct VerifyArgs {
    const StreamDesc* streams;
    uint32_t n_streams;
    const uint32_t* chunk_off;  // per-chunk candidate offsets (n_chunks + 1)
    const uint64_t* c_pos;
    const uint32_t* c_stream;
    const uint64_t* c_out;
    const uint32_t* n_frames;
    uint32_t cap;
    const uint64_t* c_end;
    const int32_t* c_err;
    const uint32_t* c_info;
    const uint32_t* c_rate;
    uint32_t* status;           // per stream: nonzero => take the sequential path
    uint64_t* units;            // per stream, STREAMINFO total unknown: the chain's output elements
                                // (written by its last frame; nullptr when every total is known)
};

// k_sync_list (scan.hip): sync codes in [lo, hi) with a parseable header matching the
// stream's first frame (channels, depth code, rate), for the sequential planner.
struct SyncListArgs {
    const uint8_t* in;
    uint64_t lo, hi;       // absolute byte range to search
    uint64_t in_end;       // end of the stream's bytes
    uint32_t si_rate;      // STREAMINFO rate (rate code 0)
    uint32_t rate_hz;      // the first frame's rate
    uint32_t nch, dcode;   // the first frame's channel count and depth code
    uint64_t* pos;         // out: positions (unordered)
    uint32_t* count;       // out: number found (may exceed cap)
    uint32_t cap;
};

// k_crc16 (crc16.hip): frame f covers bytes [pos[f], end[f] - 2) with its CRC-16 trailer at
// end[f] - 2 (c_end as k_decode records it). Frames with err[f] != 0 are skipped.
struct Crc16Args {
    const uint8_t* in;
    uint64_t in_size;
    const uint64_t* pos;
    const uint64_t* end;
    const int32_t* err;        // optional
    // optional (the parallel pass): candidates at or past their stream's STREAMINFO total are
    // not checked (zflac stops reading there, src/zflac.zig:341)
    const StreamDesc* streams;
    const uint32_t* c_stream;
    const uint64_t* c_out;
    const uint32_t* n_frames;  // device count ...
    uint32_t n_frames_host;    // ... or host count when n_frames == nullptr
    uint32_t cap;
    uint32_t* bad;             // per frame: 1 when the stored CRC-16 differs
};

}  // namespace zflac
