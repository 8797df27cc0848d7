// host.cpp -- host side of libzflac_hip.so: metadata parsing, batch planning, device
// buffers and launches, the sequential chain planner for streams the parallel fast path
// cannot certify, MD5 verification, and the extern "C" ABI of include/zflac_hip.h.
//
// Reference: Senryoku/zflac src/zflac.zig (decode :217-310, decode_frames :312-602).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <thread>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <new>
#include <unordered_map>
#include <vector>

#include "../../include/zflac_hip.h"
#include "common.h"
#include "md5.hpp"

namespace zflac {

hipError_t launch_scan(const ScanArgs& a, hipStream_t st);
hipError_t launch_scan_chunks(const uint32_t* cnt, const unsigned long long* units, uint32_t n, uint32_t* off,
                              unsigned long long* uoff, uint32_t* n_frames, hipStream_t st);
hipError_t launch_compact(const CompactArgs& a, hipStream_t st);
#define ZFLAC_DECL_LAUNCH(K)                                                                  \
    hipError_t launch_decode_k##K##_stereo(const DecodeArgs& a, uint32_t max_frames, hipStream_t st); \
    hipError_t launch_decode_k##K##_mono(const DecodeArgs& a, uint32_t max_frames, hipStream_t st);   \
    hipError_t launch_decode_k##K##_multi(const DecodeArgs& a, uint32_t max_frames, hipStream_t st);   \
    hipError_t launch_walk_k##K(const DecodeArgs& a, uint32_t max_frames, hipStream_t st);
ZFLAC_DECL_LAUNCH(0)
ZFLAC_DECL_LAUNCH(1)
ZFLAC_DECL_LAUNCH(2)
#undef ZFLAC_DECL_LAUNCH
hipError_t launch_walk_wave(int kind, const DecodeArgs& a, uint32_t max_frames, hipStream_t st);

// Which subframe-start walk a launch over `frames` frames of `nch` channels uses: k_walk
// (lane per frame: 64 serial chains per wave, nch - 1 subframes each) needs tens of thousands
// of subframe walks to fill the chip; k_walk_wave (wave per frame, wave-wide bit scan of each
// Rice partition) fills it with a few thousand, at several times the instructions per code.
// So the wave walk below WAVE_WALK_MAX_FRAMES subframe walks, the lane walk above, for every
// channel count (a 32,768-frame 6-channel stream: lane walk).
// ZFLAC_WALK=lane / wave forces one (timing experiments).
static bool use_wave_walk(uint64_t frames, int nch, int flags) {
    static const int forced = [] {
        const char* e = std::getenv("ZFLAC_WALK");
        return !e ? 0 : (e[0] == 'w' ? 1 : (e[0] == 'l' ? 2 : 0));
    }();
    if (flags & ZFLAC_FLAG_WALK_WAVE) return true;
    if (flags & ZFLAC_FLAG_WALK_LANE) return false;
    if (forced) return forced == 1;
    return frames * (uint64_t)(nch - 1) < WAVE_WALK_MAX_FRAMES;
}

// k_walk or k_walk_wave (subframe start offsets, 2+ channels) then k_decode; `mid`
// (optional) is recorded between the two launches. With a `front` stream the walk runs
// there and k_decode waits for it on `st` through the event `join`. `est_frames`: the
// frame count the walk choice is made for (the launch grid is sized for `max_frames`).
static hipError_t launch_decode(int kind, const DecodeArgs& a, uint32_t max_frames, hipStream_t st,
                                hipEvent_t mid = nullptr, hipStream_t front = nullptr, hipEvent_t join = nullptr,
                                uint64_t est_frames = 0, int flags = 0) {
    const int lay = a.nch == 2 ? 2 : (a.nch == 1 ? 1 : 0);
    hipStream_t ws = front ? front : st;
    if (a.nch > 1 && !a.rest_only) {
        hipError_t e;
        if (use_wave_walk(est_frames ? est_frames : max_frames, a.nch, flags)) e = launch_walk_wave(kind, a, max_frames, ws);
        else e = kind == 0 ? launch_walk_k0(a, max_frames, ws)
                           : (kind == 1 ? launch_walk_k1(a, max_frames, ws) : launch_walk_k2(a, max_frames, ws));
        if (e != hipSuccess) return e;
    }
    if (mid) {
        const hipError_t e = hipEventRecord(mid, ws);
        if (e != hipSuccess) return e;
    }
    if (front) {
        hipError_t e = hipEventRecord(join, front);
        if (e == hipSuccess) e = hipStreamWaitEvent(st, join, 0);
        if (e != hipSuccess) return e;
    }
    if (kind == 0) {
        if (lay == 2) return launch_decode_k0_stereo(a, max_frames, st);
        if (lay == 1) return launch_decode_k0_mono(a, max_frames, st);
        return launch_decode_k0_multi(a, max_frames, st);
    }
    if (kind == 1) {
        if (lay == 2) return launch_decode_k1_stereo(a, max_frames, st);
        if (lay == 1) return launch_decode_k1_mono(a, max_frames, st);
        return launch_decode_k1_multi(a, max_frames, st);
    }
    if (lay == 2) return launch_decode_k2_stereo(a, max_frames, st);
    if (lay == 1) return launch_decode_k2_mono(a, max_frames, st);
    return launch_decode_k2_multi(a, max_frames, st);
}
hipError_t launch_verify(const VerifyArgs& a, uint32_t max_items, hipStream_t st);
hipError_t launch_crc16(const Crc16Args& a, uint32_t max_frames, hipStream_t st);
hipError_t launch_sync_list(const SyncListArgs& a, hipStream_t st);
// coop_mode: the Md5Mode every job shares with 16-byte aligned samples (the cooperative-load
// kernel), or -1 (lane-per-stream loads)
hipError_t launch_md5(const Md5Job* jobs, uint32_t n_jobs, uint32_t* digests, hipStream_t st, int coop_mode);
hipError_t launch_md5_multi(const Md5Segs& sg, hipStream_t st, int coop_mode);

namespace {

double now_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

struct DeviceError {};
inline void ck(hipError_t e) {
    if (e != hipSuccess) throw DeviceError{};
}

// ---------------------------------------------------------------------------------
// Host-side parsing with zflac semantics
// ---------------------------------------------------------------------------------
struct ByteReader {
    const uint8_t* d;
    size_t n;
    size_t pos = 0;
    bool get(size_t k, uint64_t& v) {  // readInt(uK*8, .big)
        if (n - pos < k) return false;
        v = 0;
        for (size_t i = 0; i < k; i++) v = (v << 8) | d[pos + i];
        pos += k;
        return true;
    }
};

struct StreamInfoH {
    uint16_t min_block = 0, max_block = 0;
    uint32_t sample_rate = 0;
    uint32_t channels = 0;  // count
    uint32_t bps = 0;       // bits
    uint64_t total = 0;     // per channel
    uint8_t md5[16] = {};
};

// decode() up to the first frame (src/zflac.zig:217-253)
int parse_metadata(const uint8_t* d, size_t n, StreamInfoH& si, size_t& frames_begin) {
    ByteReader r{d, n};
    uint64_t v;
    if (!r.get(4, v)) return E_END_OF_STREAM;
    if (v != 0x664C6143) return E_INVALID_SIGNATURE;  // :218-220
    bool have = false;
    for (;;) {
        uint64_t h;
        if (!r.get(4, h)) return E_END_OF_STREAM;
        const unsigned info = (unsigned)(h >> 24) & 0x7F;
        const bool last = (h >> 31) & 1;
        const uint64_t length = h & 0xFFFFFF;
        if (info == 0) {  // STREAMINFO, always 34 bytes (:228-240)
            if (r.n - r.pos < 34) return E_END_OF_STREAM;
            const uint8_t* p = d + r.pos;
            si.min_block = (uint16_t)((p[0] << 8) | p[1]);
            si.max_block = (uint16_t)((p[2] << 8) | p[3]);
            si.sample_rate = ((uint32_t)p[10] << 12) | ((uint32_t)p[11] << 4) | (p[12] >> 4);
            si.channels = ((p[12] >> 1) & 7) + 1;
            si.bps = (((p[12] & 1) << 4) | (p[13] >> 4)) + 1;
            si.total = ((uint64_t)(p[13] & 15) << 32) | ((uint64_t)p[14] << 24) | ((uint64_t)p[15] << 16) |
                       ((uint64_t)p[16] << 8) | p[17];
            std::memcpy(si.md5, p + 18, 16);
            r.pos += 34;
            have = true;
        } else if (info >= 1 && info <= 6) {  // skipped (:243-247)
            if (r.n - r.pos < length) return E_END_OF_STREAM;
            r.pos += length;
        } else {
            return E_INVALID_METADATA_HEADER;  // :248
        }
        if (last) break;
    }
    if (!have) return E_MISSING_STREAMINFO;  // :309
    frames_begin = r.pos;
    return E_OK;
}

int channels_count_h(uint32_t code) { return code <= 7 ? (int)code + 1 : (code <= 10 ? 2 : 0); }
int depth_bits_h(uint32_t dcode, int si_bps) {
    static const int B[8] = {0, 8, 12, -1, 16, 20, 24, 32};
    return dcode == 0 ? si_bps : B[dcode];
}

struct FrameHdrH {
    uint32_t bs = 0, rate = 0, chan_code = 0, dcode = 0, byte1 = 0;
    uint32_t hdr_len = 0;  // header bytes, CRC-8 included (when err == 0 and !crc_eof)
    int err = 0;       // before the consistency checks
    bool crc_eof = false;
};

// Frame header (src/zflac.zig:343-375, 203-214, 407), host copy of the device parser.
FrameHdrH parse_frame_header_h(const uint8_t* p, uint64_t avail, uint32_t si_rate) {
    FrameHdrH h;
    if (avail < 4) { h.err = E_END_OF_STREAM; return h; }
    const uint32_t b0 = p[0], b1 = p[1], b2 = p[2], b3 = p[3];
    h.byte1 = b1;
    h.chan_code = b3 >> 4;
    h.dcode = (b3 >> 1) & 7;
    if (((b0 << 7) | (b1 >> 1)) != 0x7FFC) { h.err = E_INVALID_FRAME_HEADER; return h; }
    uint64_t idx = 4;
    if (avail <= idx) { h.err = E_END_OF_STREAM; return h; }
    const uint32_t first = p[idx++];
    uint32_t ones = 0;
    while (ones < 8 && (first & (0x80u >> ones))) ones++;
    if (first == 0xFF || ones == 1) { h.err = E_INVALID_CODED_NUMBER; return h; }
    if (ones >= 2) {
        if (avail < idx + (ones - 1)) { h.err = E_END_OF_STREAM; return h; }
        idx += ones - 1;
    }
    const uint32_t bc = b2 >> 4;
    if (bc == 0) { h.err = E_INVALID_FRAME_HEADER; return h; }
    if (bc == 6) {
        if (avail <= idx) { h.err = E_END_OF_STREAM; return h; }
        h.bs = (uint32_t)p[idx++] + 1;
    } else if (bc == 7) {
        if (avail < idx + 2) { h.err = E_END_OF_STREAM; return h; }
        const uint32_t v = ((uint32_t)p[idx] << 8) | p[idx + 1];
        idx += 2;
        if (v == 0xFFFF) { h.err = E_INVALID_FRAME_HEADER; return h; }
        h.bs = v + 1;
    } else if (bc == 1) {
        h.bs = 192;
    } else if (bc <= 5) {
        h.bs = 144u << bc;
    } else {
        h.bs = 1u << bc;
    }
    static const uint32_t T[12] = {0, 88200, 176400, 192000, 8000, 16000, 22050, 24000, 32000, 44100, 48000, 96000};
    const uint32_t rc = b2 & 15;
    if (rc == 0) {
        h.rate = si_rate;
    } else if (rc == 12) {
        if (avail <= idx) { h.err = E_END_OF_STREAM; return h; }
        h.rate = p[idx++];
    } else if (rc == 13 || rc == 14) {
        if (avail < idx + 2) { h.err = E_END_OF_STREAM; return h; }
        h.rate = ((uint32_t)p[idx] << 8) | p[idx + 1];
        if (rc == 14) h.rate *= 10;
        idx += 2;
    } else if (rc == 15) {
        h.err = E_INVALID_FRAME_HEADER;
        return h;
    } else {
        h.rate = T[rc];
    }
    if (avail <= idx) h.crc_eof = true;
    h.hdr_len = (uint32_t)idx + 1;
    return h;
}

// ---------------------------------------------------------------------------------
// Device memory helpers
// ---------------------------------------------------------------------------------
template <typename T>
struct DevBuf {
    T* p = nullptr;
    size_t n = 0;
    DevBuf() = default;
    DevBuf(const DevBuf&) = delete;
    DevBuf& operator=(const DevBuf&) = delete;
    ~DevBuf() { release(); }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
    }
    void alloc(size_t count) {
        if (count <= n && p) return;
        release();
        ck(hipMalloc(reinterpret_cast<void**>(&p), std::max<size_t>(count, 1) * sizeof(T)));
        n = count;
    }
};

struct StreamState {
    // host parse
    int host_err = 0;  // error known without the GPU (metadata / first frame header)
    StreamInfoH si;
    size_t len = 0;
    size_t frames_begin = 0;
    int kind = 1;
    int nch = 0;
    FrameHdrH first;
    bool no_frames = false;  // empty frame section, total unknown: zero samples, no error
    int cls = -1;
    uint32_t slot = 0;  // index inside its class
    // result
    int err = 0;
    zflac_info info = {};
    const void* dev_samples = nullptr;  // device pointer of the decoded samples
    int md5_dev = 0;                    // 0 not hashed on the device, 1 match, 2 mismatch
    uint8_t md5_dig[16] = {};           // device digest (md5_dev != 0)
    std::unique_ptr<DevBuf<uint8_t>> override_out;
};

struct Class {
    int kind = 1;
    int nch = 2;
    std::vector<uint32_t> members;  // stream indices
    std::vector<StreamDesc> desc;
    std::vector<ChunkDesc> chunks;
    uint64_t in_bytes = 0, out_elems = 0;
    uint32_t cap = 0;
    uint64_t est_frames = 0;  // frames expected from the STREAMINFO totals (walk choice)
    // frames the walk / decode grids are sized for (their loops stride over any excess): the
    // exact frame count of fixed-blocking streams with a STREAMINFO total, plus slack; raised
    // when a run finds more candidates (false syncs) than that
    uint32_t grid_frames = 0;
    // decode launches given a full grid (DecodeArgs::full_mask): the buckets predicted from
    // the first subframe of each member's first frame, at batch creation (plan_buckets)
    uint32_t full_mask = 0;
    bool redone = false;  // the last run re-ran the class (candidate table regrown)
    DevBuf<uint8_t> in;
    DevBuf<uint8_t> out;
    DevBuf<StreamDesc> d_desc;
    DevBuf<ChunkDesc> d_chunks;
    DevBuf<uint32_t> chunk_cnt, chunk_off, chunk_slot_units, misc;  // misc: 4 counters, then `status`
    uint32_t* status = nullptr;  // per-member status words, misc.p + 4 (one read-back for both)
    DevBuf<unsigned long long> chunk_units, chunk_uoff;
    DevBuf<uint64_t> chunk_slots;
    DevBuf<uint64_t> c_pos, c_out, c_end;
    DevBuf<uint32_t> c_stream, c_info, c_rate, sub, group_mb;
    DevBuf<int32_t> c_err;
    DevBuf<uint32_t> crc_bad;  // k_crc16 verdict per candidate (ZFLAC_FLAG_CHECK_CRC16)
    DevBuf<uint8_t> dummy;  // sink of masked-off packed stores (64 lanes x 32 B)
    // pinned host mirror, so the per-run read-backs are plain DMA on the batch stream:
    // [0] n_frames, [1] overflow, [2] decode buckets used, [3] unused, then one status word per member
    struct Pinned {
        uint32_t* p = nullptr;
        ~Pinned() {
            if (p) (void)hipHostFree(p);
        }
    } pin;
    uint32_t* h_misc = nullptr;
    uint32_t* h_status = nullptr;
    // members whose STREAMINFO total is unknown but whose output is reserved (unknown_total_cap):
    // k_verify certifies their chain to the end of the stream and writes its length here
    bool any_unknown = false;
    DevBuf<uint64_t> units;
    uint64_t* h_units = nullptr;  // pinned mirror, after the status words
};

}  // namespace

// ---------------------------------------------------------------------------------
// Batch
// ---------------------------------------------------------------------------------
void hub_release_ext(zflac_batch* b);  // flush a run still pending in its device's md5 hub
void hub_forget_ext(zflac_batch* b);   // drop a run from its device's md5 hub without hashing it
}  // namespace zflac

struct zflac_batch {
    int device = 0;
    int flags = 0;
    hipStream_t stream = nullptr;
    // ZFLAC_FRONT_PRIORITY=1: a second, highest-priority stream for the scan / compact / walk
    // of each run, so that with several runs in flight their workgroups are dispatched ahead
    // of another run's decode workgroups (an experiment knob; nullptr = one stream)
    hipStream_t front = nullptr;
    hipEvent_t front_join = nullptr;
    std::vector<zflac::StreamState> streams;
    std::vector<std::unique_ptr<zflac::Class>> classes;
    hipEvent_t ev[10] = {};
    hipEvent_t ev_done = nullptr;  // recorded behind the last work _submit enqueued (_ready)
    // the HIP stream of the run in flight: one of the device's run streams (DeviceStreams),
    // so that many batches in flight share a few hardware queues; `stream` (the batch's own)
    // carries the synchronous work (upload, regrowth, the sequential planner, read-backs)
    hipStream_t rs = nullptr;
    // ZFLAC_FLAG_DEVICE_MD5 runs hash in the device's md5 hub (one k_md5_coop launch over
    // the runs of several batches, on the hub's stream): ev_done then marks the decode only,
    // ev_md5 the hash and its digest read-back; md5_pending until the hub launched it
    hipEvent_t ev_md5 = nullptr;
    // written under the hub's lock, read without it by _ready / hub_release (other threads
    // flush the hub from their own batches' submit / wait / ready)
    std::atomic<bool> md5_pending{false};
    bool md5_failed = false;  // the hub launch that held this run threw: its digests are void
    bool md5_hub = false;  // this run's hash goes through the hub
    bool have_timing = false;
    bool ran = false;        // results exist only after a completed batch_run / batch_wait
    bool submitted = false;  // batch_submit enqueued a run that batch_wait has not finished
    double submit_t0 = 0;    // host clock at submit (run_wall_ms)
    zflac::DevBuf<zflac::Md5Job> md5_jobs;
    zflac::DevBuf<uint32_t> md5_dig;
    // ZFLAC_FLAG_DEVICE_MD5: k_md5 over every certifiable stream, enqueued by submit behind
    // the run's k_verify (pipe_who[k] = stream of job k, longest first); its digests land in
    // pinned memory with the run's other read-backs
    zflac::DevBuf<zflac::Md5Job> pipe_jobs;
    int pipe_coop = -1;  // coop_mode_of(the pipe jobs)
    zflac::DevBuf<uint32_t> pipe_dig;
    std::vector<uint32_t> pipe_who;
    uint32_t* pipe_pin = nullptr;
    zflac_timings timings = {};
    ~zflac_batch() {
        if (stream) (void)hipStreamSynchronize(stream);  // a submitted run may still use the buffers
        if (ev_done) (void)hipEventSynchronize(ev_done);  // ... on its run stream
        if (md5_pending) {  // still in the md5 hub: flush it, then let the hash finish
            try {
                zflac::hub_release_ext(this);
            } catch (...) {
            }
            try {
                zflac::hub_forget_ext(this);  // never leave a pointer to this batch in the hub
            } catch (...) {
            }
        }
        if (md5_hub && ev_md5) (void)hipEventSynchronize(ev_md5);
        if (front) (void)hipStreamSynchronize(front);
        classes.clear();
        for (auto& s : streams) s.override_out.reset();
        for (auto& e : ev)
            if (e) (void)hipEventDestroy(e);
        if (ev_done) (void)hipEventDestroy(ev_done);
        if (ev_md5) (void)hipEventDestroy(ev_md5);
        if (pipe_pin) (void)hipHostFree(pipe_pin);
        if (stream) (void)hipStreamDestroy(stream);
        if (front) (void)hipStreamDestroy(front);
        if (front_join) (void)hipEventDestroy(front_join);
    }
};

namespace zflac {
namespace {

int kind_of_bps(uint32_t bps) {
    const uint32_t aligned = (bps + 7) / 8 * 8;  // src/zflac.zig:256-264
    if (aligned == 8) return 0;
    if (aligned == 16) return 1;
    return 2;
}
int esz_of_kind(int kind) { return kind == 0 ? 1 : (kind == 1 ? 2 : 4); }
uint8_t justify_of(uint32_t bps) {  // src/zflac.zig:287-306
    if (bps >= 9 && bps <= 15) return (uint8_t)(16 - bps);
    if (bps >= 17 && bps <= 31) return (uint8_t)(32 - bps);
    return 0;
}

// Host planning of one stream: metadata and the first frame header.
void plan_stream(StreamState& s, const uint8_t* d, size_t n) {
    s.len = n;
    s.host_err = parse_metadata(d, n, s.si, s.frames_begin);
    if (s.host_err) return;
    s.kind = kind_of_bps(s.si.bps);
    s.nch = (int)s.si.channels;
    const bool valid_total = s.si.total > 0;
    const uint64_t avail = n - s.frames_begin;
    if (avail < 4) {  // readInt(u32) of the first frame header fails (:343-350)
        if (valid_total) s.host_err = E_END_OF_STREAM;
        else s.no_frames = true;
        return;
    }
    s.first = parse_frame_header_h(d + s.frames_begin, avail, s.si.sample_rate);
    if (s.first.err) { s.host_err = s.first.err; return; }
    if (depth_bits_h(s.first.dcode, (int)s.si.bps) < 0) { s.host_err = E_OUT_OF_DOMAIN; return; }  // :143
    if (channels_count_h(s.first.chan_code) != s.nch) { s.host_err = E_INCONSISTENT_PARAMETERS; return; }  // :386
}

// Copy streams into their HBM layout (stream m at in_off[m], zeros elsewhere, `total`
// bytes) through two pinned 32 MiB windows: host threads fill one window while the DMA
// engine drains the other. The windows are a lazily created per-process context, shared
// by all batches under a lock.
struct Uploader {
    static constexpr uint64_t WIN = 32ull << 20;
    std::mutex mu;
    uint8_t* pin[2] = {nullptr, nullptr};
    hipEvent_t done[2] = {nullptr, nullptr};
    bool used[2] = {false, false};
};

// One per device: the windows' events are recorded on the streams of that device's batches.
Uploader& uploader(int device) {
    static std::mutex mu;
    static std::unordered_map<int, Uploader*> per_device;  // never destroyed: outlives every batch
    std::lock_guard<std::mutex> lock(mu);
    Uploader*& u = per_device[device];
    if (!u) u = new Uploader();
    return *u;
}

// The device's run streams: every batch run (zflac_hip_batch_submit) goes to the next one
// in turn, so any number of batches in flight use n_run (3 by default) hardware queues (runs
// on one stream execute in submit order). bench.py keeps four runs in flight and sets
// ZFLAC_RUN_STREAMS from its --inflight (four: 1-3 % faster than three since round 4).
// Created before any batch's own stream, so that with enough hardware queues
// (GPU_MAX_HW_QUEUES) the run streams and the md5 hub stream each hold one of their own.
// ZFLAC_RUN_STREAMS / ZFLAC_HUB_STREAMS override the counts (at most 8 / 4).
constexpr int MAX_RUN_STREAMS = 8;
struct Md5Hub;
struct DeviceStreams {
    std::mutex mu;
    hipStream_t run[MAX_RUN_STREAMS] = {};
    uint32_t n_run = 3, next = 0;
    std::unique_ptr<Md5Hub> hub_p;
    Md5Hub& hub;
    DeviceStreams();
};

DeviceStreams& device_streams(int device);

// bytes [a, b) of the layout into dst
void fill_window(uint8_t* dst, uint64_t a, uint64_t b, const std::vector<uint64_t>& in_off,
                 const std::vector<const uint8_t*>& srcs, const std::vector<uint64_t>& lens) {
    size_t m = std::upper_bound(in_off.begin(), in_off.end(), a) - in_off.begin();
    m = m ? m - 1 : 0;
    uint64_t p = a;
    for (; p < b && m < in_off.size(); m++) {
        const uint64_t s0 = in_off[m], s1 = in_off[m] + lens[m];
        if (s1 <= p) continue;
        if (s0 >= b) break;
        if (s0 > p) {
            std::memset(dst + (p - a), 0, s0 - p);
            p = s0;
        }
        const uint64_t e = std::min(s1, b);
        std::memcpy(dst + (p - a), srcs[m] + (p - s0), e - p);
        p = e;
    }
    if (p < b) std::memset(dst + (p - a), 0, b - p);
}

void upload_streams(int device, uint8_t* dev, uint64_t total, const std::vector<uint64_t>& in_off,
                    const std::vector<const uint8_t*>& srcs, const std::vector<uint64_t>& lens, hipStream_t st) {
    Uploader& U = uploader(device);
    std::lock_guard<std::mutex> lock(U.mu);
    for (int k = 0; k < 2; k++) {
        if (!U.pin[k]) ck(hipHostMalloc(reinterpret_cast<void**>(&U.pin[k]), Uploader::WIN, hipHostMallocDefault));
        if (!U.done[k]) ck(hipEventCreate(&U.done[k]));
    }
    int k = 0;
    for (uint64_t a = 0; a < total; a += Uploader::WIN, k ^= 1) {
        const uint64_t b = std::min(a + Uploader::WIN, total);
        if (U.used[k]) ck(hipEventSynchronize(U.done[k]));  // the DMA of this window's last use
        const uint64_t n = b - a;
        const int nt = n >= (8ull << 20) ? 4 : 1;
        std::vector<std::thread> ts;
        for (int t = 1; t < nt; t++)
            ts.emplace_back(fill_window, U.pin[k] + n * t / nt, a + n * t / nt, a + n * (t + 1) / nt,
                            std::cref(in_off), std::cref(srcs), std::cref(lens));
        fill_window(U.pin[k], a, a + n / nt, in_off, srcs, lens);
        for (auto& t : ts) t.join();
        ck(hipMemcpyAsync(dev + a, U.pin[k], n, hipMemcpyHostToDevice, st));
        ck(hipEventRecord(U.done[k], st));
        U.used[k] = true;
    }
    ck(hipStreamSynchronize(st));
}

// The k_decode buckets (history size MB, MIX for constant / verbatim subframes) that get a
// launch of their own: predicted from the first subframe of each member's first frame, whose
// type byte follows the frame header (src/zflac.zig:426-429). k_decode classifies every frame
// group itself (the order-8 launch); groups of a bucket without a launch are decoded by the
// `rest` launch (enqueue_rest), after which the bucket is added to the mask (finish_batch).
uint32_t plan_buckets(const zflac_batch* b, const Class& C, const zflac_stream* src) {
    uint32_t mask = bucket_bit(8, false);
    for (uint32_t i : C.members) {
        const StreamState& s = b->streams[i];
        const uint64_t p = s.frames_begin + s.first.hdr_len;
        if (s.first.crc_eof || p >= s.len) continue;
        const uint32_t t = (src[i].data[p] >> 1) & 63;
        const uint32_t ord = t >= 32 ? t - 31 : (t >= 8 && t <= 12 ? t - 8 : 0);
        if (t <= 1) mask |= bucket_bit(8, true) | bucket_bit(32, true);  // the wave's order is unknown
        else mask |= bucket_bit(ord <= 4 ? 4 : ord <= 8 ? 8 : ord <= 12 ? 12 : ord <= 16 ? 16 : 32, false);
    }
    return mask;
}

// Output room for a stream whose STREAMINFO total is 0 (unknown): zflac then reads frames until
// fewer than 4 bytes are left (src/zflac.zig:343-350) and grows its buffer as it goes. Once per
// batch (here, at creation) a k_scan over the class gives every stream's frame-sync candidates
// and the sample units their headers claim; the chain zflac walks is made of candidates, so
// their units bound its output. That is the stream's reservation, and the parallel pass then
// certifies its chain to the end of the stream (k_verify). A stream whose candidates claim more
// than UNKNOWN_MAX_PER_BYTE output elements per input byte (a flood of false syncs) gets no
// reservation and goes to the sequential planner. (Silence as constant subframes, the most
// compressible content, is ~800 elements per byte at 4,096-sample blocks.)
constexpr uint64_t UNKNOWN_MAX_PER_BYTE = 4096;

void prescan_unknown_totals(zflac_batch* b, Class& C, std::vector<uint64_t>& units, std::vector<uint64_t>& cands) {
    hipStream_t st = b->stream;
    ScanArgs sa;
    sa.in = C.in.p;
    sa.streams = C.d_desc.p;
    sa.chunks = C.d_chunks.p;
    sa.n_chunks = (uint32_t)C.chunks.size();
    sa.chunk_cnt = C.chunk_cnt.p;
    sa.chunk_units = C.chunk_units.p;
    sa.chunk_slots = C.chunk_slots.p;
    sa.chunk_slot_units = C.chunk_slot_units.p;
    sa.status = C.status;
    sa.n_status = (uint32_t)C.members.size();
    sa.misc = C.misc.p;
    ck(launch_scan(sa, st));
    std::vector<uint32_t> cnt(C.chunks.size());
    std::vector<unsigned long long> u(C.chunks.size());
    if (!C.chunks.empty()) {
        ck(hipMemcpyAsync(cnt.data(), C.chunk_cnt.p, cnt.size() * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
        ck(hipMemcpyAsync(u.data(), C.chunk_units.p, u.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost, st));
    }
    ck(hipStreamSynchronize(st));
    units.assign(C.members.size(), 0);
    cands.assign(C.members.size(), 0);
    for (size_t k = 0; k < C.chunks.size(); k++) {
        units[C.chunks[k].stream] += u[k];
        cands[C.chunks[k].stream] += cnt[k];
    }
}

void alloc_class(zflac_batch* b, Class& C, const zflac_stream* src) {
    C.full_mask = plan_buckets(b, C, src);
    const int esz = esz_of_kind(C.kind);
    // input layout: each stream 16-byte aligned
    std::vector<uint64_t> in_off(C.members.size());
    uint64_t off = 0;
    for (size_t m = 0; m < C.members.size(); m++) {
        in_off[m] = off;
        off += (b->streams[C.members[m]].len + 15) & ~(uint64_t)15;
    }
    C.in_bytes = off;
    C.in.alloc(off + INPUT_PAD);
    uint64_t est_frames = 0, grid_frames = 0;
    C.desc.resize(C.members.size());
    C.chunks.clear();
    C.any_unknown = false;
    for (size_t m = 0; m < C.members.size(); m++) {
        StreamState& s = b->streams[C.members[m]];
        s.slot = (uint32_t)m;
        StreamDesc& D = C.desc[m];
        std::memset(&D, 0, sizeof(D));
        D.in_begin = in_off[m] + s.frames_begin;
        D.in_end = in_off[m] + s.len;
        D.valid_total = s.si.total > 0;
        D.total = D.valid_total ? s.si.total * (uint64_t)s.nch : 0;
        D.out_cap = D.total;  // (total unknown: from the pre-scan below)
        if (!D.valid_total) C.any_unknown = true;
        D.rate_hz = s.first.rate;
        D.si_rate = s.si.sample_rate;
        D.byte1 = (uint8_t)s.first.byte1;
        D.nch = (uint8_t)s.nch;
        D.dcode = (uint8_t)s.first.dcode;
        D.si_bps = (uint8_t)s.si.bps;
        D.justify = justify_of(s.si.bps);
        D.first_chunk = (uint32_t)C.chunks.size();
        const uint64_t abase0 = D.in_begin & ~(uint64_t)15;
        for (uint64_t a = abase0; a < D.in_end; a += CHUNK_BYTES) {
            ChunkDesc ch;
            ch.begin = std::max(a, D.in_begin);
            ch.end = std::min(a + CHUNK_BYTES, D.in_end);
            ch.stream = (uint32_t)m;
            ch.pad_ = 0;
            C.chunks.push_back(ch);
        }
        D.end_chunk = (uint32_t)C.chunks.size();
        const uint64_t minb = std::max<uint64_t>(16, s.si.min_block ? s.si.min_block : 16);
        // (at most one candidate per two bytes: a huge STREAMINFO total cannot inflate it)
        const uint64_t est = std::min<uint64_t>(s.si.total ? s.si.total / minb : s.len / 16, s.len / 2) + 2;
        if (D.valid_total) est_frames += est;  // (total unknown: the pre-scan's candidate count)
        // fixed blocking with a known total: zflac reads exactly ceil(total / block) frames (:341)
        const bool fixed = s.si.min_block == s.si.max_block && s.si.min_block >= 16;
        if (D.valid_total) grid_frames += fixed ? (s.si.total + s.si.min_block - 1) / s.si.min_block : est;
    }
    std::vector<const uint8_t*> srcs(C.members.size());
    std::vector<uint64_t> lens(C.members.size());
    for (size_t m = 0; m < C.members.size(); m++) {
        srcs[m] = src[C.members[m]].data;
        lens[m] = b->streams[C.members[m]].len;
    }
    upload_streams(b->device, C.in.p, C.in.n, in_off, srcs, lens, b->stream);  // inputs resident in HBM
    C.d_desc.alloc(C.desc.size());
    const size_t nc = std::max<size_t>(C.chunks.size(), 1);
    C.d_chunks.alloc(nc);
    if (!C.chunks.empty())
        ck(hipMemcpy(C.d_chunks.p, C.chunks.data(), C.chunks.size() * sizeof(ChunkDesc), hipMemcpyHostToDevice));
    C.chunk_cnt.alloc(nc);
    C.chunk_units.alloc(nc);
    C.chunk_slots.alloc(nc * CHUNK_CAP);
    C.chunk_slot_units.alloc(nc * CHUNK_CAP);
    C.chunk_off.alloc(nc + 1);
    C.chunk_uoff.alloc(nc + 1);
    C.misc.alloc(4 + C.members.size());
    C.status = C.misc.p + 4;
    C.dummy.alloc(DUMMY_BYTES + PROBE_BYTES);
    if (C.any_unknown) {  // reservations of the streams without a STREAMINFO total
        ck(hipMemcpy(C.d_desc.p, C.desc.data(), C.desc.size() * sizeof(StreamDesc), hipMemcpyHostToDevice));
        std::vector<uint64_t> units, cands;
        prescan_unknown_totals(b, C, units, cands);
        for (size_t m = 0; m < C.members.size(); m++) {
            StreamDesc& D = C.desc[m];
            if (D.valid_total) continue;
            const uint64_t avail = D.in_end - D.in_begin;
            D.out_cap = units[m] <= UNKNOWN_MAX_PER_BYTE * avail + (1u << 20) ? units[m] : 0;
            est_frames += cands[m] + 2;
            grid_frames += cands[m] + 2;
        }
    }
    // output layout: each stream's region starts on a 32-byte boundary, whatever the length of
    // the streams before it: the packed 16-byte stores of the fast path need 16-byte aligned
    // frames, and zflac's backing is 32-byte aligned (:331)
    const uint64_t align_elems = 32 / (uint64_t)esz;
    auto layout = [&]() {
        uint64_t o = 0;
        for (StreamDesc& D : C.desc) {
            o = (o + align_elems - 1) & ~(align_elems - 1);
            D.out_base = o;
            o += D.out_cap;
        }
        return o;
    };
    uint64_t out = layout();
    if (C.any_unknown) {
        // The reservations of unknown totals come from candidate headers, which planted false
        // syncs can inflate: together with the rest of the class they get at most half of the
        // device's free memory (the largest dropped first, to the planner), and none at all if
        // the allocation still fails.
        size_t free_b = 0, total_b = 0;
        if (hipMemGetInfo(&free_b, &total_b) != hipSuccess) free_b = 0;
        while (out * esz > free_b / 2) {
            StreamDesc* big = nullptr;
            for (StreamDesc& D : C.desc)
                if (!D.valid_total && D.out_cap && (!big || D.out_cap > big->out_cap)) big = &D;
            if (!big) break;
            big->out_cap = 0;
            out = layout();
        }
    }
    try {
        C.out.alloc(out * esz + 32);
    } catch (const DeviceError&) {
        bool dropped = false;
        for (StreamDesc& D : C.desc)
            if (!D.valid_total && D.out_cap) {
                D.out_cap = 0;
                dropped = true;
            }
        if (!dropped) throw;
        (void)hipGetLastError();  // (the failed hipMalloc's error must not surface at a later check)
        out = layout();
        C.out.alloc(out * esz + 32);
    }
    C.out_elems = out;
    ck(hipMemcpy(C.d_desc.p, C.desc.data(), C.desc.size() * sizeof(StreamDesc), hipMemcpyHostToDevice));
    const size_t units_at = (4 + C.members.size() + 1) & ~(size_t)1;  // (u32 index, 8-byte aligned)
    const size_t pin_words = units_at + (C.any_unknown ? 2 * C.members.size() : 0);
    ck(hipHostMalloc(reinterpret_cast<void**>(&C.pin.p), pin_words * sizeof(uint32_t), hipHostMallocDefault));
    std::memset(C.pin.p, 0, pin_words * sizeof(uint32_t));
    C.h_misc = C.pin.p;
    C.h_status = C.pin.p + 4;
    if (C.any_unknown) {
        C.units.alloc(C.members.size());
        C.h_units = reinterpret_cast<uint64_t*>(C.pin.p + units_at);
    }
    C.cap = (uint32_t)std::min<uint64_t>(est_frames + C.chunks.size() * 2 + 1024, 0x7FFFFFFFull);
    C.est_frames = est_frames;
    C.grid_frames = (uint32_t)std::min<uint64_t>(grid_frames + grid_frames / 64 + 64, C.cap);
}

void alloc_candidates(Class& C) {
    C.c_pos.alloc(C.cap);
    C.c_out.alloc(C.cap);
    C.c_end.alloc(C.cap);
    C.c_stream.alloc(C.cap);
    C.c_info.alloc(C.cap);
    C.c_rate.alloc(C.cap);
    C.c_err.alloc(C.cap);
    C.sub.alloc((size_t)C.cap * MAX_CH);
    C.group_mb.alloc((size_t)C.cap / 4 + 2);  // one per k_decode frame group (>= 8 frames each)
}

DecodeArgs decode_args(Class& C) {
    DecodeArgs a;
    std::memset(&a, 0, sizeof(a));
    a.in = C.in.p;
    a.in_size = C.in.n;
    a.out = C.out.p;
    a.streams = C.d_desc.p;
    a.c_pos = C.c_pos.p;
    a.c_stream = C.c_stream.p;
    a.c_out = C.c_out.p;
    a.n_frames = C.misc.p;
    a.cap = C.cap;
    a.c_end = C.c_end.p;
    a.c_err = C.c_err.p;
    a.c_info = C.c_info.p;
    a.c_rate = C.c_rate.p;
    a.nch = C.nch;
    a.write = 1;
    a.dummy = C.dummy.p;
    a.sub_start = C.sub.p;
    a.group_mb = C.group_mb.p;
    return a;
}

// Launch the whole parallel pipeline of one class on the batch stream.
void enqueue_class(zflac_batch* b, Class& C, bool timing_first, bool timing_last) {
    hipStream_t st = b->front ? b->front : b->rs;  // scan, compact (and the walk) there
    const uint32_t nch = (uint32_t)C.chunks.size();
    if (nch == 0)  // (k_scan zeroes them otherwise)
        ck(hipMemsetAsync(C.misc.p, 0, (4 + C.members.size()) * sizeof(uint32_t), st));
    if (timing_first) ck(hipEventRecord(b->ev[0], st));
    ScanArgs sa;
    sa.in = C.in.p;
    sa.streams = C.d_desc.p;
    sa.chunks = C.d_chunks.p;
    sa.n_chunks = nch;
    sa.chunk_cnt = C.chunk_cnt.p;
    sa.chunk_units = C.chunk_units.p;
    sa.chunk_slots = C.chunk_slots.p;
    sa.chunk_slot_units = C.chunk_slot_units.p;
    sa.status = C.status;
    sa.n_status = (uint32_t)C.members.size();
    sa.misc = C.misc.p;
    ck(launch_scan(sa, st));
    if (nch) ck(launch_scan_chunks(C.chunk_cnt.p, C.chunk_units.p, nch, C.chunk_off.p, C.chunk_uoff.p, C.misc.p, st));
    CompactArgs ca;
    ca.in = C.in.p;
    ca.streams = C.d_desc.p;
    ca.chunks = C.d_chunks.p;
    ca.n_chunks = nch;
    ca.chunk_cnt = C.chunk_cnt.p;
    ca.chunk_slots = C.chunk_slots.p;
    ca.chunk_slot_units = C.chunk_slot_units.p;
    ca.chunk_off = C.chunk_off.p;
    ca.chunk_uoff = C.chunk_uoff.p;
    ca.cap = C.cap;
    ca.c_pos = C.c_pos.p;
    ca.c_stream = C.c_stream.p;
    ca.c_out = C.c_out.p;
    ca.overflow = C.misc.p + 1;
    ck(launch_compact(ca, st));
    if (timing_last) ck(hipEventRecord(b->ev[1], st));
    DecodeArgs da = decode_args(C);
    da.bucket_used = C.misc.p + 2;
    da.full_mask = C.full_mask;
    ck(launch_decode(C.kind, da, std::min(C.grid_frames, C.cap), b->rs, timing_last ? b->ev[4] : nullptr,
                     b->front, b->front_join, C.est_frames, b->flags));
    st = b->rs;  // decode, verify and the read-backs
    if (timing_last) ck(hipEventRecord(b->ev[2], st));
    VerifyArgs va;
    va.streams = C.d_desc.p;
    va.n_streams = (uint32_t)C.members.size();
    va.chunk_off = C.chunk_off.p;
    va.c_pos = C.c_pos.p;
    va.c_stream = C.c_stream.p;
    va.c_out = C.c_out.p;
    va.n_frames = C.misc.p;
    va.cap = C.cap;
    va.c_end = C.c_end.p;
    va.c_err = C.c_err.p;
    va.c_info = C.c_info.p;
    va.c_rate = C.c_rate.p;
    va.status = C.status;
    va.units = C.any_unknown ? C.units.p : nullptr;
    ck(launch_verify(va, C.cap, st));
    if (timing_last) ck(hipEventRecord(b->ev[3], st));
    // the counters and the status words in one read-back (contiguous on both sides)
    ck(hipMemcpyAsync(C.h_misc, C.misc.p, (4 + C.members.size()) * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    if (C.any_unknown)
        ck(hipMemcpyAsync(C.h_units, C.units.p, C.members.size() * sizeof(uint64_t), hipMemcpyDeviceToHost, st));
}

// After a run whose order-8 launch found frame groups of a bucket the host did not
// predict (bucket_used outside full_mask): the rest launch decodes them, then the chain
// check and the read-backs run again (synchronous; a correct prediction never gets here).
void enqueue_rest(zflac_batch* b, Class& C) {
    hipStream_t st = b->stream;
    DecodeArgs da = decode_args(C);
    da.full_mask = C.full_mask;
    da.rest_only = 1;
    ck(launch_decode(C.kind, da, std::min(C.grid_frames, C.cap), st));
    ck(hipMemsetAsync(C.status, 0, C.members.size() * sizeof(uint32_t), st));
    VerifyArgs va;
    va.streams = C.d_desc.p;
    va.n_streams = (uint32_t)C.members.size();
    va.chunk_off = C.chunk_off.p;
    va.c_pos = C.c_pos.p;
    va.c_stream = C.c_stream.p;
    va.c_out = C.c_out.p;
    va.n_frames = C.misc.p;
    va.cap = C.cap;
    va.c_end = C.c_end.p;
    va.c_err = C.c_err.p;
    va.c_info = C.c_info.p;
    va.c_rate = C.c_rate.p;
    va.status = C.status;
    va.units = C.any_unknown ? C.units.p : nullptr;
    ck(launch_verify(va, C.cap, st));
    ck(hipMemcpyAsync(C.h_status, C.status, C.members.size() * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    if (C.any_unknown)
        ck(hipMemcpyAsync(C.h_units, C.units.p, C.members.size() * sizeof(uint64_t), hipMemcpyDeviceToHost, st));
    ck(hipStreamSynchronize(st));
}

// ---------------------------------------------------------------------------------
// Sequential chain planner (src/zflac.zig:340-581 state machine) for streams the
// fast path could not certify. Frame records come from the fast pass when the chain
// position is a sync candidate, otherwise from a one-frame device probe.
// ---------------------------------------------------------------------------------
struct FrameRec {
    uint64_t end;
    int32_t err;
    uint32_t info;
    uint32_t rate;
};

struct SeqRunner {
    zflac_batch* b;
    Class& C;
    uint32_t slot;
    DevBuf<uint64_t> p_pos, p_out, p_end;
    DevBuf<uint32_t> p_stream, p_info, p_rate;
    DevBuf<int32_t> p_err;
    DevBuf<uint32_t> p_sub, p_mb, p_crc, p_cnt;
    DevBuf<uint64_t> p_sync;
    DevBuf<StreamDesc> p_desc;

    SeqRunner(zflac_batch* b_, Class& C_, uint32_t slot_) : b(b_), C(C_), slot(slot_) {}

    // decode the explicit frame list `pos` (absolute input offsets) with output offsets
    // `outoff` relative to `desc.out_base`; returns records
    void run_list(const std::vector<uint64_t>& pos, const std::vector<uint64_t>& outoff, const StreamDesc& desc,
                  void* out, int write, std::vector<FrameRec>& recs) {
        const size_t n = pos.size();
        p_pos.alloc(n);
        p_out.alloc(n);
        p_end.alloc(n);
        p_stream.alloc(n);
        p_info.alloc(n);
        p_rate.alloc(n);
        p_err.alloc(n);
        p_desc.alloc(1);
        std::vector<uint32_t> zeros(n, 0);
        hipStream_t st = b->stream;
        ck(hipMemcpyAsync(p_pos.p, pos.data(), n * 8, hipMemcpyHostToDevice, st));
        ck(hipMemcpyAsync(p_out.p, outoff.data(), n * 8, hipMemcpyHostToDevice, st));
        ck(hipMemcpyAsync(p_stream.p, zeros.data(), n * 4, hipMemcpyHostToDevice, st));
        ck(hipMemcpyAsync(p_desc.p, &desc, sizeof(desc), hipMemcpyHostToDevice, st));
        DecodeArgs a;
        std::memset(&a, 0, sizeof(a));
        a.in = C.in.p;
        a.in_size = C.in.n;
        a.out = out;
        a.streams = p_desc.p;
        a.c_pos = p_pos.p;
        a.c_stream = p_stream.p;
        a.c_out = p_out.p;
        a.n_frames = nullptr;
        a.n_frames_host = (uint32_t)n;
        a.cap = (uint32_t)n;
        a.c_end = p_end.p;
        a.c_err = p_err.p;
        a.c_info = p_info.p;
        a.c_rate = p_rate.p;
        a.nch = C.nch;
        a.write = write;
        a.dummy = C.dummy.p;
        p_sub.alloc(n * MAX_CH);
        a.sub_start = p_sub.p;
        p_mb.alloc(n / 4 + 2);
        a.group_mb = p_mb.p;
        ck(launch_decode(C.kind, a, (uint32_t)n, st, nullptr, nullptr, nullptr, 0, b->flags));
        std::vector<uint64_t> e(n);
        std::vector<int32_t> er(n);
        std::vector<uint32_t> in(n), ra(n);
        ck(hipMemcpyAsync(e.data(), p_end.p, n * 8, hipMemcpyDeviceToHost, st));
        ck(hipMemcpyAsync(er.data(), p_err.p, n * 4, hipMemcpyDeviceToHost, st));
        ck(hipMemcpyAsync(in.data(), p_info.p, n * 4, hipMemcpyDeviceToHost, st));
        ck(hipMemcpyAsync(ra.data(), p_rate.p, n * 4, hipMemcpyDeviceToHost, st));
        ck(hipStreamSynchronize(st));
        recs.resize(n);
        for (size_t i = 0; i < n; i++) recs[i] = FrameRec{e[i], er[i], in[i], ra[i]};
    }

    // Sync codes in [lo, hi) whose header matches the stream (k_sync_list), sorted.
    std::vector<uint64_t> sync_list(uint64_t lo, uint64_t hi, const StreamDesc& D) {
        hipStream_t st = b->stream;
        uint32_t cap = 4096, n = 0;
        for (int attempt = 0; attempt < 2; attempt++) {
            p_sync.alloc(cap);
            p_cnt.alloc(1);
            ck(hipMemsetAsync(p_cnt.p, 0, 4, st));
            SyncListArgs a;
            a.in = C.in.p;
            a.lo = lo;
            a.hi = hi;
            a.in_end = D.in_end;
            a.si_rate = D.si_rate;
            a.rate_hz = D.rate_hz;
            a.nch = D.nch;
            a.dcode = D.dcode;
            a.pos = p_sync.p;
            a.count = p_cnt.p;
            a.cap = cap;
            ck(launch_sync_list(a, st));
            ck(hipMemcpyAsync(&n, p_cnt.p, 4, hipMemcpyDeviceToHost, st));
            ck(hipStreamSynchronize(st));
            if (n <= cap) break;
            cap = n;  // more than fit: once more with room for all
        }
        std::vector<uint64_t> out(std::min(n, cap));
        if (!out.empty()) {
            ck(hipMemcpyAsync(out.data(), p_sync.p, out.size() * 8, hipMemcpyDeviceToHost, st));
            ck(hipStreamSynchronize(st));
        }
        std::sort(out.begin(), out.end());
        return out;
    }

    // k_crc16 over the frames [pos[i], end[i]); true when every trailer matches
    bool crc16_ok(const std::vector<uint64_t>& pos, const std::vector<uint64_t>& end) {
        const size_t n = pos.size();
        if (!n) return true;
        hipStream_t st = b->stream;
        p_pos.alloc(n);
        p_end.alloc(n);
        p_crc.alloc(n);
        ck(hipMemcpyAsync(p_pos.p, pos.data(), n * 8, hipMemcpyHostToDevice, st));
        ck(hipMemcpyAsync(p_end.p, end.data(), n * 8, hipMemcpyHostToDevice, st));
        Crc16Args a;
        std::memset(&a, 0, sizeof(a));
        a.in = C.in.p;
        a.in_size = C.in.n;
        a.pos = p_pos.p;
        a.end = p_end.p;
        a.n_frames_host = (uint32_t)n;
        a.cap = (uint32_t)n;
        a.bad = p_crc.p;
        ck(launch_crc16(a, (uint32_t)n, st));
        std::vector<uint32_t> bad(n);
        ck(hipMemcpyAsync(bad.data(), p_crc.p, n * 4, hipMemcpyDeviceToHost, st));
        ck(hipStreamSynchronize(st));
        return std::none_of(bad.begin(), bad.end(), [](uint32_t x) { return x != 0; });
    }
};

void finish_stream_sequential(zflac_batch* b, Class& C, uint32_t slot, const std::vector<uint32_t>& h_chunk_off,
                              uint32_t nframes) {
    StreamState& s = b->streams[C.members[slot]];
    const StreamDesc D = C.desc[slot];
    hipStream_t st = b->stream;
    // fast-pass records of this stream's candidates
    std::unordered_map<uint64_t, FrameRec> recs;
    const uint32_t f0 = std::min(h_chunk_off[D.first_chunk], nframes);
    const uint32_t f1 = std::min(h_chunk_off[D.end_chunk], nframes);
    if (f1 > f0 && !(b->flags & ZFLAC_FLAG_FORCE_SLOW)) {
        const size_t n = f1 - f0;
        std::vector<uint64_t> pos(n), end(n);
        std::vector<int32_t> err(n);
        std::vector<uint32_t> info(n), rate(n);
        ck(hipMemcpyAsync(pos.data(), C.c_pos.p + f0, n * 8, hipMemcpyDeviceToHost, st));
        ck(hipMemcpyAsync(end.data(), C.c_end.p + f0, n * 8, hipMemcpyDeviceToHost, st));
        ck(hipMemcpyAsync(err.data(), C.c_err.p + f0, n * 4, hipMemcpyDeviceToHost, st));
        ck(hipMemcpyAsync(info.data(), C.c_info.p + f0, n * 4, hipMemcpyDeviceToHost, st));
        ck(hipMemcpyAsync(rate.data(), C.c_rate.p + f0, n * 4, hipMemcpyDeviceToHost, st));
        ck(hipStreamSynchronize(st));
        for (size_t i = 0; i < n; i++) recs[pos[i]] = FrameRec{end[i], err[i], info[i], rate[i]};
    }
    SeqRunner R(b, C, slot);
    StreamDesc probe_desc = D;
    probe_desc.out_base = 0;
    probe_desc.out_cap = 0;
    probe_desc.valid_total = 0;
    probe_desc.total = 0;

    // state machine of decode_frames (src/zflac.zig:321-581)
    bool valid_total = s.si.total > 0;
    const uint64_t expC = s.si.channels;
    const uint64_t total = expC * (valid_total ? s.si.total : 4096);
    uint64_t buf_len = total;
    uint64_t offset = 0;
    uint64_t p = D.in_begin;
    bool first = true;
    uint32_t rate0 = 0, count0 = 0, dcode0 = 0;
    int bps0 = 0;
    std::vector<uint64_t> list_pos, list_out, list_end;
    int err = 0;
    // batched probes: a chain position without a record asks for every matching sync code
    // in a window ahead of it (doubling, 1 .. 64 MiB) and decodes them in one launch
    uint64_t probe_win = 1ull << 20;
    for (;;) {
        if (valid_total && offset >= total) break;  // :341
        if (D.in_end - p < 4) {                     // :343-350
            if (valid_total) err = E_END_OF_STREAM;
            break;
        }
        FrameRec rec;
        auto it = recs.find(p);
        if (it != recs.end()) {
            rec = it->second;
        } else {
            const uint64_t hi = std::min<uint64_t>(D.in_end, p + probe_win);
            probe_win = std::min<uint64_t>(probe_win * 2, 64ull << 20);
            std::vector<uint64_t> pos = R.sync_list(p, hi, D);
            if (pos.empty() || pos[0] != p) pos.insert(pos.begin(), p);  // zflac reads p whatever it holds
            std::vector<FrameRec> got;
            R.run_list(pos, std::vector<uint64_t>(pos.size(), 0), probe_desc, C.out.p, 0, got);
            for (size_t i = 0; i < pos.size(); i++) recs[pos[i]] = got[i];
            rec = recs[p];
        }
        if (rec.info & INFO_PRE_ERR) { err = rec.err; break; }
        const uint32_t bs = (rec.info & 0xFFFF) + 1, code = (rec.info >> 16) & 15, dcode = (rec.info >> 20) & 7;
        if (first) {  // :376-388
            rate0 = rec.rate;
            count0 = (uint32_t)channels_count_h(code);
            dcode0 = dcode;
            bps0 = depth_bits_h(dcode, (int)s.si.bps);
            if (bps0 < 0) { err = E_OUT_OF_DOMAIN; break; }
            if (count0 != expC) { err = E_INCONSISTENT_PARAMETERS; break; }
            first = false;
        } else if (rate0 != rec.rate || count0 != (uint32_t)channels_count_h(code) || dcode0 != dcode) {
            err = E_INCONSISTENT_PARAMETERS;  // :391
            break;
        }
        const uint64_t expected = offset + (uint64_t)bs * count0;  // :394-402
        if (buf_len < expected) {
            buf_len = std::max(2 * buf_len, expected);
            valid_total = false;
        }
        if (bs == 1 && valid_total && offset + count0 < total) { err = E_INVALID_FRAME_HEADER; break; }  // :405
        if (rec.info & INFO_CRC_EOF) { err = E_END_OF_STREAM; break; }
        if (rec.err) { err = rec.err; break; }
        list_pos.push_back(p);
        list_out.push_back(offset);
        list_end.push_back(rec.end);
        offset += (uint64_t)bs * count0;
        p = rec.end;
    }
    // optional CRC-16 of the frames read before the loop stopped: zflac would read each
    // trailer before the next frame, so a mismatch there comes before `err`
    if ((b->flags & ZFLAC_FLAG_CHECK_CRC16) && !R.crc16_ok(list_pos, list_end)) err = E_FRAME_CRC;
    s.err = err;
    if (err) return;
    // final decode of the certified chain into this stream's region (or an override)
    const int esz = esz_of_kind(C.kind);
    StreamDesc wd = D;
    wd.out_base = 0;
    wd.out_cap = offset;
    wd.valid_total = 0;
    wd.total = 0;
    uint8_t* dst;
    if (offset <= D.out_cap) {
        dst = C.out.p + D.out_base * esz;
    } else {
        s.override_out.reset(new DevBuf<uint8_t>());
        s.override_out->alloc(offset * esz + 16);
        dst = s.override_out->p;
    }
    if (!list_pos.empty()) {
        std::vector<FrameRec> out_recs;
        R.run_list(list_pos, list_out, wd, dst, 1, out_recs);
        for (auto& r : out_recs)
            if (r.err) { s.err = r.err; return; }
    }
    s.dev_samples = dst;
    s.info.n_samples = offset;
    s.info.channels = (uint8_t)count0;
    s.info.sample_rate = rate0;
    s.info.bits_per_sample = (uint8_t)bps0;
}

void run_md5_device(zflac_batch* b, const std::vector<uint32_t>& which, bool timing);
void finish_md5(zflac_batch* b, bool timing);

// ---------------------------------------------------------------------------------
// md5 hub: one per device. MD5 is one serial chain per stream (~8 ms for a C5 stream of
// 32 frames), so a run's hash lasts as long as its longest chain whatever its lane count.
// Hashing each run on its own batch stream made the decode+MD5 throughput the number of
// batches in flight over (decode + hash latency), and each batch held a hardware queue for
// its whole hash. The hub collects the DEVICE_MD5 runs whose decode has been enqueued and
// hashes up to MD5_MAX_SEGS of them in ONE k_md5_coop launch on its own stream (waiting
// on each run's decode event), so few launches and few hardware queues carry every chain.
// A run is flushed into a launch once `runs` are pending, when its batch is waited on, or
// when its batch polls _ready with its decode done and no hub launch in flight.
// ---------------------------------------------------------------------------------
constexpr int MAX_HUB_STREAMS = 4;
struct Md5Hub {
    std::mutex mu;
    hipStream_t st[MAX_HUB_STREAMS] = {};  // launches alternate between the first n_st
    uint32_t n_st = 1, next = 0;
    hipEvent_t last = nullptr;  // behind the newest hub launch
    bool any = false;
    std::vector<zflac_batch*> pend;
    uint32_t runs = 8;
    int device = 0;  // the hub's launches and copies run with this device current
};

// Makes `dev` the calling thread's current device for a scope and restores the previous
// one: hub flushes can be triggered from any batch's call (ready / wait / destroy), on a
// thread whose current device is another one.
struct DeviceScope {
    int prev = -1;
    explicit DeviceScope(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) ck(hipSetDevice(dev));
    }
    ~DeviceScope() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};

// ZFLAC_HUB_CUS=N (N > 0): the md5 hub's streams on N CUs of their own and the run streams on
// the others (hipExtStreamCreateWithCUMask; the lowest N bits of the device's CU mask). The
// hash is one serial chain per stream, compute-only: on CUs it shares with the decode, its
// waves slow the decode waves there, and a decode launch ends with its slowest wave.
static uint32_t hub_cus() {
    const char* e = std::getenv("ZFLAC_HUB_CUS");
    return e ? (uint32_t)std::max(0, atoi(e)) : 0u;
}

DeviceStreams::DeviceStreams() : hub_p(new Md5Hub()), hub(*hub_p) {
    if (const char* e = std::getenv("ZFLAC_RUN_STREAMS")) n_run = (uint32_t)std::max(1, std::min(atoi(e), MAX_RUN_STREAMS));
    if (const char* e = std::getenv("ZFLAC_HUB_STREAMS")) hub.n_st = (uint32_t)std::max(1, std::min(atoi(e), MAX_HUB_STREAMS));
    const uint32_t nh = hub_cus();
    int dev = 0, ncu = 0;
    ck(hipGetDevice(&dev));
    ck(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    if (nh > 0 && nh < (uint32_t)ncu) {
        const uint32_t words = ((uint32_t)ncu + 31) / 32;
        std::vector<uint32_t> hm(words, 0u), rm(words, 0u);
        for (uint32_t c = 0; c < (uint32_t)ncu; c++) (c < nh ? hm : rm)[c / 32] |= 1u << (c % 32);
        for (uint32_t i = 0; i < n_run; i++) ck(hipExtStreamCreateWithCUMask(&run[i], words, rm.data()));
        for (uint32_t i = 0; i < hub.n_st; i++) ck(hipExtStreamCreateWithCUMask(&hub.st[i], words, hm.data()));
    } else {
        for (uint32_t i = 0; i < n_run; i++) ck(hipStreamCreateWithFlags(&run[i], hipStreamNonBlocking));
        for (uint32_t i = 0; i < hub.n_st; i++) ck(hipStreamCreateWithFlags(&hub.st[i], hipStreamNonBlocking));
    }
    ck(hipEventCreateWithFlags(&hub.last, hipEventDisableTiming));
    if (const char* e = std::getenv("ZFLAC_MD5_RUNS")) hub.runs = (uint32_t)std::max(1, std::min(atoi(e), MD5_MAX_SEGS));
}

// (call with the device current)
DeviceStreams& device_streams(int device) {
    static std::mutex mu;
    static std::unordered_map<int, DeviceStreams*> per_device;  // never destroyed: outlives every batch
    std::lock_guard<std::mutex> lock(mu);
    DeviceStreams*& d = per_device[device];
    if (!d) {
        d = new DeviceStreams();
        d->hub.device = device;
    }
    return *d;
}

Md5Hub& md5_hub(int device) { return device_streams(device).hub; }

hipStream_t next_run_stream(int device) {
    DeviceStreams& d = device_streams(device);
    std::lock_guard<std::mutex> lock(d.mu);
    return d.run[d.next++ % d.n_run];
}

// One launch over every pending run (caller holds hub.mu). Any exit, a throwing HIP call
// included, leaves the hub empty: the runs of a launch that failed part way are marked
// md5_failed (their wait reports DeviceError) instead of staying queued, so no later flush
// can touch a batch destroyed in between.
void hub_flush_runs(Md5Hub& h);
void hub_flush(Md5Hub& h) {
    if (h.pend.empty()) return;
    try {
        DeviceScope dev(h.device);
        hub_flush_runs(h);
    } catch (...) {
        for (zflac_batch* b : h.pend) {
            if (b->md5_pending) b->md5_failed = true;
            b->md5_pending = false;
        }
        h.pend.clear();
        throw;
    }
}

void hub_flush_runs(Md5Hub& h) {
    // fault injection for the tests only (tests/test_gpu.py: a failed hub launch must not
    // poison the batch's next run): ZFLAC_FAULT_HUB_FLUSH=1 makes this flush throw
    if (const char* f = std::getenv("ZFLAC_FAULT_HUB_FLUSH"); f && f[0] == '1') throw DeviceError{};
    hipStream_t hs = h.st[h.next++ % h.n_st];
    Md5Segs sg;
    std::memset(&sg, 0, sizeof(sg));
    uint32_t n = 0;
    int coop = h.pend[0]->pipe_coop;  // the cooperative kernel only when every run's jobs allow it
    for (zflac_batch* b : h.pend) {
        if (b->pipe_coop != coop) coop = -1;
        ck(hipStreamWaitEvent(hs, b->ev_done, 0));
        sg.jobs[sg.nseg] = b->pipe_jobs.p;
        sg.dig[sg.nseg] = b->pipe_dig.p;
        sg.start[sg.nseg] = n;
        n += (uint32_t)b->pipe_who.size();
        sg.nseg++;
    }
    sg.start[sg.nseg] = n;
    for (zflac_batch* b : h.pend)  // every run gets the shared launch's time (md5_ms)
        if (b->flags & ZFLAC_FLAG_TIMING) ck(hipEventRecord(b->ev[8], hs));
    ck(launch_md5_multi(sg, hs, coop));
    for (zflac_batch* b : h.pend) {
        if (b->flags & ZFLAC_FLAG_TIMING) ck(hipEventRecord(b->ev[9], hs));
        ck(hipMemcpyAsync(b->pipe_pin, b->pipe_dig.p, b->pipe_who.size() * 16, hipMemcpyDeviceToHost, hs));
        ck(hipEventRecord(b->ev_md5, hs));
        b->md5_pending = false;
    }
    ck(hipEventRecord(h.last, hs));
    h.any = true;
    h.pend.clear();
}

// The run's hash launched (flushing the hub if it is still pending).
void hub_release(zflac_batch* b) {
    if (!b->md5_pending) return;
    Md5Hub& h = md5_hub(b->device);
    std::lock_guard<std::mutex> lock(h.mu);
    if (b->md5_pending) hub_flush(h);
}

// Drop the run from the hub without hashing it (a failed submit or wait, a destroyed batch).
void hub_forget(zflac_batch* b) {
    Md5Hub& h = md5_hub(b->device);
    std::lock_guard<std::mutex> lock(h.mu);
    h.pend.erase(std::remove(h.pend.begin(), h.pend.end(), b), h.pend.end());
    b->md5_pending = false;
    b->md5_failed = false;  // a forgotten run has no hash to fail; never leak into the next run
}

// Phase 1 of a run: every class's parallel pipeline on the next of the device's run streams,
// no host wait. Batches submitted back to back overlap on the device (each has its own
// buffers, consecutive runs different streams): the scan and walk of one run beside the
// decode of the other.
void submit_batch(zflac_batch* b) {
    ck(hipSetDevice(b->device));
    const bool timing = (b->flags & ZFLAC_FLAG_TIMING) != 0;
    // (no wait on the batch's own stream: everything create and finish enqueue there is
    // synchronized before they return. A marker recorded there would sit in a hardware queue
    // it may share with a run or md5 hub stream, behind a hash of several milliseconds.)
    b->rs = next_run_stream(b->device);
    for (size_t ci = 0; ci < b->classes.size(); ci++) {
        Class& C = *b->classes[ci];
        C.redone = false;
        alloc_candidates(C);
        enqueue_class(b, C, timing && ci == 0, timing && ci + 1 == b->classes.size());
    }
    b->md5_hub = !b->pipe_who.empty() && !std::getenv("ZFLAC_MD5_NOHUB");
    if (!b->pipe_who.empty() && !b->md5_hub) {  // STREAMINFO MD5 of the streams this run certifies
        const uint32_t n = (uint32_t)b->pipe_who.size();
        if (timing) ck(hipEventRecord(b->ev[8], b->rs));
        ck(launch_md5(b->pipe_jobs.p, n, b->pipe_dig.p, b->rs, b->pipe_coop));
        if (timing) ck(hipEventRecord(b->ev[9], b->rs));
        ck(hipMemcpyAsync(b->pipe_pin, b->pipe_dig.p, (size_t)n * 16, hipMemcpyDeviceToHost, b->rs));
    }
    ck(hipEventRecord(b->ev_done, b->rs));  // zflac_hip_batch_ready
    if (b->md5_hub) {  // the hash of the streams this run certifies, in the device's md5 hub
        Md5Hub& h = md5_hub(b->device);
        std::lock_guard<std::mutex> lock(h.mu);
        b->md5_failed = false;  // (a failure of an earlier run of this batch is that run's)
        b->md5_pending = true;
        h.pend.push_back(b);
        if (h.pend.size() >= std::min<uint32_t>(h.runs, MD5_MAX_SEGS)) hub_flush(h);
    }
}

// Phase 2: wait for the pipeline, redo a class whose candidate table overflowed (grown,
// synchronously; not part of the recorded kernel timings), then the per-stream results,
// the sequential planner for streams the chain check did not certify, CRC-16 and MD5.
void finish_batch(zflac_batch* b) {
    ck(hipSetDevice(b->device));
    const bool timing = (b->flags & ZFLAC_FLAG_TIMING) != 0;
    ck(hipEventSynchronize(b->ev_done));  // the run, on its run stream
    b->rs = b->stream;  // from here on (regrowth, rest launch, planner): the batch's own stream
    if (b->md5_hub) {  // the run's hash (and its digests' read-back) in the md5 hub
        hub_release(b);
        if (b->md5_failed) {
            b->md5_failed = false;
            throw DeviceError{};  // the md5 hub launch holding this run failed
        }
        ck(hipEventSynchronize(b->ev_md5));
    }
    uint32_t rest_launches = 0, sequential = 0;
    for (size_t ci = 0; ci < b->classes.size(); ci++) {
        Class& C = *b->classes[ci];
        for (int attempt = 0; attempt < 3; attempt++) {
            if (!C.h_misc[1] && C.h_misc[0] <= C.cap) break;
            C.cap = std::max<uint32_t>(C.h_misc[0] + 1024, C.cap * 2);  // candidate table overflow: grow, redo
            C.grid_frames = std::max(C.grid_frames, C.h_misc[0]);
            alloc_candidates(C);
            C.redone = true;
            enqueue_class(b, C, false, false);
            ck(hipStreamSynchronize(b->stream));
        }
        // more candidates than the grids were sized for (false syncs): correct (the kernels
        // stride over them), but slower; size the next run's grids for them
        if (C.h_misc[0] > C.grid_frames) C.grid_frames = std::min(C.cap, C.h_misc[0] + C.h_misc[0] / 64 + 64);
        if (C.full_mask && (C.h_misc[2] & ~C.full_mask)) {  // a bucket without a launch was used
            enqueue_rest(b, C);
            C.redone = true;
            rest_launches++;
            // from now on that bucket gets a launch of its own: later runs keep the pipelined
            // MD5 and skip the synchronous rest launch (launches are only ever added)
            C.full_mask |= C.h_misc[2] & BUCKET_MASK_ALL;
        }
    }
    const bool crc = (b->flags & ZFLAC_FLAG_CHECK_CRC16) != 0;
    b->timings.crc16_ms = 0;
    if (crc && !b->classes.empty()) {  // every candidate's trailer, after the chain checks
        if (timing) ck(hipEventRecord(b->ev[5], b->stream));
        for (auto& cp : b->classes) {
            Class& C = *cp;
            C.crc_bad.alloc(C.cap);
            Crc16Args a;
            std::memset(&a, 0, sizeof(a));
            a.in = C.in.p;
            a.in_size = C.in.n;
            a.pos = C.c_pos.p;
            a.end = C.c_end.p;
            a.err = C.c_err.p;
            a.streams = C.d_desc.p;
            a.c_stream = C.c_stream.p;
            a.c_out = C.c_out.p;
            a.n_frames = C.misc.p;
            a.cap = C.cap;
            a.bad = C.crc_bad.p;
            ck(launch_crc16(a, std::min(C.h_misc[0], C.cap), b->stream));
        }
        if (timing) ck(hipEventRecord(b->ev[6], b->stream));
        ck(hipStreamSynchronize(b->stream));
        if (timing) {
            float tc = 0;
            ck(hipEventElapsedTime(&tc, b->ev[5], b->ev[6]));
            b->timings.crc16_ms = tc;
        }
    }
    if (timing && !b->classes.empty()) {
        float t01 = 0, t14 = 0, t42 = 0, t23 = 0, t03 = 0;
        ck(hipEventElapsedTime(&t01, b->ev[0], b->ev[1]));
        ck(hipEventElapsedTime(&t14, b->ev[1], b->ev[4]));
        ck(hipEventElapsedTime(&t42, b->ev[4], b->ev[2]));
        ck(hipEventElapsedTime(&t23, b->ev[2], b->ev[3]));
        ck(hipEventElapsedTime(&t03, b->ev[0], b->ev[3]));
        b->timings.scan_ms = t01;
        b->timings.walk_ms = t14;
        b->timings.decode_ms = t42;
        b->timings.verify_ms = t23;
        b->timings.total_ms = t03;
        b->have_timing = true;
    }
    // results
    uint64_t frames = 0, in_bytes = 0, out_bytes = 0, samples = 0;
    for (auto& cp : b->classes) {
        Class& C = *cp;
        const int esz = esz_of_kind(C.kind);
        std::vector<uint32_t> h_off, h_crc;
        const uint32_t nfr = std::min(C.h_misc[0], C.cap);
        if (crc && nfr) {
            h_crc.resize(nfr);
            ck(hipMemcpy(h_crc.data(), C.crc_bad.p, nfr * 4, hipMemcpyDeviceToHost));
        }
        for (size_t m = 0; m < C.members.size(); m++) {
            StreamState& s = b->streams[C.members[m]];
            s.override_out.reset();
            s.info = zflac_info{};
            s.info.sample_kind = (uint8_t)C.kind;
            if (C.h_status[m] == 0 && !(b->flags & ZFLAC_FLAG_FORCE_SLOW)) {
                const StreamDesc& D = C.desc[m];
                s.err = 0;
                s.dev_samples = C.out.p + D.out_base * esz;
                s.info.n_samples = D.valid_total ? D.total : C.h_units[m];
                s.info.channels = (uint8_t)s.nch;
                s.info.sample_rate = s.first.rate;
                s.info.bits_per_sample = (uint8_t)depth_bits_h(s.first.dcode, (int)s.si.bps);
                if (crc) {  // a certified stream's candidates up to its total are exactly its frames
                            // (k_crc16 passes the ones past the total: zflac never reads them)
                    if (h_off.empty()) {
                        h_off.resize(C.chunks.size() + 1);
                        ck(hipMemcpy(h_off.data(), C.chunk_off.p, h_off.size() * 4, hipMemcpyDeviceToHost));
                    }
                    const uint32_t f0 = std::min(h_off[D.first_chunk], nfr), f1 = std::min(h_off[D.end_chunk], nfr);
                    for (uint32_t f = f0; f < f1; f++)
                        if (h_crc[f]) {
                            s.err = E_FRAME_CRC;
                            s.info = zflac_info{};
                            s.info.sample_kind = (uint8_t)C.kind;
                            break;
                        }
                }
            } else {
                if (h_off.empty()) {
                    h_off.resize(C.chunks.size() + 1);
                    ck(hipMemcpy(h_off.data(), C.chunk_off.p, h_off.size() * 4, hipMemcpyDeviceToHost));
                }
                finish_stream_sequential(b, C, (uint32_t)m, h_off, std::min(C.h_misc[0], C.cap));
                sequential++;
            }
            s.info.samples_bytes = s.info.n_samples * esz;
            if (!s.err) {
                in_bytes += s.len - s.frames_begin;
                out_bytes += s.info.samples_bytes;
                samples += s.info.n_samples;
            }
        }
        frames += std::min(C.h_misc[0], C.cap);
    }
    b->timings.md5_ms = 0;
    if (b->flags & ZFLAC_FLAG_DEVICE_MD5) finish_md5(b, timing && !b->classes.empty());
    else
        for (auto& s : b->streams) s.md5_dev = 0;
    b->timings.frames = frames;
    b->timings.input_bytes = in_bytes;
    b->timings.output_bytes = out_bytes;
    b->timings.samples = samples;
    b->timings.rest_launches = rest_launches;
    b->timings.sequential_streams = sequential;
}

// MD5 of the decoded stream exactly as zflac hashes it: before left-justify, 24-bit
// containers hash 3 bytes per sample (src/zflac.zig:267-280). Fed in element-aligned
// pieces, so the read can hash chunks as they land.
class SampleHasher {
public:
    explicit SampleHasher(const StreamState& s)
        : kind_(s.kind), js_(justify_of(s.si.bps)), w24_((s.si.bps + 7) / 8 * 8 == 24) {}
    void update(const void* samples, uint64_t n) {  // n elements of the stream's container
        if (kind_ == 0 || (kind_ == 1 && !js_) || (kind_ == 2 && !js_ && !w24_)) {
            md_.update(samples, n * (kind_ == 0 ? 1 : kind_ == 1 ? 2 : 4));
            return;
        }
        uint8_t tmp[4096 * 4];
        for (uint64_t i = 0; i < n; i += 4096) {
            const uint64_t m = std::min<uint64_t>(4096, n - i);
            if (kind_ == 1) {
                const int16_t* v = static_cast<const int16_t*>(samples) + i;
                int16_t* t = reinterpret_cast<int16_t*>(tmp);
                for (uint64_t k = 0; k < m; k++) t[k] = (int16_t)(v[k] >> js_);
                md_.update(tmp, m * 2);
            } else {
                const int32_t* v = static_cast<const int32_t*>(samples) + i;
                const int w = w24_ ? 3 : 4;
                for (uint64_t k = 0; k < m; k++) {
                    const uint32_t x = (uint32_t)(v[k] >> js_);
                    for (int bb = 0; bb < w; bb++) tmp[k * w + bb] = (uint8_t)(x >> (8 * bb));
                }
                md_.update(tmp, m * w);
            }
        }
    }
    bool matches(const uint8_t* expected) {
        uint8_t dig[16];
        md_.finish(dig);
        return std::memcmp(dig, expected, 16) == 0;
    }

private:
    Md5 md_;
    int kind_;
    uint32_t js_;
    bool w24_;
};

bool md5_matches(const StreamState& s, const void* host_samples) {
    SampleHasher h(s);
    h.update(host_samples, s.info.n_samples);
    return h.matches(s.si.md5);
}

// D2H of one stream's samples into caller memory, with the STREAMINFO MD5 when `hash`.
// Long streams: the calling thread copies chunk after chunk while a helper thread hashes
// every chunk already landed, so the call costs about max(D2H, MD5) instead of their sum.
int read_samples(zflac_batch* b, StreamState& s, void* out, bool hash) {
    const uint64_t bytes = s.info.samples_bytes;
    const uint64_t esz = (uint64_t)esz_of_kind(s.kind);
    constexpr uint64_t CHUNK = 32ull << 20;  // a multiple of every element size
    const double t0 = now_ms();
    double t_md5 = 0;
    bool ok = true;
    if (!hash || bytes <= 2 * CHUNK) {
        if (bytes) ck(hipMemcpy(out, s.dev_samples, bytes, hipMemcpyDeviceToHost));
        if (hash) {
            const double t1 = now_ms();
            ok = md5_matches(s, out);
            t_md5 = now_ms() - t1;
        }
    } else {
        std::atomic<uint64_t> landed{0};
        std::thread hasher([&] {
            const double h0 = now_ms();
            SampleHasher h(s);
            uint64_t done = 0;
            while (done < bytes) {
                const uint64_t l = landed.load(std::memory_order_acquire);
                if (l == done) {
                    std::this_thread::yield();
                    continue;
                }
                h.update(static_cast<const uint8_t*>(out) + done, (l - done) / esz);
                done = l;
            }
            ok = h.matches(s.si.md5);
            t_md5 = now_ms() - h0;
        });
        hipError_t e = hipSuccess;
        for (uint64_t off = 0; off < bytes; off += CHUNK) {
            const uint64_t len = std::min(CHUNK, bytes - off);
            if (e == hipSuccess)
                e = hipMemcpy(static_cast<uint8_t*>(out) + off, static_cast<const uint8_t*>(s.dev_samples) + off, len,
                              hipMemcpyDeviceToHost);
            landed.store(off + len, std::memory_order_release);  // on failure: drain the hasher
        }
        hasher.join();
        ck(e);
    }
    b->timings.read_ms = now_ms() - t0;
    b->timings.host_md5_ms = t_md5;
    return ok ? E_OK : E_INVALID_CHECKSUM;
}

// k_md5 job of stream s over `n` samples at `data` (device), as zflac hashes them.
Md5Job md5_job(const StreamState& s, const void* data, uint64_t n, const uint32_t* status) {
    Md5Job j{};
    j.data = static_cast<const uint8_t*>(data);
    j.n = n;
    j.status = status;
    const uint32_t js = justify_of(s.si.bps);
    j.js = js;
    if (s.kind == 0) {
        j.mode = MD5_RAW, j.width = 1;
    } else if (s.kind == 1) {
        j.mode = js ? MD5_S16_SHIFT : MD5_RAW, j.width = 2;
    } else if ((s.si.bps + 7) / 8 * 8 == 24) {
        j.mode = MD5_S24, j.width = 3;
    } else {
        j.mode = js ? MD5_S32_SHIFT : MD5_RAW, j.width = 4;
    }
    return j;
}

// The Md5Mode all `jobs` share when every one's samples are 16-byte aligned: k_md5_coop
// (cooperative loads) can hash them; else -1 (k_md5, each lane its own loads).
int coop_mode_of(const std::vector<Md5Job>& jobs) {
    if (jobs.empty() || std::getenv("ZFLAC_MD5_LANE_LOADS")) return -1;
    for (const Md5Job& j : jobs)
        if (j.mode != jobs[0].mode || (reinterpret_cast<uintptr_t>(j.data) & 15) != 0) return -1;
    return (int)jobs[0].mode;
}

// Order of `jobs` longest message first: the lanes of a wave then run chains of similar length.
std::vector<uint32_t> longest_first(const std::vector<Md5Job>& jobs) {
    std::vector<uint32_t> ord(jobs.size());
    for (uint32_t k = 0; k < ord.size(); k++) ord[k] = k;
    std::stable_sort(ord.begin(), ord.end(), [&](uint32_t x, uint32_t y) {
        return jobs[x].n * jobs[x].width > jobs[y].n * jobs[y].width;
    });
    return ord;
}

// Digest words (k_md5 layout) -> the stream's verdict; a mismatch becomes its error, as
// decode() returns InvalidChecksum (src/zflac.zig:279-280).
void take_digest(StreamState& s, const uint32_t* d) {
    for (int w = 0; w < 4; w++)
        for (int q = 0; q < 4; q++) s.md5_dig[4 * w + q] = (uint8_t)(d[w] >> (8 * q));
    s.md5_dev = std::memcmp(s.md5_dig, s.si.md5, 16) == 0 ? 1 : 2;
    if (s.md5_dev == 2) s.err = E_INVALID_CHECKSUM;
}

// ZFLAC_FLAG_DEVICE_MD5 at batch creation: one k_md5 job per stream the parallel pass can
// certify (STREAMINFO total known), over its region of the class output, gated on the run's
// k_verify status; submit enqueues them behind the run (pipelined: the hash of one batch runs
// beside the decode of the others in flight).
void plan_md5_pipeline(zflac_batch* b) {
    std::vector<Md5Job> jobs;
    std::vector<uint32_t> who;
    for (auto& cp : b->classes) {
        Class& C = *cp;
        const int esz = esz_of_kind(C.kind);
        for (size_t m = 0; m < C.members.size(); m++) {
            const StreamDesc& D = C.desc[m];
            if (!D.valid_total) continue;
            jobs.push_back(md5_job(b->streams[C.members[m]], C.out.p + D.out_base * esz, D.total, C.status + m));
            who.push_back(C.members[m]);
        }
    }
    if (jobs.empty()) return;
    const std::vector<uint32_t> ord = longest_first(jobs);
    std::vector<Md5Job> sorted(jobs.size());
    b->pipe_who.resize(jobs.size());
    for (size_t k = 0; k < ord.size(); k++) {
        sorted[k] = jobs[ord[k]];
        b->pipe_who[k] = who[ord[k]];
    }
    b->pipe_coop = coop_mode_of(sorted);
    b->pipe_jobs.alloc(sorted.size());
    b->pipe_dig.alloc(sorted.size() * 4);
    ck(hipMemcpy(b->pipe_jobs.p, sorted.data(), sorted.size() * sizeof(Md5Job), hipMemcpyHostToDevice));
    ck(hipHostMalloc(reinterpret_cast<void**>(&b->pipe_pin), sorted.size() * 16, hipHostMallocDefault));
}

// STREAMINFO MD5 of the streams `which` on the device (k_md5, one lane per stream),
// synchronously: the streams the pipelined hash could not cover (decoded by the sequential
// planner, or re-run after a candidate-table regrowth).
void run_md5_device(zflac_batch* b, const std::vector<uint32_t>& which, bool timing) {
    std::vector<Md5Job> jobs;
    for (uint32_t i : which) {
        const StreamState& s = b->streams[i];
        jobs.push_back(md5_job(s, s.dev_samples, s.info.n_samples, nullptr));
    }
    if (jobs.empty()) return;
    const std::vector<uint32_t> ord = longest_first(jobs);
    std::vector<Md5Job> sorted(jobs.size());
    for (size_t k = 0; k < ord.size(); k++) sorted[k] = jobs[ord[k]];
    b->md5_jobs.alloc(sorted.size());
    b->md5_dig.alloc(sorted.size() * 4);
    ck(hipMemcpyAsync(b->md5_jobs.p, sorted.data(), sorted.size() * sizeof(Md5Job), hipMemcpyHostToDevice,
                      b->stream));
    if (timing) ck(hipEventRecord(b->ev[5], b->stream));
    ck(launch_md5(b->md5_jobs.p, (uint32_t)sorted.size(), b->md5_dig.p, b->stream, coop_mode_of(sorted)));
    if (timing) ck(hipEventRecord(b->ev[6], b->stream));
    std::vector<uint32_t> dig(sorted.size() * 4);
    ck(hipMemcpyAsync(dig.data(), b->md5_dig.p, dig.size() * 4, hipMemcpyDeviceToHost, b->stream));
    ck(hipStreamSynchronize(b->stream));
    if (timing) {
        float t = 0;
        ck(hipEventElapsedTime(&t, b->ev[5], b->ev[6]));
        b->timings.md5_ms += t;
    }
    for (size_t k = 0; k < ord.size(); k++) take_digest(b->streams[which[ord[k]]], &dig[k * 4]);
}

// After a run: the pipelined digests of the streams the run certified, then a synchronous
// k_md5 for every other decoded stream.
void finish_md5(zflac_batch* b, bool timing) {
    std::vector<char> done(b->streams.size(), 0);
    for (auto& s : b->streams) s.md5_dev = 0;
    if (!b->pipe_who.empty()) {
        if (timing) {
            float t = 0;
            ck(hipEventElapsedTime(&t, b->ev[8], b->ev[9]));
            b->timings.md5_ms = t;
        }
        for (size_t k = 0; k < b->pipe_who.size(); k++) {
            const uint32_t i = b->pipe_who[k];
            StreamState& s = b->streams[i];
            const Class& C = *b->classes[s.cls];
            if (s.err || !s.dev_samples || C.redone || C.h_status[s.slot] != 0 || (b->flags & ZFLAC_FLAG_FORCE_SLOW))
                continue;
            take_digest(s, b->pipe_pin + k * 4);
            done[i] = 1;
        }
    }
    std::vector<uint32_t> rest;
    for (uint32_t i = 0; i < b->streams.size(); i++)
        if (!done[i] && !b->streams[i].err && b->streams[i].dev_samples) rest.push_back(i);
    run_md5_device(b, rest, timing);
}

int create_batch(const zflac_stream* streams, size_t n, int device, int flags, zflac_batch** out) {
    if (!out || (n && !streams)) return E_INVALID_ARGUMENT;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0 || device < 0 || device >= ndev) return E_DEVICE;
    std::unique_ptr<zflac_batch> b(new (std::nothrow) zflac_batch());
    if (!b) return E_OUT_OF_MEMORY;
    b->device = device;
    b->flags = flags;
    try {
        ck(hipSetDevice(device));
        (void)device_streams(device);  // the run and md5 hub streams first (their own hardware queues)
        ck(hipStreamCreateWithFlags(&b->stream, hipStreamNonBlocking));
        b->rs = b->stream;
        if (const char* fp = std::getenv("ZFLAC_FRONT_PRIORITY"); fp && fp[0] == '1') {
            int least = 0, greatest = 0;
            ck(hipDeviceGetStreamPriorityRange(&least, &greatest));
            ck(hipStreamCreateWithPriority(&b->front, hipStreamNonBlocking, greatest));
            ck(hipEventCreateWithFlags(&b->front_join, hipEventDisableTiming));
        }
        // timing-only events: no system-scope fence (cache writeback + invalidate) at each
        // record, which would otherwise slow the kernel after it
        for (auto& e : b->ev) ck(hipEventCreateWithFlags(&e, hipEventDisableSystemFence));
        ck(hipEventCreateWithFlags(&b->ev_done, hipEventDisableTiming));
        ck(hipEventCreateWithFlags(&b->ev_md5, hipEventDisableTiming));
        const double t0 = now_ms();
        b->streams.resize(n);
        for (size_t i = 0; i < n; i++) {
            if (!streams[i].data && streams[i].len) return E_INVALID_ARGUMENT;
            plan_stream(b->streams[i], streams[i].data, streams[i].len);
        }
        const double t1 = now_ms();
        b->timings.plan_ms = t1 - t0;
        for (size_t i = 0; i < n; i++) {
            StreamState& s = b->streams[i];
            if (s.host_err || s.no_frames) continue;
            int ci = -1;
            for (size_t k = 0; k < b->classes.size(); k++)
                if (b->classes[k]->kind == s.kind && b->classes[k]->nch == s.nch) ci = (int)k;
            if (ci < 0) {
                b->classes.emplace_back(new Class());
                b->classes.back()->kind = s.kind;
                b->classes.back()->nch = s.nch;
                ci = (int)b->classes.size() - 1;
            }
            s.cls = ci;
            b->classes[ci]->members.push_back((uint32_t)i);
        }
        for (auto& C : b->classes) alloc_class(b.get(), *C, streams);
        if (flags & ZFLAC_FLAG_DEVICE_MD5) plan_md5_pipeline(b.get());
        b->timings.upload_ms = now_ms() - t1;
        // streams resolved on the host
        for (auto& s : b->streams) {
            if (s.host_err) s.err = s.host_err;
            if (s.no_frames) {
                s.err = 0;
                s.info = zflac_info{};
                s.info.sample_kind = (uint8_t)s.kind;
            }
        }
    } catch (const DeviceError&) {
        return E_DEVICE;
    } catch (const std::bad_alloc&) {
        return E_OUT_OF_MEMORY;
    } catch (const std::exception&) {  // e.g. std::system_error from an upload helper thread
        return E_DEVICE;
    }
    *out = b.release();
    return E_OK;
}

}  // namespace

void hub_release_ext(zflac_batch* b) { hub_release(b); }
void hub_forget_ext(zflac_batch* b) { hub_forget(b); }
}  // namespace zflac

// ---------------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------------
using namespace zflac;

extern "C" {

const char* zflac_hip_error_name(int code) {
    switch (code) {
        case 0: return "OK";
        case 1: return "InvalidSignature";
        case 2: return "InvalidMetadataHeader";
        case 3: return "MissingStreaminfo";
        case 4: return "Unimplemented";
        case 5: return "InvalidChecksum";
        case 6: return "InvalidFrameHeader";
        case 7: return "InconsistentParameters";
        case 8: return "InvalidCodedNumber";
        case 9: return "InvalidSubframeHeader";
        case 10: return "InvalidResidualCodingMethod";
        case 11: return "EndOfStream";
        case 12: return "OutOfMemory";
        case 13: return "DeviceError";
        case 14: return "InvalidArgument";
        case 15: return "OutOfDomain";
        case 16: return "FrameCrcMismatch";
        default: return "Unknown";
    }
}

int zflac_hip_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

const char* zflac_hip_version(void) { return "zflac_hip gfx950 r4"; }

#ifndef ZFLAC_BUILD_ID
#define ZFLAC_BUILD_ID "unknown"
#endif
const char* zflac_hip_build_id(void) { return ZFLAC_BUILD_ID; }

int zflac_hip_batch_create(const zflac_stream* streams, size_t n, int device, int flags, zflac_batch** out) {
    return create_batch(streams, n, device, flags, out);
}

// After a failed submit: the work already enqueued (on the batch stream and, with
// ZFLAC_FRONT_PRIORITY, the front stream) may still use the candidate buffers a retry
// reallocates.
static void drain_failed_submit(zflac_batch* b) {
    try {
        hub_forget(b);
    } catch (...) {
    }
    (void)hipStreamSynchronize(b->stream);
    if (b->rs) (void)hipStreamSynchronize(b->rs);
    if (b->front) (void)hipStreamSynchronize(b->front);
    b->rs = b->stream;
    b->submitted = false;
}

int zflac_hip_batch_submit(zflac_batch* b) {
    if (!b || b->submitted) return E_INVALID_ARGUMENT;
    b->ran = false;
    try {
        b->submit_t0 = now_ms();
        b->submitted = true;
        submit_batch(b);
    } catch (const DeviceError&) {
        drain_failed_submit(b);
        return E_DEVICE;
    } catch (const std::bad_alloc&) {
        drain_failed_submit(b);
        return E_OUT_OF_MEMORY;
    } catch (const std::exception&) {
        drain_failed_submit(b);
        return E_DEVICE;
    }
    return E_OK;
}

int zflac_hip_batch_wait(zflac_batch* b) {
    if (!b || !b->submitted) return E_INVALID_ARGUMENT;
    b->submitted = false;
    int rc = E_OK;
    try {
        finish_batch(b);
        b->timings.run_wall_ms = now_ms() - b->submit_t0;
        b->ran = true;
    } catch (const DeviceError&) {
        rc = E_DEVICE;
    } catch (const std::bad_alloc&) {
        rc = E_OUT_OF_MEMORY;
    } catch (const std::exception&) {
        rc = E_DEVICE;
    }
    if (rc != E_OK && b->md5_pending) {  // failed before the hub released this run
        try {
            hub_forget(b);
        } catch (...) {
        }
    }
    return rc;
}

int zflac_hip_batch_ready(zflac_batch* b) {
    if (!b || !b->submitted) return -E_INVALID_ARGUMENT;
    hipError_t e = hipEventQuery(b->ev_done);
    if (e == hipSuccess && b->md5_hub) {
        try {
            Md5Hub& h = md5_hub(b->device);
            std::lock_guard<std::mutex> lock(h.mu);
            if (b->md5_pending) {  // decoded, hash not launched: launch it if the hub is idle
                if (!h.any || hipEventQuery(h.last) == hipSuccess) hub_flush(h);
                return 0;
            }
            // the hub launch holding this run failed (possibly another thread's flush): ev_md5
            // was never recorded for this run, so it must not be queried
            if (b->md5_failed) return -E_DEVICE;
        } catch (const DeviceError&) {
            return -E_DEVICE;
        }
        e = hipEventQuery(b->ev_md5);
    }
    if (e == hipSuccess) return 1;
    if (e == hipErrorNotReady) return 0;
    return -E_DEVICE;
}

int zflac_hip_batch_run(zflac_batch* b) {
    const int rc = zflac_hip_batch_submit(b);
    return rc ? rc : zflac_hip_batch_wait(b);
}

size_t zflac_hip_batch_size(zflac_batch* b) { return b ? b->streams.size() : 0; }

int zflac_hip_batch_info(zflac_batch* b, size_t i, zflac_info* info) {
    if (!b || !b->ran || i >= b->streams.size()) return E_INVALID_ARGUMENT;
    const StreamState& s = b->streams[i];
    if (info) *info = s.info;
    return s.err;
}

const void* zflac_hip_batch_device_samples(zflac_batch* b, size_t i) {
    if (!b || !b->ran || i >= b->streams.size() || b->streams[i].err) return nullptr;
    return b->streams[i].dev_samples;
}

int zflac_hip_batch_read(zflac_batch* b, size_t i, void* out, size_t out_bytes, int verify_md5) {
    if (!b || !b->ran || i >= b->streams.size()) return E_INVALID_ARGUMENT;
    StreamState& s = b->streams[i];
    if (s.err) return s.err;
    if (out_bytes < s.info.samples_bytes || (!out && s.info.samples_bytes)) return E_INVALID_ARGUMENT;
    try {
        ck(hipSetDevice(b->device));
        // a device verdict stands in for the host hash (a mismatch is already s.err)
        return read_samples(b, s, out, verify_md5 && !s.md5_dev);  // InvalidChecksum at :279-280
    } catch (const DeviceError&) {
        return E_DEVICE;
    } catch (const std::exception&) {  // std::system_error: the hashing thread could not start
        return E_DEVICE;
    }
}

int zflac_hip_batch_md5(zflac_batch* b, size_t i, uint8_t* digest) {
    if (!b || !b->ran || i >= b->streams.size() || !digest) return E_INVALID_ARGUMENT;
    const StreamState& s = b->streams[i];
    if (!s.md5_dev) return E_INVALID_ARGUMENT;
    std::memcpy(digest, s.md5_dig, 16);
    return E_OK;
}

int zflac_hip_batch_timings(zflac_batch* b, zflac_timings* t) {
    return zflac_hip_batch_timings_ex(b, t, ZFLAC_TIMINGS_V1_SIZE);
}

int zflac_hip_batch_timings_ex(zflac_batch* b, zflac_timings* t, size_t size) {
    if (!b || !t || size == 0) return E_INVALID_ARGUMENT;
    // the caller's struct may be older (shorter) or newer (longer) than this library's
    std::memcpy(t, &b->timings, std::min(size, sizeof(zflac_timings)));
    if (size > sizeof(zflac_timings)) std::memset(reinterpret_cast<uint8_t*>(t) + sizeof(zflac_timings), 0,
                                                  size - sizeof(zflac_timings));
    return b->have_timing ? E_OK : E_INVALID_ARGUMENT;  // the host wall-clock fields are always filled
}

int zflac_hip_abi_version(void) { return ZFLAC_HIP_ABI_VERSION; }

#ifdef ZFLAC_PROBE
// Timing-probe build only (tools/probe.sh): cycle counters the decode kernels accumulate
// behind the dummy store region of the first class; zeroed after reading.
extern "C" int zflac_hip_probe(zflac_batch* b, unsigned long long* out, int n) {
    if (!b || b->classes.empty() || n > (int)(PROBE_BYTES / 8)) return E_INVALID_ARGUMENT;
    auto& C = *b->classes[0];
    uint8_t* p = reinterpret_cast<uint8_t*>(C.dummy.p) + DUMMY_BYTES;
    if (hipMemcpy(out, p, n * 8, hipMemcpyDeviceToHost) != hipSuccess) return E_DEVICE;
    if (hipMemset(p, 0, PROBE_BYTES) != hipSuccess) return E_DEVICE;
    return E_OK;
}
#endif

#ifdef ZFLAC_REPLAY
// Diagnostic build only (tools/replay.py): re-enqueue parts of each batch's last run `reps`
// times, batch i on its own run stream, with no host work in between, and return the wall
// time: what = 1 walk, 2 decode, 3 walk + decode, 4 the whole run (enqueue_class: fills, scan,
// compact, walk, decode, verify, read-backs). Separates the device's throughput for each part
// from the host side of submit / wait. Outputs are rewritten with the same values.
extern "C" int zflac_hip_replay(zflac_batch** bs, int nb, int reps, int what, double* ms) {
    try {
        if (nb <= 0 || !bs || !ms) return E_INVALID_ARGUMENT;
        ck(hipSetDevice(bs[0]->device));
        for (int i = 0; i < nb; i++) {  // one run stream (hardware queue) per batch, as submit
            ck(hipStreamSynchronize(bs[i]->rs));
            bs[i]->rs = next_run_stream(bs[i]->device);
        }
        const double t0 = now_ms();
        for (int r = 0; r < reps; r++) {
            for (int i = 0; i < nb; i++) {
                zflac_batch* b = bs[i];
                Class& C = *b->classes[0];
                if (what == 4) {
                    enqueue_class(b, C, false, false);
                    continue;
                }
                if (what >= 8) {  // the front alone: 8 k_scan, 16 k_scan + k_scan_chunks + k_compact
                    ScanArgs sa{};
                    sa.in = C.in.p;
                    sa.streams = C.d_desc.p;
                    sa.chunks = C.d_chunks.p;
                    sa.n_chunks = (uint32_t)C.chunks.size();
                    sa.chunk_cnt = C.chunk_cnt.p;
                    sa.chunk_units = C.chunk_units.p;
                    sa.chunk_slots = C.chunk_slots.p;
                    sa.chunk_slot_units = C.chunk_slot_units.p;
                    sa.status = C.status;
                    sa.n_status = (uint32_t)C.members.size();
                    sa.misc = C.misc.p;
                    ck(launch_scan(sa, b->rs));
                    if (what == 16) {
                        ck(launch_scan_chunks(C.chunk_cnt.p, C.chunk_units.p, sa.n_chunks, C.chunk_off.p,
                                              C.chunk_uoff.p, C.misc.p, b->rs));
                        CompactArgs ca{};
                        ca.in = C.in.p;
                        ca.streams = C.d_desc.p;
                        ca.chunks = C.d_chunks.p;
                        ca.n_chunks = sa.n_chunks;
                        ca.chunk_cnt = C.chunk_cnt.p;
                        ca.chunk_slots = C.chunk_slots.p;
                        ca.chunk_slot_units = C.chunk_slot_units.p;
                        ca.chunk_off = C.chunk_off.p;
                        ca.chunk_uoff = C.chunk_uoff.p;
                        ca.cap = C.cap;
                        ca.c_pos = C.c_pos.p;
                        ca.c_stream = C.c_stream.p;
                        ca.c_out = C.c_out.p;
                        ca.overflow = C.misc.p + 1;
                        ck(launch_compact(ca, b->rs));
                    }
                    continue;
                }
                DecodeArgs da = decode_args(C);
                da.full_mask = C.full_mask;
                const uint32_t mf = std::min(C.grid_frames, C.cap);
                if (what & 1) ck(launch_walk_k1(da, mf, b->rs));
                if (what & 2) ck(launch_decode_k1_stereo(da, mf, b->rs));
            }
        }
        for (int i = 0; i < nb; i++) ck(hipStreamSynchronize(bs[i]->rs));
        *ms = now_ms() - t0;
        for (int i = 0; i < nb; i++) bs[i]->rs = bs[i]->stream;
        return E_OK;
    } catch (const DeviceError&) {
        return E_DEVICE;
    }
}
#endif

void zflac_hip_batch_destroy(zflac_batch* b) {
    if (!b) return;
    (void)hipSetDevice(b->device);
    delete b;
}

int zflac_hip_open(const uint8_t* buf, size_t len, int device, zflac_batch** out_batch, zflac_info* info) {
    return zflac_hip_open_ex(buf, len, device, 0, out_batch, info);
}

int zflac_hip_open_ex(const uint8_t* buf, size_t len, int device, int flags, zflac_batch** out_batch,
                      zflac_info* info) {
    if (!out_batch) return E_INVALID_ARGUMENT;
    zflac_stream s{buf, len};
    int rc = create_batch(&s, 1, device, flags, out_batch);
    if (rc) return rc;
    rc = zflac_hip_batch_run(*out_batch);
    if (rc) return rc;
    return zflac_hip_batch_info(*out_batch, 0, info);
}

int zflac_hip_read(zflac_batch* b, void* out_samples, size_t out_bytes) {
    return zflac_hip_batch_read(b, 0, out_samples, out_bytes, 1);
}

void zflac_hip_close(zflac_batch* b) { zflac_hip_batch_destroy(b); }

}  // extern "C"
