// calib_pmc.hip -- calibrates rocprofv3 FETCH_SIZE / WRITE_SIZE against known byte counts
// for the access pattern of k_decode: every lane streams its OWN byte range (one FLAC
// subframe per lane), reading two 16-byte quads per top-up and storing 16-byte packed PCM
// quads into its own output range. Lanes of a wave are therefore not coalesced with each
// other; the guide's x2 correction is stated only for coalesced streaming reads.
//
// Usage: calib_pmc  (prints the byte counts; run under rocprofv3 --pmc FETCH_SIZE, then
// --pmc WRITE_SIZE, and divide the per-dispatch counter by these counts)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr uint64_t LANE_BYTES = 64 * 1024;   // like a 4096-sample 16-bit subframe (~8-10 KiB) x 6
constexpr int THREADS = 256;
constexpr int LANES = 1250 * 64;             // enough lanes to exceed the 256 MiB Infinity Cache

__global__ __launch_bounds__(THREADS) void k_read_private(const uint4* __restrict__ in, uint32_t* __restrict__ sink) {
    const uint32_t lane = blockIdx.x * THREADS + threadIdx.x;
    const uint4* p = in + (uint64_t)lane * (LANE_BYTES / 16);
    uint32_t acc = 0;
    for (uint32_t q = 0; q < LANE_BYTES / 16; q += 2) {
        const uint4 a = p[q], b = p[q + 1];
        acc ^= a.x + a.y * 3 + a.z * 5 + a.w * 7 + b.x * 11 + b.y * 13 + b.z * 17 + b.w * 19;
    }
    if (acc == 0x12345678u) sink[lane] = acc;  // keeps the loads alive, never true for zero-filled input
}

__global__ __launch_bounds__(THREADS) void k_write_private(uint4* __restrict__ out) {
    const uint32_t lane = blockIdx.x * THREADS + threadIdx.x;
    uint4* p = out + (uint64_t)lane * (LANE_BYTES / 16);
    for (uint32_t q = 0; q < LANE_BYTES / 16; q++) p[q] = make_uint4(lane, q, lane ^ q, 7);
}

// The staged write-back of k_decode's stereo fast path: every group of 8 lanes stores one
// frame's 128 contiguous bytes per chunk (lane L: 16 B at run + (L & 7) * 16), frames far
// apart (one region per lane group, like one output region per frame).
__global__ __launch_bounds__(THREADS) void k_write_runs(uint4* __restrict__ out) {
    const uint32_t lane = blockIdx.x * THREADS + threadIdx.x;
    const uint32_t group = lane >> 3, piece = lane & 7;
    uint4* p = out + (uint64_t)group * (8 * LANE_BYTES / 16) + piece;
    for (uint32_t q = 0; q < 8 * LANE_BYTES / 16; q += 8) p[q] = make_uint4(lane, q, lane ^ q, 7);
}

__global__ __launch_bounds__(THREADS) void k_read_coalesced(const uint4* __restrict__ in, uint32_t* __restrict__ sink,
                                                            uint64_t nq) {
    uint32_t acc = 0;
    for (uint64_t q = blockIdx.x * THREADS + threadIdx.x; q < nq; q += (uint64_t)gridDim.x * THREADS) {
        const uint4 a = in[q];
        acc ^= a.x + a.y * 3 + a.z * 5 + a.w * 7;
    }
    if (acc == 0x12345678u) sink[threadIdx.x] = acc;
}

#define CK(x)                                                                         \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(e_));            \
            return 1;                                                                 \
        }                                                                             \
    } while (0)

int main() {
    const uint64_t bytes = LANE_BYTES * LANES;  // 5.2 GB
    uint4* buf = nullptr;
    uint32_t* sink = nullptr;
    CK(hipMalloc(&buf, bytes));
    CK(hipMalloc(&sink, LANES * 4));
    CK(hipMemset(buf, 0, bytes));
    const int blocks = LANES / THREADS;
    for (int it = 0; it < 3; it++) {
        k_read_private<<<blocks, THREADS>>>(buf, sink);
        k_write_private<<<blocks, THREADS>>>(buf);
        k_write_runs<<<blocks, THREADS>>>(buf);
        k_read_coalesced<<<4096, THREADS>>>(buf, sink, bytes / 16);
    }
    CK(hipDeviceSynchronize());
    printf("{\"read_private_bytes\": %llu, \"write_private_bytes\": %llu, \"write_runs_bytes\": %llu, "
           "\"read_coalesced_bytes\": %llu}\n",
           (unsigned long long)bytes, (unsigned long long)bytes, (unsigned long long)bytes, (unsigned long long)bytes);
    CK(hipFree(buf));
    CK(hipFree(sink));
    return 0;
}
