// tools/ubench_read.hip -- read-bandwidth floor of k_scan's access pattern (diagnostic).
// Reads N bytes with workgroups of 256 threads, each thread R x 16 B (buffer loads, all in
// flight), XOR-reduces them (so the loads cannot be dropped), one word out per workgroup.
// Variants: R = 4, 8, 16 per thread (chunk = 256 * 16 * R bytes), and a grid-stride form.
// Prints GB/s per variant (hipEvent, median of 20 launches).
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

template <int R>
__global__ __launch_bounds__(256) void k_chunk(const uint8_t* in, uint64_t n, uint32_t* out) {
    const uint64_t base = (uint64_t)blockIdx.x * 256 * 16 * R;
    const uint64_t len = n - base < 256ull * 16 * R ? n - base : 256ull * 16 * R;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(in) + base, (short)0, (int)len, 0x00020000);
    uint4 v[R];
#pragma unroll
    for (int r = 0; r < R; r++)
        v[r] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, threadIdx.x * 16u, r * 256 * 16, 0));
    uint32_t x = 0;
#pragma unroll
    for (int r = 0; r < R; r++) x ^= v[r].x ^ v[r].y ^ v[r].z ^ v[r].w;
    if (__builtin_amdgcn_ballot_w64(x == 0x12345678u)) out[blockIdx.x] = x;  // practically never stored
}

// persistent grid-stride: each workgroup walks chunks blockIdx, blockIdx + grid, ...
template <int R>
__global__ __launch_bounds__(256) void k_stride(const uint8_t* in, uint64_t n, uint32_t nchunks, uint32_t* out) {
    uint32_t x = 0;
    for (uint32_t c = blockIdx.x; c < nchunks; c += gridDim.x) {
        const uint64_t base = (uint64_t)c * 256 * 16 * R;
        const uint64_t len = n - base < 256ull * 16 * R ? n - base : 256ull * 16 * R;
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(in) + base, (short)0, (int)len, 0x00020000);
        uint4 v[R];
#pragma unroll
        for (int r = 0; r < R; r++)
            v[r] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, threadIdx.x * 16u, r * 256 * 16, 0));
#pragma unroll
        for (int r = 0; r < R; r++) x ^= v[r].x ^ v[r].y ^ v[r].z ^ v[r].w;
    }
    if (__builtin_amdgcn_ballot_w64(x == 0x12345678u)) out[blockIdx.x] = x;
}

template <typename F>
float timeit(F&& launch) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    std::vector<float> ts;
    for (int i = 0; i < 25; i++) {
        (void)hipEventRecord(a, 0);
        launch();
        (void)hipEventRecord(b, 0);
        (void)hipEventSynchronize(b);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, a, b);
        if (i >= 5) ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    return ts[ts.size() / 2];
}

int main() {
    const uint64_t n = 358ull << 20;
    uint8_t* in;
    uint32_t* out;
    CK(hipMalloc(&in, n + 65536));
    CK(hipMalloc(&out, 1 << 22));
    CK(hipMemset(in, 0x5a, n + 65536));
    CK(hipDeviceSynchronize());
    auto run_chunk = [&](auto rc) {
        constexpr int R = decltype(rc)::value;
        const uint32_t blocks = (uint32_t)((n + 256ull * 16 * R - 1) / (256ull * 16 * R));
        float ms = timeit([&] { hipLaunchKernelGGL(k_chunk<R>, dim3(blocks), dim3(256), 0, 0, in, n, out); });
        printf("{\"kind\": \"chunk\", \"R\": %d, \"blocks\": %u, \"ms\": %.4f, \"GBs\": %.1f}\n", R, blocks, ms, n / (ms * 1e-3) / 1e9);
    };
    run_chunk(std::integral_constant<int, 4>{});
    run_chunk(std::integral_constant<int, 8>{});
    run_chunk(std::integral_constant<int, 16>{});
    for (uint32_t grid : {1024u, 2048u, 4096u}) {
        constexpr int R = 8;
        const uint32_t nch = (uint32_t)((n + 256ull * 16 * R - 1) / (256ull * 16 * R));
        float ms = timeit([&] { hipLaunchKernelGGL(k_stride<R>, dim3(grid), dim3(256), 0, 0, in, n, nch, out); });
        printf("{\"kind\": \"stride\", \"R\": %d, \"grid\": %u, \"ms\": %.4f, \"GBs\": %.1f}\n", R, grid, ms, n / (ms * 1e-3) / 1e9);
    }
    return 0;
}
