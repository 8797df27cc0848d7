// ubench_lat.hip -- dependent-issue latency of the VALU ops on the decode loop's critical
// path (one wave per SIMD, one dependency chain), and an LDS read -> use chain, on gfx950.
// Output: cycles per dependent op (s_memtime, shader clock).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr int ITER = 4096;

#define LAT_KERNEL(NAME, ASM)                                                                 \
    __global__ __launch_bounds__(64) void NAME(uint32_t* out, uint64_t* cyc, uint32_t seed) { \
        uint32_t a = seed ^ threadIdx.x;                                                    \
        const uint32_t b = seed | 1, c = (seed >> 3) | 5;                                   \
        const uint64_t t0 = __builtin_amdgcn_s_memtime();                                   \
        for (int i = 0; i < ITER; i++) {                                                    \
            asm volatile(ASM "\n\t" ASM "\n\t" ASM "\n\t" ASM : "+v"(a) : "v"(b), "v"(c));   \
        }                                                                                   \
        const uint64_t t1 = __builtin_amdgcn_s_memtime();                                   \
        out[blockIdx.x * 64 + threadIdx.x] = a;                                             \
        if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;                                    \
    }

LAT_KERNEL(l_add, "v_add_u32 %0, %0, %1")
LAT_KERNEL(l_alignbit, "v_alignbit_b32 %0, %0, %1, %2")
LAT_KERNEL(l_ffbh, "v_ffbh_u32 %0, %0")
LAT_KERNEL(l_add3, "v_add3_u32 %0, %0, %1, %2")
LAT_KERNEL(l_cndmask, "v_cmp_gt_u32 vcc, %0, %1\n\tv_cndmask_b32 %0, %0, %2, vcc")
LAT_KERNEL(l_dot2c, "v_dot2c_i32_i16 %0, %1, %0")

__shared__ uint32_t g_lds[64 * 64];
__global__ __launch_bounds__(64) void l_lds(uint32_t* out, uint64_t* cyc, uint32_t seed) {
    for (int i = 0; i < 64; i++) g_lds[i * 64 + threadIdx.x] = ((threadIdx.x + i + 1) & 63) * 256 + threadIdx.x * 4;
    __syncthreads();
    uint32_t a = threadIdx.x * 4;
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < ITER; i++) {
        asm volatile("ds_read_b32 %0, %0\n\ts_waitcnt lgkmcnt(0)" : "+v"(a));
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * 64 + threadIdx.x] = a;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

typedef void (*KFn)(uint32_t*, uint64_t*, uint32_t);
int main() {
    struct K { const char* name; KFn f; int ops; };
    K ks[] = {{"v_add_u32", l_add, 4}, {"v_alignbit_b32", l_alignbit, 4}, {"v_ffbh_u32", l_ffbh, 4},
              {"v_add3_u32", l_add3, 4}, {"v_cmp+v_cndmask", l_cndmask, 8}, {"v_dot2c_i32_i16", l_dot2c, 4},
              {"ds_read_b32+wait", l_lds, 1}};
    uint32_t* out;
    uint64_t* cyc;
    (void)hipMalloc(&out, 1024 * 64 * 4);
    (void)hipMalloc(&cyc, 1024 * 8);
    uint64_t h[1024];
    printf("{\"iter\": %d, \"results\": [\n", ITER);
    for (int i = 0; i < 7; i++) {
        for (int waves : {1, 1024}) {  // one wave on the chip / one wave per SIMD everywhere
            ks[i].f<<<waves, 64>>>(out, cyc, 99);
            ks[i].f<<<waves, 64>>>(out, cyc, 7);
            (void)hipDeviceSynchronize();
            (void)hipMemcpy(h, cyc, waves * 8, hipMemcpyDeviceToHost);
            double s = 0;
            for (int w = 0; w < waves; w++) s += (double)h[w];
            s /= waves;
            printf("%s{\"op\": \"%s\", \"waves\": %d, \"cyc_per_dep_op\": %.2f}", (i || waves > 1) ? ",\n" : "",
                   ks[i].name, waves, s / ((double)ITER * ks[i].ops));
        }
    }
    printf("\n]}\n");
    return 0;
}
