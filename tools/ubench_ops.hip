// ubench_ops.hip -- issue cost of the integer VALU ops the decode loop is made of, on
// gfx950, with 1, 2 and 4 waves per SIMD. Each kernel runs 8 independent chains of one op
// (inline asm so the compiler keeps exactly that instruction), ITER x 8 ops per lane.
// Output: cycles per wave-instruction per SIMD, from s_memtime around the loop (shader
// clock) and from wall time with the clock from s_memtime / s_memrealtime.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

constexpr int ITER = 4096;

#define OP_KERNEL(NAME, ASM)                                                                      \
    __global__ __launch_bounds__(64) void NAME(uint32_t* out, uint64_t* cyc, uint32_t seed) {     \
        uint32_t a0 = seed ^ threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 * 11,  \
                 a5 = a0 * 13, a6 = a0 * 17, a7 = a0 * 19;                                      \
        const uint32_t b = seed | 1, c = (seed >> 3) | 5;                                       \
        const uint64_t t0 = __builtin_amdgcn_s_memtime();                                       \
        const uint64_t r0 = __builtin_amdgcn_s_memrealtime();                                   \
        for (int i = 0; i < ITER; i++) {                                                        \
            asm volatile(ASM : "+v"(a0) : "v"(b), "v"(c));                                      \
            asm volatile(ASM : "+v"(a1) : "v"(b), "v"(c));                                      \
            asm volatile(ASM : "+v"(a2) : "v"(b), "v"(c));                                      \
            asm volatile(ASM : "+v"(a3) : "v"(b), "v"(c));                                      \
            asm volatile(ASM : "+v"(a4) : "v"(b), "v"(c));                                      \
            asm volatile(ASM : "+v"(a5) : "v"(b), "v"(c));                                      \
            asm volatile(ASM : "+v"(a6) : "v"(b), "v"(c));                                      \
            asm volatile(ASM : "+v"(a7) : "v"(b), "v"(c));                                      \
        }                                                                                       \
        const uint64_t t1 = __builtin_amdgcn_s_memtime();                                       \
        const uint64_t r1 = __builtin_amdgcn_s_memrealtime();                                   \
        out[blockIdx.x * 64 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;             \
        if (threadIdx.x == 0) {                                                                 \
            cyc[2 * blockIdx.x] = t1 - t0;                                                      \
            cyc[2 * blockIdx.x + 1] = r1 - r0;                                                  \
        }                                                                                       \
    }

OP_KERNEL(k_add, "v_add_u32 %0, %0, %1")
OP_KERNEL(k_and, "v_and_b32 %0, %0, %1")
OP_KERNEL(k_cndmask, "v_cmp_gt_u32 vcc, %0, %1\n\tv_cndmask_b32 %0, %0, %2, vcc")
OP_KERNEL(k_alignbit, "v_alignbit_b32 %0, %0, %1, %2")
OP_KERNEL(k_bfe, "v_bfe_u32 %0, %0, %1, %2")
OP_KERNEL(k_ffbh, "v_ffbh_u32 %0, %0")
OP_KERNEL(k_perm, "v_perm_b32 %0, %0, %1, %2")
OP_KERNEL(k_lshl_or, "v_lshl_or_b32 %0, %0, %1, %2")
OP_KERNEL(k_xad, "v_xad_u32 %0, %0, %1, %2")
OP_KERNEL(k_dot2c, "v_dot2c_i32_i16 %0, %1, %2")
OP_KERNEL(k_pk_add, "v_pk_add_u16 %0, %0, %1")
OP_KERNEL(k_mul_lo, "v_mul_lo_u32 %0, %0, %1")
OP_KERNEL(k_ashr, "v_ashrrev_i32 %0, %1, %0")
OP_KERNEL(k_permlane32, "v_permlane32_swap_b32 %0, %1")

// 64-bit accumulator chains (the 32-bit-container LPC: i64 MACs, or exact f64 FMAs)
#define OP_KERNEL64(NAME, T, ASM, CLOB)                                                           \
    __global__ __launch_bounds__(64) void NAME(uint32_t* out, uint64_t* cyc, uint32_t seed) {     \
        T a[8];                                                                                 \
        for (int j = 0; j < 8; j++) a[j] = (T)(seed ^ (threadIdx.x * (j + 3)));                \
        const uint32_t bi = seed | 1, ci = (seed >> 3) | 5;                                     \
        const T bd = (T)bi, cd = (T)ci;                                                         \
        (void)bd; (void)cd;                                                                     \
        const uint64_t t0 = __builtin_amdgcn_s_memtime();                                       \
        const uint64_t r0 = __builtin_amdgcn_s_memrealtime();                                   \
        for (int i = 0; i < ITER; i++) {                                                        \
            for (int j = 0; j < 8; j++) asm volatile(ASM : "+v"(a[j]) : "v"(bi), "v"(ci), "v"(bd), "v"(cd) CLOB); \
        }                                                                                       \
        const uint64_t t1 = __builtin_amdgcn_s_memtime();                                       \
        const uint64_t r1 = __builtin_amdgcn_s_memrealtime();                                   \
        uint64_t x = 0;                                                                         \
        for (int j = 0; j < 8; j++) x ^= (uint64_t)a[j];                                        \
        out[blockIdx.x * 64 + threadIdx.x] = (uint32_t)x;                                       \
        if (threadIdx.x == 0) {                                                                 \
            cyc[2 * blockIdx.x] = t1 - t0;                                                      \
            cyc[2 * blockIdx.x + 1] = r1 - r0;                                                  \
        }                                                                                       \
    }
OP_KERNEL64(k_mad_i64, uint64_t, "v_mad_i64_i32 %0, vcc, %1, %2, %0", : "vcc")
OP_KERNEL64(k_fma_f64, double, "v_fma_f64 %0, %3, %4, %0", )

typedef void (*KFn)(uint32_t*, uint64_t*, uint32_t);

int main() {
    struct K { const char* name; KFn f; int ops_per_asm; };
    std::vector<K> ks = {{"v_add_u32", k_add, 1},       {"v_and_b32", k_and, 1},
                         {"v_cmp+v_cndmask", k_cndmask, 2}, {"v_alignbit_b32", k_alignbit, 1},
                         {"v_bfe_u32", k_bfe, 1},       {"v_ffbh_u32", k_ffbh, 1},
                         {"v_perm_b32", k_perm, 1},     {"v_lshl_or_b32", k_lshl_or, 1},
                         {"v_xad_u32", k_xad, 1},       {"v_dot2c_i32_i16", k_dot2c, 1},
                         {"v_pk_add_u16", k_pk_add, 1}, {"v_mul_lo_u32", k_mul_lo, 1},
                         {"v_ashrrev_i32", k_ashr, 1},  {"v_permlane32_swap", k_permlane32, 1},
                         {"v_mad_i64_i32", k_mad_i64, 1}, {"v_fma_f64", k_fma_f64, 1}};
    hipDeviceProp_t prop;
    hipGetDeviceProperties(&prop, 0);
    const int cus = prop.multiProcessorCount;
    const int max_waves = cus * 4 * 4;
    uint32_t* out;
    uint64_t* cyc;
    hipMalloc(&out, (size_t)max_waves * 64 * 4);
    hipMalloc(&cyc, (size_t)max_waves * 16);
    std::vector<uint64_t> h(2 * max_waves);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    printf("{\"cus\": %d, \"iter\": %d, \"results\": [\n", cus, ITER);
    bool first = true;
    for (auto& k : ks) {
        for (int wps : {1, 2, 4}) {
            const int waves = cus * 4 * wps;
            k.f<<<waves, 64>>>(out, cyc, 12345);  // warm
            hipEventRecord(e0);
            k.f<<<waves, 64>>>(out, cyc, 777);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            hipMemcpy(h.data(), cyc, (size_t)waves * 16, hipMemcpyDeviceToHost);
            double sc = 0, rt = 0;
            for (int w = 0; w < waves; w++) {
                sc += (double)h[2 * w];
                rt += (double)h[2 * w + 1];
            }
            sc /= waves;
            rt /= waves;
            const double ghz = sc / (rt * 10.0);  // memrealtime ticks at 100 MHz
            const double ops = (double)ITER * 8 * k.ops_per_asm;
            // per wave: loop cycles / ops; per SIMD with wps waves sharing it
            const double cyc_per_op_wave = sc / ops;
            const double cyc_per_op_simd = ms * 1e-3 * ghz * 1e9 / (ops * wps);
            printf("%s{\"op\": \"%s\", \"waves_per_simd\": %d, \"ghz\": %.3f, \"cyc_per_op_per_wave\": %.2f, "
                   "\"simd_cyc_per_op_wall\": %.2f, \"ms\": %.3f}",
                   first ? "" : ",\n", k.name, wps, ghz, cyc_per_op_wave, cyc_per_op_simd, ms);
            first = false;
        }
    }
    printf("\n]}\n");
    hipFree(out);
    hipFree(cyc);
    return 0;
}
