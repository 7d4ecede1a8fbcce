// VALU issue rate on gfx950, per instruction: wave64 instructions retired per cycle per CU, with
// 8 independent chains per lane, at 1 and at 8 waves per SIMD (HIP events, the clock read from
// hipDeviceProp_t::clockRate is only used to print the cycles figure next to the ns one).
// f32 controls (v_fma_f32, v_add_f32, v_pk_fma_f32, v_pk_add_f32) next to the integer / packed-f16 ops the
// front-end kernels issue, so that the wave64 issue peak used in bench.py (VALU_PEAK_GIPS) rests on a
// committed measurement (profiles/r03/mulrate_r3*.log).
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/dbg/mulrate tools/dbg/mulrate.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef float f2 __attribute__((ext_vector_type(2)));

#define OPS(X)                                                     \
    X(0, "v_add_u32", u, "v_add_u32 %0, %0, %1")                   \
    X(1, "v_mul_lo_u32", u, "v_mul_lo_u32 %0, %0, %1")             \
    X(2, "v_mul_u32_u24", u, "v_mul_u32_u24 %0, %0, %1")           \
    X(3, "v_mul_hi_u32", u, "v_mul_hi_u32 %0, %0, %1")             \
    X(4, "v_and_b32", u, "v_and_b32 %0, %0, %1")                   \
    X(5, "v_perm_b32", u, "v_perm_b32 %0, %0, %1, %0")             \
    X(6, "v_pk_maximum3_f16", u, "v_pk_maximum3_f16 %0, %0, %1, %0") \
    X(7, "v_pk_add_u16", u, "v_pk_add_u16 %0, %0, %1")             \
    X(8, "v_dot4_u32_u8", u, "v_dot4_u32_u8 %0, %0, %1, %0")       \
    X(9, "v_dot2_u32_u16", u, "v_dot2_u32_u16 %0, %0, %1, %0")     \
    X(10, "v_sad_u16", u, "v_sad_u16 %0, %0, %1, %0")              \
    X(11, "v_cndmask_b32(vcc)", u, "v_cndmask_b32 %0, %0, %1, vcc") \
    X(12, "v_fma_f32", f, "v_fma_f32 %0, %0, %1, %0")              \
    X(13, "v_add_f32", f, "v_add_f32 %0, %0, %1")                  \
    X(14, "v_max3_f32", f, "v_max3_f32 %0, %0, %1, %0")            \
    X(15, "v_mul_f32", f, "v_mul_f32 %0, %0, %1")                  \
    X(16, "v_pk_fma_f32", p, "v_pk_fma_f32 %0, %0, %1, %0")        \
    X(17, "v_pk_add_f32", p, "v_pk_add_f32 %0, %0, %1")            \
    X(18, "v_cvt_f32_u32", u, "v_cvt_f32_u32 %0, %0")                 \
    X(19, "v_add_u32_e64", u, "v_add_u32_e64 %0, %0, %1")             \
    X(20, "v_and_b32_e64", u, "v_and_b32_e64 %0, %0, %1")             \
    X(21, "v_add_f32_e64", f, "v_add_f32_e64 %0, %0, %1")             \
    X(22, "v_fmac_f32", f, "v_fmac_f32 %0, %0, %1")                   \
    X(23, "v_add3_u32", u, "v_add3_u32 %0, %0, %1, %0")               \
    X(24, "v_lshl_add_u32", u, "v_lshl_add_u32 %0, %0, 1, %1")        \
    X(25, "v_bfe_u32", u, "v_bfe_u32 %0, %0, 3, 5")                   \
    X(26, "v_max_u32", u, "v_max_u32 %0, %0, %1")                     \
    X(27, "v_min_u16", u, "v_min_u16 %0, %0, %1")                     \
    X(28, "v_pk_max_f16", u, "v_pk_max_f16 %0, %0, %1")               \
    X(29, "v_max_f16", u, "v_max_f16 %0, %0, %1")                     \
    X(30, "v_dot2c_f32_f16", f, "v_dot2c_f32_f16 %0, %1, %1")         \
    X(31, "v_dot4c_i32_i8", u, "v_dot4c_i32_i8 %0, %1, %1")           \
    X(32, "v_mov_b32", u, "v_mov_b32 %0, %1")                         \
    X(33, "v_xor_b32", u, "v_xor_b32 %0, %0, %1")                     \
    X(34, "v_lshlrev_b32", u, "v_lshlrev_b32 %0, 1, %0")              \
    X(35, "v_sub_u32", u, "v_sub_u32 %0, %1, %0")                     \
    X(36, "v_cndmask_b32_e64", u, "v_cndmask_b32_e64 %0, %0, %1, s[0:1]") \
    X(37, "v_alignbyte_b32", u, "v_alignbyte_b32 %0, %0, %1, 1")      \
    X(38, "v_pk_fma_f16", u, "v_pk_fma_f16 %0, %0, %1, %0")           \
    X(39, "v_fma_f16", u, "v_fma_f16 %0, %0, %1, %0")

constexpr int kOps = 40;

template <int OP>
__global__ __launch_bounds__(256) void k(unsigned* out, unsigned s, int n, unsigned long long* clk) {
    const unsigned long long c0 = __builtin_readcyclecounter(), w0 = wall_clock64();
    unsigned u[8];
    float f[8];
    f2 p[8];
    const float fs = __builtin_bit_cast(float, 0x3f800001u);
    const f2 ps = {fs, fs};
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        u[i] = threadIdx.x + i;
        f[i] = (float)(threadIdx.x + i) * 1e-3f;
        p[i] = f2{f[i], f[i] + 1.f};
    }
    for (int it = 0; it < n; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
#define EMIT(id, name, kind, text)                                                        \
    if constexpr (OP == id) {                                                             \
        if constexpr (#kind[0] == 'u') asm volatile(text : "+v"(u[i]) : "v"(s));          \
        if constexpr (#kind[0] == 'f') asm volatile(text : "+v"(f[i]) : "v"(fs));         \
        if constexpr (#kind[0] == 'p') asm volatile(text : "+v"(p[i]) : "v"(ps));         \
    }
            OPS(EMIT)
#undef EMIT
        }
    }
    unsigned r = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) r += u[i] + __builtin_bit_cast(unsigned, f[i]) + __builtin_bit_cast(unsigned, p[i].x + p[i].y);
    out[blockIdx.x * 256 + threadIdx.x] = r;
    if (threadIdx.x == 0) {
        clk[2 * blockIdx.x] = __builtin_readcyclecounter() - c0;
        clk[2 * blockIdx.x + 1] = wall_clock64() - w0;
    }
}

template <int... I>
struct Table {
    static constexpr void (*f[sizeof...(I)])(unsigned*, unsigned, int, unsigned long long*) = {k<I>...};
};

int main() {
    hipDeviceProp_t prop;
    hipGetDeviceProperties(&prop, 0);
    const int cus = prop.multiProcessorCount;
    const char* names[kOps] = {
#define NAME(id, name, kind, text) name,
        OPS(NAME)
#undef NAME
    };
    using T = Table<0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17, 18, 19, 20, 21, 22, 23, 24, 25, 26, 27, 28, 29,
                     30, 31, 32, 33, 34, 35, 36, 37, 38, 39>;
    unsigned* out;
    hipMalloc(&out, (size_t)cus * 8 * 256 * 4);
    unsigned long long* clk;
    hipMalloc(&clk, (size_t)cus * 8 * 16);
    std::vector<unsigned long long> hclk((size_t)cus * 16);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const int n = 4096;
    printf("%d CUs, clockRate %.0f MHz (peak; the chip may run lower under load)\n", cus, prop.clockRate / 1e3);
    printf("cycles: shader clock (s_memtime) per wave-instruction per SIMD, from each block's own cycle count;\n"
           "GHz: shader cycles / 100 MHz wall-clock ticks of the same blocks\n");
    printf("%-20s %12s %12s %10s %10s %7s\n", "instruction", "1 wave/SIMD", "8 waves/SIMD", "cyc 1w", "cyc 8w", "GHz 8w");
    for (int op = 0; op < kOps; ++op) {
        double rate[2], cyc[2], ghz8 = 0;
        for (int m = 0; m < 2; ++m) {
            const int blocks = m ? cus * 8 : cus;  // 256 threads = 4 waves = 1 per SIMD per block
            hipLaunchKernelGGL(T::f[op], dim3(blocks), dim3(256), 0, 0, out, 3u, n, clk);
            hipEventRecord(a);
            for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(T::f[op], dim3(blocks), dim3(256), 0, 0, out, 3u, n, clk);
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms;
            hipEventElapsedTime(&ms, a, b);
            const double inst = 3.0 * blocks * 4 * n * 8;      // wave-instructions
            rate[m] = inst / (ms * 1e6) / cus;                 // wave-instructions per ns per CU
            hipMemcpy(hclk.data(), clk, (size_t)blocks * 16, hipMemcpyDeviceToHost);
            double sc = 0, sw = 0;
            for (int b2 = 0; b2 < blocks; ++b2) {
                sc += (double)hclk[2 * b2];
                sw += (double)hclk[2 * b2 + 1];
            }
            // a block's wave is one of (m ? 8 : 1) waves sharing its SIMD: cycles per instruction per SIMD
            cyc[m] = sc / blocks / ((double)n * 8 * (m ? 8 : 1));
            if (m) ghz8 = sc / sw * 0.1;  // shader cycles per 10 ns tick -> GHz
        }
        printf("%-20s %8.3f /ns %8.3f /ns %10.2f %10.2f %7.3f\n", names[op], rate[0], rate[1], cyc[0], cyc[1], ghz8);
    }
    return 0;
}
