// Debug aid: issue cost of v_mul_lo_u32 / v_mul_hi_u32 / v_mad_u64_u32 against v_mul_u32_u24 and v_add_u32 on
// gfx950 (8 independent chains per lane, 8 waves per SIMD, HIP events).  Build: hipcc --offload-arch=gfx950 -O3
#include <hip/hip_runtime.h>
#include <cstdio>

template <int OP>
__global__ __launch_bounds__(256) void k(unsigned* out, unsigned s, int n) {
    unsigned x[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = threadIdx.x + i;
    for (int it = 0; it < n; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            if (OP == 0) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(x[i]) : "s"(s));
            if (OP == 1) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(x[i]) : "s"(s));
            if (OP == 2) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x[i]) : "s"(s));
            if (OP == 3) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(x[i]) : "s"(s));
            if (OP == 4) asm volatile("v_pk_maximum3_f16 %0, %0, %1, %0" : "+v"(x[i]) : "s"(s));
            if (OP == 5) asm volatile("v_dot4_u32_u8 %0, %0, %1, %0" : "+v"(x[i]) : "s"(s));
        }
    }
    unsigned r = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) r += x[i];
    out[blockIdx.x * 256 + threadIdx.x] = r;
}

int main() {
    const int blocks = 256 * 8, n = 4096;
    unsigned* out;
    hipMalloc(&out, blocks * 256 * 4);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const char* names[] = {"v_mul_lo_u32", "v_mul_u32_u24", "v_add_u32", "v_mul_hi_u32", "v_pk_maximum3_f16", "v_dot4_u32_u8"};
    for (int rep = 0; rep < 2; ++rep)
        for (int op = 0; op < 6; ++op) {
            auto f = op == 0 ? k<0> : op == 1 ? k<1> : op == 2 ? k<2> : op == 3 ? k<3> : op == 4 ? k<4> : k<5>;
            hipLaunchKernelGGL(f, dim3(blocks), dim3(256), 0, 0, out, 3u, n);
            hipEventRecord(a);
            hipLaunchKernelGGL(f, dim3(blocks), dim3(256), 0, 0, out, 3u, n);
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms;
            hipEventElapsedTime(&ms, a, b);
            const double inst = (double)blocks * 4 * n * 8;  // wave-instructions
            if (rep) printf("%-20s %.3f ms  %.2f wave-inst/ns/CU\n", names[op], ms, inst / (ms * 1e6) / 256);
        }
    return 0;
}
