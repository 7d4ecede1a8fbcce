// Does gfx950 LDS serve 2-byte-aligned dword reads (unaligned access mode), and what does the compiler emit?
// hipcc --offload-arch=gfx950 -O3 -mllvm -amdgpu-... ; run: ./lds_unaligned
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
__global__ void k(uint32_t* out, int sh) {
    __shared__ uint8_t b[1024];
    for (int i = threadIdx.x; i < 1024; i += 64) b[i] = (uint8_t)(i * 7 + 3);
    __syncthreads();
    const uint32_t off = 4 * threadIdx.x + sh;
    uint32_t v;
    __builtin_memcpy(&v, b + off, 4);   // unaligned dword (the compiler picks the access)
    out[threadIdx.x] = v;
}
int main() {
    uint32_t* d; hipMalloc(&d, 256);
    uint32_t h[64];
    int bad = 0;
    for (int sh = 0; sh < 4; ++sh) {
        hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, sh);
        hipMemcpy(h, d, 256, hipMemcpyDeviceToHost);
        for (int t = 0; t < 64; ++t) {
            uint32_t e = 0;
            for (int j = 0; j < 4; ++j) e |= (uint32_t)(uint8_t)((4 * t + sh + j) * 7 + 3) << (8 * j);
            if (h[t] != e) { if (bad < 4) printf("sh %d t %d got %08x want %08x\n", sh, t, h[t], e); ++bad; }
        }
    }
    printf("mismatches: %d\n", bad);
    return bad != 0;
}
