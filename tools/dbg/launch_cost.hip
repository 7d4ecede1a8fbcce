// Debug aid: host cost of hipLaunchKernelGGL by kernel-argument size (an empty kernel, 16-byte vs ~3 KB by-value
// arguments like orbfe's Geo), and of hipGetLastError / hipEventRecord, on one stream.
// build: hipcc --offload-arch=gfx950 -O2 -o tools/dbg/launch_cost tools/dbg/launch_cost.hip
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

struct Small { int a[4]; };
struct Big { int a[736]; };  // 2 944 bytes

__global__ void k_small(Small s, int* out) { if (threadIdx.x == 0 && s.a[0] < 0) *out = s.a[1]; }
__global__ void k_big(Big b, int* out) { if (threadIdx.x == 0 && b.a[0] < 0) *out = b.a[735]; }

template <typename F>
static double per_call_us(int n, F&& f) {
    auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < n; ++i) f();
    auto t1 = std::chrono::steady_clock::now();
    return std::chrono::duration<double, std::micro>(t1 - t0).count() / n;
}

int main() {
    hipStream_t s;
    hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    int* out;
    hipMalloc(&out, 4);
    Small sm{};
    Big bg{};
    hipEvent_t ev;
    hipEventCreateWithFlags(&ev, hipEventDisableTiming);
    for (int r = 0; r < 3; ++r) {
        hipDeviceSynchronize();
        const double a = per_call_us(2000, [&] { hipLaunchKernelGGL(k_small, dim3(64), dim3(64), 0, s, sm, out); });
        hipDeviceSynchronize();
        const double b = per_call_us(2000, [&] { hipLaunchKernelGGL(k_big, dim3(64), dim3(64), 0, s, bg, out); });
        hipDeviceSynchronize();
        const double c = per_call_us(2000, [&] { hipLaunchKernelGGL(k_big, dim3(64), dim3(1024), 48 * 1024, s, bg, out); });
        hipDeviceSynchronize();
        const double d = per_call_us(2000, [&] { (void)hipGetLastError(); });
        const double e = per_call_us(2000, [&] { hipEventRecord(ev, s); });
        hipDeviceSynchronize();
        printf("launch us: 16-B args %.2f, 2944-B args %.2f, 2944-B + 48 KiB LDS %.2f; hipGetLastError %.3f; hipEventRecord %.2f\n",
               a, b, c, d, e);
    }
    return 0;
}
