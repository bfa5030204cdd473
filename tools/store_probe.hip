// Per-CU store / load throughput probe (diagnostic, not part of the library).
//   hipcc --offload-arch=gfx950 -O3 -o tools/store_probe tools/store_probe.hip && tools/store_probe
// Each workgroup streams `kb` KB per wave through 16-B-per-lane stores (or loads), coalesced in
// 1-KB wave-instructions; grids of 1..4 workgroups per CU on 8..256 CUs.  Reports GB/s per CU.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ __launch_bounds__(256) void st(float4* out, int n16) {
    float4* p = out + (size_t)blockIdx.x * blockDim.x * n16 + threadIdx.x;
    const float4 v = make_float4(threadIdx.x, 1.f, 2.f, 3.f);
#pragma unroll 8
    for (int i = 0; i < n16; ++i) p[(size_t)i * blockDim.x] = v;
}
__global__ __launch_bounds__(256) void ld(const float4* in, float* sink, int n16) {
    const float4* p = in + (size_t)blockIdx.x * blockDim.x * n16 + threadIdx.x;
    float4 a = make_float4(0, 0, 0, 0);
#pragma unroll 8
    for (int i = 0; i < n16; ++i) {
        const float4 v = p[(size_t)i * blockDim.x];
        a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
    }
    if (a.x == 12345.f) sink[0] = a.y + a.z + a.w;
}

int main() {
    const size_t cap = 2ull << 30;   // 2 GB buffer
    float4* buf;
    float* sink;
    hipMalloc(&buf, cap);
    hipMalloc(&sink, 64);
    hipMemset(buf, 0, cap);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    int cus = 256;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const int kbs[] = {64, 256};
    const int nblks[] = {8, 32, 128, 256, 512, 1024};
    for (int mode = 0; mode < 2; ++mode)
        for (int kb : kbs)
            for (int nb : nblks) {
                const int n16 = kb * 1024 / (256 * 16) * 4;     // per thread: 4 waves x kb KB per block
                const size_t bytes = (size_t)nb * 256 * n16 * 16;
                if (bytes > cap) continue;
                for (int w = 0; w < 3; ++w) {
                    if (mode == 0) st<<<nb, 256>>>(buf, n16);
                    else ld<<<nb, 256>>>(buf, sink, n16);
                }
                hipEventRecord(a);
                const int reps = 10;
                for (int r = 0; r < reps; ++r) {
                    if (mode == 0) st<<<nb, 256>>>(buf, n16);
                    else ld<<<nb, 256>>>(buf, sink, n16);
                }
                hipEventRecord(b);
                hipEventSynchronize(b);
                float ms = 0;
                hipEventElapsedTime(&ms, a, b);
                const double s = ms * 1e-3 / reps;
                const int active = nb < cus ? nb : cus;
                printf("%s  %4d KB/block  %5d blocks  %8.1f us  %7.2f TB/s chip  %6.1f GB/s per active CU\n",
                       mode ? "load " : "store", kb * 4, nb, s * 1e6, bytes / s / 1e12, bytes / s / 1e9 / active);
            }
    return 0;
}
