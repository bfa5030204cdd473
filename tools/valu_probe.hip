// VALU issue-rate probe for the GEMM epilogue design (one wave per SIMD, no MFMA): cycles per
// wave-instruction of independent v_fma_f32 / v_pk_fma_f32 / v_pk_fma_f16 / v_exp_f32 / v_exp_f16
// chains, from s_memtime around an unrolled loop.  hipcc --offload-arch=gfx950 -O3 tools/valu_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>

typedef _Float16 h2 __attribute__((ext_vector_type(2)));
typedef float f2 __attribute__((ext_vector_type(2)));

template <int KIND>
__global__ __launch_bounds__(256, 1) void probe(float* out, long long* cyc, int iters) {
    float a[8];
    f2 p[8];
    h2 q[8];
    for (int i = 0; i < 8; ++i) {
        a[i] = threadIdx.x * 1e-3f + i;
        p[i] = f2{a[i], a[i] + 1};
        q[i] = h2{(_Float16)(a[i] * 1e-2f), (_Float16)(a[i] * 2e-2f)};
    }
    const float m = 0.999f;
    const f2 pm = {0.999f, 0.998f};
    const h2 qm = {(_Float16)0.999f, (_Float16)0.998f};
    __syncthreads();
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int r = 0; r < 16; ++r)
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                if constexpr (KIND == 0) asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(a[i]) : "v"(m));
                if constexpr (KIND == 1) asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(p[i]) : "v"(pm));
                if constexpr (KIND == 2) asm volatile("v_pk_fma_f16 %0, %0, %1, %1" : "+v"(q[i]) : "v"(qm));
                if constexpr (KIND == 3) asm volatile("v_exp_f32 %0, %0" : "+v"(a[i]));
                if constexpr (KIND == 4) asm volatile("v_exp_f16 %0, %0" : "+v"(q[i]));
                if constexpr (KIND == 5) asm volatile("v_pk_mul_f16 %0, %0, %1" : "+v"(q[i]) : "v"(qm));
                if constexpr (KIND == 6) asm volatile("v_cvt_pk_bf16_f32 %0, %1, %1" : "=v"(q[i]) : "v"(a[i]));
            }
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    float s = 0;
    for (int i = 0; i < 8; ++i) s += a[i] + p[i].x + (float)q[i].x;
    out[blockIdx.x * 256 + threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
    float* out;
    long long* cyc;
    const int nb = 256, iters = 2000;
    hipMalloc(&out, nb * 256 * 4);
    hipMalloc(&cyc, nb * 8);
    const char* names[] = {"v_fma_f32", "v_pk_fma_f32", "v_pk_fma_f16", "v_exp_f32", "v_exp_f16", "v_pk_mul_f16",
                           "v_cvt_pk_bf16_f32"};
    for (int k = 0; k < 7; ++k) {
        for (int rep = 0; rep < 2; ++rep) {
            switch (k) {
                case 0: hipLaunchKernelGGL(probe<0>, dim3(nb), dim3(256), 0, 0, out, cyc, iters); break;
                case 1: hipLaunchKernelGGL(probe<1>, dim3(nb), dim3(256), 0, 0, out, cyc, iters); break;
                case 2: hipLaunchKernelGGL(probe<2>, dim3(nb), dim3(256), 0, 0, out, cyc, iters); break;
                case 3: hipLaunchKernelGGL(probe<3>, dim3(nb), dim3(256), 0, 0, out, cyc, iters); break;
                case 4: hipLaunchKernelGGL(probe<4>, dim3(nb), dim3(256), 0, 0, out, cyc, iters); break;
                case 5: hipLaunchKernelGGL(probe<5>, dim3(nb), dim3(256), 0, 0, out, cyc, iters); break;
                case 6: hipLaunchKernelGGL(probe<6>, dim3(nb), dim3(256), 0, 0, out, cyc, iters); break;
            }
            hipDeviceSynchronize();
        }
        long long h[256];
        hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
        double avg = 0;
        for (int i = 0; i < nb; ++i) avg += h[i];
        avg /= nb;
        printf("%-20s %8.2f cycles per wave-instruction (s_memtime)\n", names[k], avg / (iters * 16.0 * 8));
    }
    return 0;
}
