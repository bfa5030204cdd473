// Device-side helpers shared by the gfx950 kernels of libclipembed.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint16_t bf16_t;  // raw bf16 bits in memory

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;   // MFMA bf16 operand (4 VGPRs)
typedef __attribute__((ext_vector_type(4))) short s16x4;     // ds_read_b64_tr_b16 result
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;

#define CE_LDS __attribute__((address_space(3)))
#define CE_GLOBAL __attribute__((address_space(1)))

__device__ __forceinline__ float bf2f(bf16_t v) { return __uint_as_float((uint32_t)v << 16); }

// Round-to-nearest-even, NaN stays NaN (hipcc lowers the cast to v_cvt_pk_bf16_f32).
__device__ __forceinline__ bf16_t f2bf(float f) {
    return __builtin_bit_cast(bf16_t, (__bf16)f);
}

// two floats -> packed bf16 pair (one v_cvt_pk_bf16_f32, round-to-nearest-even, NaN stays NaN)
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2_t;
typedef __attribute__((ext_vector_type(2))) float f32x2_t;
__device__ __forceinline__ uint32_t pack_bf2(float lo, float hi) {
    return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2_t){lo, hi}, bf16x2_t));
}

// Residual stream as two bf16 planes (EPI_LN_STATS_HL): hi = bf16(v), lo = bf16(v - hi); hi + lo
// keeps ~16 significand bits (|v - (hi + lo)| <= 2^-16 |v|: 2^-8 of v for hi, 2^-8 of that for lo) in 4 bytes, and hi is exactly the bf16
// copy the LN-folded GEMMs read as their A operand.
__device__ __forceinline__ void split_hl(float a, float b, uint32_t& hi, uint32_t& lo) {
    hi = pack_bf2(a, b);
    lo = pack_bf2(a - __uint_as_float(hi << 16), b - __uint_as_float(hi & 0xffff0000u));
}
__device__ __forceinline__ float2 join_hl(uint32_t hi, uint32_t lo) {
    return make_float2(__uint_as_float(hi << 16) + __uint_as_float(lo << 16),
                       __uint_as_float(hi & 0xffff0000u) + __uint_as_float(lo & 0xffff0000u));
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}
__device__ __forceinline__ float wave_min(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fminf(v, __shfl_xor(v, o, 64));
    return v;
}

// erf via Abramowitz & Stegun 7.1.26 (|error| <= 1.5e-7): one exp + one reciprocal, branch-free.
__device__ __forceinline__ float erf_fast(float x) {
    const float a = fabsf(x);
    const float t = __frcp_rn(fmaf(0.3275911f, a, 1.0f));
    float p = fmaf(1.061405429f, t, -1.453152027f);
    p = fmaf(p, t, 1.421413741f);
    p = fmaf(p, t, -0.284496736f);
    p = fmaf(p, t, 0.254829592f);
    p *= t;
    const float y = fmaf(-p, __expf(-a * a), 1.0f);
    return copysignf(y, x);
}
// Exact-erf GELU (torch.nn.GELU default; erf to 1.5e-7) and QuickGELU (transformer.py:32-35).
__device__ __forceinline__ float gelu_erf(float x) { return 0.5f * x * (1.0f + erf_fast(x * 0.70710678118654752f)); }
__device__ __forceinline__ float quick_gelu(float x) {
    return x * __builtin_amdgcn_rcpf(1.0f + __expf(-1.702f * x));
}

// GELU for a pair of values in packed f32 (v_pk_fma_f32 / v_pk_mul_f32: two lanes' worth per
// 4-cycle issue) with no transcendental: Phi(x) = 0.5 + u * P((u^2 - 12.5) / 12.5), u = clamp(x, +-5),
// P a degree-12 least-squares Chebyshev fit of (Phi(u) - 0.5) / u on u in [0, 5].  GELU error <=
// 2.5e-6 * max(1, |y|) over all x (f32 evaluation; tests/test_host.py), far below the bf16 rounding of the
// GEMM output it feeds; ~36 issue cycles per value vs ~68 for erf_fast (1 rcp + 1 exp + 13 VALU).
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f32x2 gelu_pair(f32x2 x) {
    f32x2 u;
    u.x = __builtin_amdgcn_fmed3f(x.x, -5.0f, 5.0f);
    u.y = __builtin_amdgcn_fmed3f(x.y, -5.0f, 5.0f);
    const f32x2 t = __builtin_elementwise_fma(u * u, (f32x2)(0.08f), (f32x2)(-1.0f));
    f32x2 p = (f32x2)(0.00058384275f);
    p = __builtin_elementwise_fma(p, t, (f32x2)(-0.0016009705f));
    p = __builtin_elementwise_fma(p, t, (f32x2)(0.0017913138f));
    p = __builtin_elementwise_fma(p, t, (f32x2)(-0.002716318f));
    p = __builtin_elementwise_fma(p, t, (f32x2)(0.0063403393f));
    p = __builtin_elementwise_fma(p, t, (f32x2)(-0.011136664f));
    p = __builtin_elementwise_fma(p, t, (f32x2)(0.016434977f));
    p = __builtin_elementwise_fma(p, t, (f32x2)(-0.02327942f));
    p = __builtin_elementwise_fma(p, t, (f32x2)(0.031435322f));
    p = __builtin_elementwise_fma(p, t, (f32x2)(-0.040440924f));
    p = __builtin_elementwise_fma(p, t, (f32x2)(0.051521037f));
    p = __builtin_elementwise_fma(p, t, (f32x2)(-0.070296355f));
    p = __builtin_elementwise_fma(p, t, (f32x2)(0.14136378f));
    const f32x2 phi = __builtin_elementwise_fma(u, p, (f32x2)(0.5f));
    return x * phi;
}

// GELU as x * sigmoid(z(x)) with z(x) = u * P(u^2), u = clamp(x, +-4.75), P a degree-2 fit of
// logit(Phi) (times -log2 e, so the exponential is one v_exp_f32):  y = x / (1 + 2^(u * P(u^2))).
// Error <= 6.2e-5 * max(1, |y|) vs the exact-erf GELU over all x in f32 (tests/test_host.py), 30x
// below the bf16 rounding (2^-9) of the GEMM output it feeds.  7 VALU + 2 transcendental ops (~44
// issue cycles per value for one wave on a SIMD) vs 17 VALU for the degree-12 polynomial above;
// gelu_fast4 shares one reciprocal between two values (1.5 transcendentals per value).
#define CE_GELU_CLAMP 4.75f
#define CE_GELU_C0 -2.29998779296875f
#define CE_GELU_C1 -0.10797221958637238f
#define CE_GELU_C2 0.0012323867995291948f
// four independent values per call, so the dependent chains interleave
__device__ __forceinline__ f32x4 gelu_fast4(f32x4 x) {
    f32x4 u;
#pragma unroll
    for (int e = 0; e < 4; ++e) u[e] = __builtin_amdgcn_fmed3f(x[e], -CE_GELU_CLAMP, CE_GELU_CLAMP);
    const f32x4 u2 = u * u;
    f32x4 p = __builtin_elementwise_fma(u2, (f32x4)(CE_GELU_C2), (f32x4)(CE_GELU_C1));
    p = __builtin_elementwise_fma(p, u2, (f32x4)(CE_GELU_C0));
    const f32x4 z = u * p;
    f32x4 d;
#pragma unroll
    for (int e = 0; e < 4; ++e) d[e] = 1.0f + __builtin_amdgcn_exp2f(z[e]);
    // one reciprocal per pair of denominators (1 <= d <= 1 + 2^19.5): 1/d0 = d1 / (d0 d1); a
    // v_rcp_f32 (quarter rate) traded for two multiplies, ~3 ulp added to an error budget of 6.2e-5
    const float ra = __builtin_amdgcn_rcpf(d[0] * d[1]), rb = __builtin_amdgcn_rcpf(d[2] * d[3]);
    const f32x4 inv = {d[1] * ra, d[0] * ra, d[3] * rb, d[2] * rb};
    return x * inv;
}
__device__ __forceinline__ float gelu_fast(float x) {
    const float u = __builtin_amdgcn_fmed3f(x, -CE_GELU_CLAMP, CE_GELU_CLAMP);
    const float u2 = u * u;
    const float p = fmaf(fmaf(u2, CE_GELU_C2, CE_GELU_C1), u2, CE_GELU_C0);
    return x * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(u * p));
}

enum { ACT_NONE = 0, ACT_GELU = 1, ACT_QGELU = 2,
       // (device-side template codes of the activation-backward GEMM epilogue, launch_gemm_act_bwd:
       // out = dh * act'(pre) for the GELU / QuickGELU forward activation)
       ACT_GELU_BWD = 3, ACT_QGELU_BWD = 4 };

// d/dx [x * Phi(x)] = Phi(x) + x phi(x), with erf by Abramowitz & Stegun 7.1.26 (|error| <= 1.5e-7,
// as erf_fast) sharing its one exponential with phi: exp(-a^2) = exp(-x^2 / 2) for a = |x| / sqrt(2).
// One exp + one rcp + ~10 FMA per value instead of libm erff + expf: the activation backward over the
// C4 batch's 363 M values was VALU-bound, not HBM-bound.
// (v_rcp_f32, 1 ulp, in place of the IEEE-rounded reciprocal's 10-instruction division sequence:
// t is in (0, 1], far inside the approximation's own 1.5e-7)
__device__ __forceinline__ float gelu_grad(float x) {
    const float a = fabsf(x) * 0.70710678118654752f;
    const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, a, 1.0f));
    float p = fmaf(1.061405429f, t, -1.453152027f);
    p = fmaf(p, t, 1.421413741f);
    p = fmaf(p, t, -0.284496736f);
    p = fmaf(p, t, 0.254829592f);
    p *= t;
    const float e = __expf(-a * a);
    const float erf_a = fmaf(-p, e, 1.0f);                               // erf(|x| / sqrt 2)
    return fmaf(0.5f, copysignf(erf_a, x), 0.5f) + x * 0.3989422804014327f * e;
}
__device__ __forceinline__ float qgelu_grad(float x) {
    const float sg = __builtin_amdgcn_rcpf(1.0f + __expf(-1.702f * x));
    return sg * (1.0f + 1.702f * x * (1.0f - sg));
}


template <int ACT>
__device__ __forceinline__ float apply_act(float x) {
    if constexpr (ACT == ACT_GELU) return gelu_erf(x);
    else if constexpr (ACT == ACT_QGELU) return quick_gelu(x);
    else return x;
}

// Asynchronous 16-byte global -> LDS copy (global_load_lds_dwordx4).  The LDS destination is
// the wave-uniform `lds_wave_base` + lane*16; the global source is per lane.
__device__ __forceinline__ void glds16(const void* gsrc, void* lds_wave_base) {
    __builtin_amdgcn_global_load_lds((const CE_GLOBAL void*)gsrc, (CE_LDS void*)lds_wave_base, 16, 0, 0);
}
