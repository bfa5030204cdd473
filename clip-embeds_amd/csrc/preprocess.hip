// Eval image preprocessing on the device: RGB uint8 HWC images of any size ->
// normalised [B,3,S,S] model input, replacing the host-side PIL / torchvision pipelines
//   CLIP  open_clip/src/open_clip/transform.py:371-389  Resize(S, BICUBIC) shortest edge (Pillow)
//         -> CenterCrop(S) -> ToTensor -> Normalize(OpenAI)
//   PACL  Patch-Aligned-Contrastive-Learning/data/utils.py:33-37  ToTensor -> Resize((S,S))
//         (bilinear, antialias) -> Normalize(ImageNet)
//
// Both resamplers are separable two-pass filters with per-output-index taps (computed on the host
// exactly as Pillow's precompute_coeffs / ATen's _compute_weights_aa do).  Pass 1 (horizontal)
// writes only the S output columns of the crop window for the source rows the vertical taps
// touch; pass 2 (vertical) reduces those rows and applies ToTensor + Normalize.  The CLIP path
// keeps Pillow's arithmetic bit for bit: int32 taps with 22 fractional bits, a 2^21 rounding
// bias, >>22 and clamp to uint8 after EACH pass; ToTensor/Normalize are IEEE f32 divisions as in
// torch.  The PACL path is f32 multiply-add in tap order (ATen's loop order).
#include "ce_device.h"
#include "ce_kernels.h"

namespace ce {
namespace {

constexpr int PB = 22;   // Pillow PRECISION_BITS = 32 - 8 - 2

__device__ __forceinline__ int clip8(int ss) {
    const int v = ss >> PB;          // arithmetic shift, as Pillow's lookup index
    return v < 0 ? 0 : (v > 255 ? 255 : v);
}

// Pass 1: one block per (source row r of image b); thread loops over (output column, channel).
template <bool FLOAT>
__global__ __launch_bounds__(256) void prep_hpass_k(const uint8_t* __restrict__ img, const PrepMeta* __restrict__ meta,
                                                    const int* __restrict__ bounds, const void* __restrict__ taps,
                                                    void* __restrict__ tmp, int S) {
    const PrepMeta m = meta[blockIdx.y];
    const int r = blockIdx.x;
    if (r >= m.nrows) return;
    const uint8_t* src = img + m.in_off + (size_t)(m.ybase + r) * m.W * 3;
    const int* bx = bounds + m.bx_off;
    for (int t = threadIdx.x; t < S * 3; t += 256) {
        const int ox = t / 3, c = t - ox * 3;
        const int xmin = bx[2 * ox], n = bx[2 * ox + 1];
        const uint8_t* sp = src + (size_t)xmin * 3 + c;
        if constexpr (FLOAT) {
            const float* k = static_cast<const float*>(taps) + m.kx_off + (size_t)ox * m.ksx;
            float acc = ((float)sp[0] / 255.0f) * k[0];
            for (int j = 1; j < n; ++j) acc = __fadd_rn(acc, __fmul_rn((float)sp[3 * j] / 255.0f, k[j]));
            static_cast<float*>(tmp)[m.tmp_off + ((size_t)r * S + ox) * 3 + c] = acc;
        } else {
            const int* k = static_cast<const int*>(taps) + m.kx_off + (size_t)ox * m.ksx;
            int ss = 1 << (PB - 1);
            for (int j = 0; j < n; ++j) ss += (int)sp[3 * j] * k[j];
            static_cast<uint8_t*>(tmp)[m.tmp_off + ((size_t)r * S + ox) * 3 + c] = (uint8_t)clip8(ss);
        }
    }
}

// Pass 2: one block per (output row oy of image b); ToTensor + Normalize fused, planar output.
template <bool FLOAT, bool OUT_BF16>
__global__ __launch_bounds__(256) void prep_vpass_k(const PrepMeta* __restrict__ meta, const int* __restrict__ bounds,
                                                    const void* __restrict__ taps, const void* __restrict__ tmp,
                                                    void* __restrict__ out, int S, float m0, float m1, float m2,
                                                    float s0, float s1, float s2) {
    const int b = blockIdx.y, oy = blockIdx.x;
    const PrepMeta m = meta[b];
    const int* by = bounds + m.by_off;
    const int ymin = by[2 * oy], n = by[2 * oy + 1];      // ymin relative to m.ybase
    for (int t = threadIdx.x; t < S * 3; t += 256) {
        const int ox = t / 3, c = t - ox * 3;
        float x;
        if constexpr (FLOAT) {
            const float* k = static_cast<const float*>(taps) + m.ky_off + (size_t)oy * m.ksy;
            const float* tp = static_cast<const float*>(tmp) + m.tmp_off + ((size_t)ymin * S + ox) * 3 + c;
            float acc = tp[0] * k[0];
            for (int j = 1; j < n; ++j) acc = __fadd_rn(acc, __fmul_rn(tp[(size_t)j * S * 3], k[j]));
            x = acc;
        } else {
            const int* k = static_cast<const int*>(taps) + m.ky_off + (size_t)oy * m.ksy;
            const uint8_t* tp = static_cast<const uint8_t*>(tmp) + m.tmp_off + ((size_t)ymin * S + ox) * 3 + c;
            int ss = 1 << (PB - 1);
            for (int j = 0; j < n; ++j) ss += (int)tp[(size_t)j * S * 3] * k[j];
            x = (float)clip8(ss) / 255.0f;                  // ToTensor: float(u8) / 255
        }
        const float mean = c == 0 ? m0 : (c == 1 ? m1 : m2);
        const float sd = c == 0 ? s0 : (c == 1 ? s1 : s2);
        const float y = (x - mean) / sd;                    // Normalize: sub_ then div_
        const size_t o = (((size_t)b * 3 + c) * S + oy) * S + ox;
        if constexpr (OUT_BF16) static_cast<bf16_t*>(out)[o] = (bf16_t)f2bf(y);
        else static_cast<float*>(out)[o] = y;
    }
}

}  // namespace

hipError_t launch_preprocess(const uint8_t* images, const PrepMeta* meta, const int* bounds, const void* taps,
                             void* tmp, int B, int max_rows, int S, bool pacl, bool out_bf16, const float* mean,
                             const float* stdv, void* out, hipStream_t s) {
    if (B <= 0) return hipSuccess;
    const dim3 g1((unsigned)max_rows, (unsigned)B), g2((unsigned)S, (unsigned)B);
    if (pacl) hipLaunchKernelGGL(prep_hpass_k<true>, g1, dim3(256), 0, s, images, meta, bounds, taps, tmp, S);
    else hipLaunchKernelGGL(prep_hpass_k<false>, g1, dim3(256), 0, s, images, meta, bounds, taps, tmp, S);
#define CE_VP(F, O) hipLaunchKernelGGL((prep_vpass_k<F, O>), g2, dim3(256), 0, s, meta, bounds, taps, tmp, out, S, \
                                       mean[0], mean[1], mean[2], stdv[0], stdv[1], stdv[2])
    if (pacl) { if (out_bf16) CE_VP(true, true); else CE_VP(true, false); }
    else { if (out_bf16) CE_VP(false, true); else CE_VP(false, false); }
#undef CE_VP
    return hipGetLastError();
}

}  // namespace ce
