// Text-tower training kernels for gfx950 (the NegCLIP step of
// open_clip_train/train.py:85-189 with --lock-image, train-clip.sh:22): everything the backward
// of the text transformer, its pooling/projection/normalisation and the contrastive loss need
// beyond the forward kernels, plus AdamW.
//
// Reference semantics (the autograd of):
//   ResidualAttentionBlock     open_clip/src/open_clip/transformer.py:257-268 (MHA :242-255, MLP :235-239)
//   LayerNorm                  transformer.py:23-29 (eps 1e-5)
//   GELU (erf) / QuickGELU     torch.nn.GELU / transformer.py:32-35
//   token + positional embed   model.py:286-288;  EOT pooling + projection  transformer.py:839-855
//   F.normalize                model.py:300
//   ClipLoss / NegCLIP         open_clip/src/open_clip/loss.py:137-193 (CE, ignore_index -100)
//   AdamW                      torch.optim.AdamW (open_clip_train/main.py: betas, eps, wd groups)
#include "ce_device.h"
#include "ce_kernels.h"
#include "knobs.h"

#include <hipcub/hipcub.hpp>

#include <algorithm>

namespace ce {
namespace {

template <typename T> __device__ __forceinline__ float ld_f(const T* p);
template <> __device__ __forceinline__ float ld_f<float>(const float* p) { return *p; }
template <> __device__ __forceinline__ float ld_f<bf16_t>(const bf16_t* p) { return bf2f(*p); }
template <typename T> __device__ __forceinline__ void st_f(T* p, float v);
template <> __device__ __forceinline__ void st_f<float>(float* p, float v) { *p = v; }
template <> __device__ __forceinline__ void st_f<bf16_t>(bf16_t* p, float v) { *p = f2bf(v); }

// ---------------------------------------------------------------------------------------------
// out[c][r] = in[r][c] for r < R, c < C; rows r in [R, Rpad) of the output are zero (so a GEMM
// can contract over a K padded to a multiple of 64).  64x64 tiles through LDS.
template <typename TI, typename TO>
__global__ __launch_bounds__(256) void transpose_k(TO* __restrict__ out, long ldo, const TI* __restrict__ in,
                                                   long ldi, int R, int C, int Rpad) {
    __shared__ float tile[64][65];
    const int r0 = blockIdx.x * 64, c0 = blockIdx.y * 64;
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const int r = r0 + ty + 4 * k, c = c0 + tx;
        tile[ty + 4 * k][tx] = (r < R && c < C) ? ld_f(in + (size_t)r * ldi + c) : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const int c = c0 + ty + 4 * k, r = r0 + tx;
        if (c < C && r < Rpad) st_f(out + (size_t)c * ldo + r, tile[tx][ty + 4 * k]);
    }
}

// Vectorised form for bf16 output (C, Rpad, ldi, ldo multiples of 8): 16-B loads of 8 input
// elements, the tile in LDS as bf16, and 16-B stores of 8 consecutive output elements gathered
// down an LDS column — 2 loads + 2 stores per thread per 64x64 tile instead of 16 + 16.
template <typename TI>
__global__ __launch_bounds__(256) void transpose_v8_k(bf16_t* __restrict__ out, long ldo, const TI* __restrict__ in,
                                                      long ldi, int R, int C, int Rpad) {
    __shared__ unsigned short tile[64][72];      // 144-B rows: the 8-row column gathers hit distinct banks
    const int r0 = blockIdx.x * 64, c0 = blockIdx.y * 64;
    const int ch = threadIdx.x & 7, rr = threadIdx.x >> 3;   // 16-B chunk (8 elements), row 0..31
#pragma unroll
    for (int ps = 0; ps < 2; ++ps) {
        const int r = r0 + rr + 32 * ps, c = c0 + ch * 8;
        uint4 v = make_uint4(0, 0, 0, 0);
        if (r < R && c < C) {
            if constexpr (sizeof(TI) == 2) {
                v = *reinterpret_cast<const uint4*>(in + (size_t)r * ldi + c);
            } else {
                const float4 a = *reinterpret_cast<const float4*>(in + (size_t)r * ldi + c);
                const float4 b = *reinterpret_cast<const float4*>(in + (size_t)r * ldi + c + 4);
                v = make_uint4(pack_bf2(a.x, a.y), pack_bf2(a.z, a.w), pack_bf2(b.x, b.y), pack_bf2(b.z, b.w));
            }
        }
        *reinterpret_cast<uint4*>(&tile[rr + 32 * ps][ch * 8]) = v;
    }
    __syncthreads();
#pragma unroll
    for (int ps = 0; ps < 2; ++ps) {
        const int cl = rr + 32 * ps, c = c0 + cl, r = r0 + ch * 8;
        if (c < C && r < Rpad) {
            unsigned w[4];
#pragma unroll
            for (int e = 0; e < 4; ++e)
                w[e] = (unsigned)tile[ch * 8 + 2 * e][cl] | ((unsigned)tile[ch * 8 + 2 * e + 1][cl] << 16);
            *reinterpret_cast<uint4*>(out + (size_t)c * ldo + r) = make_uint4(w[0], w[1], w[2], w[3]);
        }
    }
}

// ---------------------------------------------------------------------------------------------
// Column sums, deterministic two-stage: part[blk][n] = sum of rows [blk*cs, (blk+1)*cs), then
// out[n] = scale * sum_blk part[blk][n] (+ out[n] when accumulate).  Blocks of 64 columns x 4 row
// lanes (a wave reads 64 consecutive columns of one row), fixed summation order.
template <typename TI>
__global__ __launch_bounds__(256) void colsum_part_k(float* __restrict__ part, const TI* __restrict__ in, long ld,
                                                     int M, int N, int cs) {
    __shared__ float red[4][64];
    const int c = threadIdx.x & 63, r4 = threadIdx.x >> 6;
    const int n = blockIdx.x * 64 + c;
    const int m0 = blockIdx.y * cs, m1 = min(M, m0 + cs);
    float a0 = 0.f, a1 = 0.f;
    if (n < N) {
        int m = m0 + r4;
        for (; m + 4 < m1; m += 8) {
            a0 += ld_f(in + (size_t)m * ld + n);
            a1 += ld_f(in + (size_t)(m + 4) * ld + n);
        }
        if (m < m1) a0 += ld_f(in + (size_t)m * ld + n);
    }
    red[r4][c] = a0 + a1;
    __syncthreads();
    if (r4 == 0 && n < N) part[(size_t)blockIdx.y * N + n] = (red[0][c] + red[1][c]) + (red[2][c] + red[3][c]);
}
__global__ __launch_bounds__(256) void colsum_finish_k(float* __restrict__ out, const float* __restrict__ part,
                                                       int nb, int N, float scale, int accumulate) {
    __shared__ float red[4][64];
    const int c = threadIdx.x & 63, r4 = threadIdx.x >> 6;
    const int n = blockIdx.x * 64 + c;
    // eight independent accumulators (eight loads in flight per lane), combined in a fixed order
    float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (n < N) {
        int b = r4;
        for (; b + 28 < nb; b += 32)
#pragma unroll
            for (int u = 0; u < 8; ++u) a[u] += part[(size_t)(b + 4 * u) * N + n];
        for (int u = 0; b < nb; b += 4, ++u) a[u] += part[(size_t)b * N + n];
    }
    red[r4][c] = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
    __syncthreads();
    if (r4 == 0 && n < N) {
        const float s = (red[0][c] + red[1][c]) + (red[2][c] + red[3][c]);
        out[n] = (accumulate ? out[n] : 0.f) + scale * s;
    }
}

// ---------------------------------------------------------------------------------------------
// LayerNorm backward, one wave per row (element e = c*256 + lane*4 .. +3, as layernorm_k):
//   xh = (x - mu) * rstd;  g = dy * w;  dx = rstd * (g - mean(g) - xh * mean(g * xh))
//   dres[row] (+)= dx;  part_w[blk] += dy * xh;  part_b[blk] += dy
// rows != null: x and dres rows are rows[i] (EOT pooling), dy row is i.
// dres_b (nullable): bf16 copy of the updated dres row (the next dX GEMM's operand); part_r (nullable):
// per-block column sums of the updated dres (the bias gradient of the GEMM that produced the residual:
// c_proj / out_proj, as the colsum of dres, fused)
constexpr int LNB_ROWS = 64;   // rows per block (partial dw/db per block)
// DYB: dy is bf16 (the dX GEMMs' output, as autocast's bf16 matmul gradients), read 8 B per 4 values
template <int NC, bool DYB>
__global__ __launch_bounds__(256) void ln_bwd_k(float* __restrict__ dres, const float* __restrict__ x,
                                                const void* __restrict__ dyv, long ldy, const float* __restrict__ w,
                                                const int* __restrict__ rows, int n, float* __restrict__ part_w,
                                                float* __restrict__ part_b, int accumulate, bf16_t* __restrict__ dres_b,
                                                float* __restrict__ part_r) {
    constexpr int D = NC * 256;
    __shared__ float red[3][4][D];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    float4 aw[NC], ab[NC], ar[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) aw[c] = ab[c] = ar[c] = make_float4(0.f, 0.f, 0.f, 0.f);
    const int r0 = blockIdx.x * LNB_ROWS;
    for (int i = r0 + wave; i < min(n, r0 + LNB_ROWS); i += 4) {
        const long xr = rows ? rows[i] : i;
        float4 v[NC], g[NC], d[NC];
        float s = 0.f;
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            const int e = c * 256 + lane * 4;
            v[c] = *reinterpret_cast<const float4*>(x + xr * D + e);
            if constexpr (DYB) {
                const uint2 u = *reinterpret_cast<const uint2*>(static_cast<const bf16_t*>(dyv) + (long)i * ldy + e);
                d[c] = make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u),
                                   __uint_as_float(u.y << 16), __uint_as_float(u.y & 0xffff0000u));
            } else {
                d[c] = *reinterpret_cast<const float4*>(static_cast<const float*>(dyv) + (long)i * ldy + e);
            }
            s += (v[c].x + v[c].y) + (v[c].z + v[c].w);
        }
        const float mean = wave_sum(s) / (float)D;
        float q = 0.f;
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            v[c].x -= mean; v[c].y -= mean; v[c].z -= mean; v[c].w -= mean;
            q += (v[c].x * v[c].x + v[c].y * v[c].y) + (v[c].z * v[c].z + v[c].w * v[c].w);
        }
        const float rstd = rsqrtf(wave_sum(q) / (float)D + 1e-5f);
        float sg = 0.f, sgx = 0.f;
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            const int e = c * 256 + lane * 4;
            const float4 ww = *reinterpret_cast<const float4*>(w + e);
            v[c].x *= rstd; v[c].y *= rstd; v[c].z *= rstd; v[c].w *= rstd;       // xh
            g[c] = make_float4(d[c].x * ww.x, d[c].y * ww.y, d[c].z * ww.z, d[c].w * ww.w);
            sg += (g[c].x + g[c].y) + (g[c].z + g[c].w);
            sgx += (g[c].x * v[c].x + g[c].y * v[c].y) + (g[c].z * v[c].z + g[c].w * v[c].w);
            aw[c].x += d[c].x * v[c].x; aw[c].y += d[c].y * v[c].y; aw[c].z += d[c].z * v[c].z; aw[c].w += d[c].w * v[c].w;
            ab[c].x += d[c].x; ab[c].y += d[c].y; ab[c].z += d[c].z; ab[c].w += d[c].w;
        }
        const float mg = wave_sum(sg) / (float)D, mgx = wave_sum(sgx) / (float)D;
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            const int e = c * 256 + lane * 4;
            float4* o = reinterpret_cast<float4*>(dres + xr * D + e);
            float4 dx = make_float4(rstd * (g[c].x - mg - v[c].x * mgx), rstd * (g[c].y - mg - v[c].y * mgx),
                                    rstd * (g[c].z - mg - v[c].z * mgx), rstd * (g[c].w - mg - v[c].w * mgx));
            if (accumulate) {
                const float4 old = *o;
                dx.x += old.x; dx.y += old.y; dx.z += old.z; dx.w += old.w;
            }
            *o = dx;
            ar[c].x += dx.x; ar[c].y += dx.y; ar[c].z += dx.z; ar[c].w += dx.w;
            if (dres_b) {
                uint2 hb;
                hb.x = (uint32_t)f2bf(dx.x) | ((uint32_t)f2bf(dx.y) << 16);
                hb.y = (uint32_t)f2bf(dx.z) | ((uint32_t)f2bf(dx.w) << 16);
                *reinterpret_cast<uint2*>(dres_b + xr * D + e) = hb;
            }
        }
    }
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        const int e = c * 256 + lane * 4;
        *reinterpret_cast<float4*>(&red[0][wave][e]) = aw[c];
        *reinterpret_cast<float4*>(&red[1][wave][e]) = ab[c];
        *reinterpret_cast<float4*>(&red[2][wave][e]) = ar[c];
    }
    __syncthreads();
    for (int e = threadIdx.x; e < D; e += 256) {
        part_w[(size_t)blockIdx.x * D + e] = (red[0][0][e] + red[0][1][e]) + (red[0][2][e] + red[0][3][e]);
        part_b[(size_t)blockIdx.x * D + e] = (red[1][0][e] + red[1][1][e]) + (red[1][2][e] + red[1][3][e]);
        if (part_r) part_r[(size_t)blockIdx.x * D + e] = (red[2][0][e] + red[2][1][e]) + (red[2][2][e] + red[2][3][e]);
    }
}

// ---------------------------------------------------------------------------------------------
// Activation forward (h = act(pre)) and backward (dpre = dh * act'(pre)), bf16, 8 per thread.
template <int ACT, bool BWD>
__global__ __launch_bounds__(256) void act_k(bf16_t* __restrict__ out, const bf16_t* __restrict__ pre,
                                             const bf16_t* __restrict__ dh, long n8) {
    const long i = (long)blockIdx.x * 256 + threadIdx.x;
    if (i >= n8) return;
    const uint4 pv = reinterpret_cast<const uint4*>(pre)[i];
    const bf16_t* ps = reinterpret_cast<const bf16_t*>(&pv);
    uint4 dv;
    if constexpr (BWD) dv = reinterpret_cast<const uint4*>(dh)[i];
    const bf16_t* ds = reinterpret_cast<const bf16_t*>(&dv);
    uint4 ov;
    bf16_t* os = reinterpret_cast<bf16_t*>(&ov);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const float x = bf2f(ps[k]);
        float y;
        if constexpr (BWD) y = bf2f(ds[k]) * (ACT == ACT_QGELU ? qgelu_grad(x) : gelu_grad(x));
        else y = apply_act<ACT>(x);
        os[k] = f2bf(y);
    }
    reinterpret_cast<uint4*>(out)[i] = ov;
}

// Activation backward fused with the bias gradient of the GEMM that produced `pre` (c_fc): out = dh *
// act'(pre) (in place allowed), part[blk][n] = sum over the block's rows of the bf16-rounded out (the
// values the old separate colsum read).  Block = 64 column chunks of 8 (512 columns) x 4 row lanes,
// rows [blk * cs, (blk + 1) * cs); fixed summation order.  N % 8 == 0.
template <int ACT>
__global__ __launch_bounds__(256) void act_bwd_colsum_k(bf16_t* out, const bf16_t* __restrict__ pre,
                                                        const bf16_t* dh, int M, int N, int cs,
                                                        float* __restrict__ part) {
    __shared__ float red[4][512];
    const int c8 = threadIdx.x & 63, r4 = threadIdx.x >> 6;
    const int n = blockIdx.x * 512 + c8 * 8;
    const int m0 = blockIdx.y * cs, m1 = min(M, m0 + cs);
    float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    // one row: out = dh * act'(pre), a += the bf16-rounded out (rows summed in order m0 + r4, +4, ...)
    auto row = [&](const uint4& pv, const uint4& dv, size_t o) {
        const bf16_t* ps = reinterpret_cast<const bf16_t*>(&pv);
        const bf16_t* ds = reinterpret_cast<const bf16_t*>(&dv);
        uint4 ov;
        bf16_t* os = reinterpret_cast<bf16_t*>(&ov);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const float x = bf2f(ps[k]);
            os[k] = f2bf(bf2f(ds[k]) * (ACT == ACT_QGELU ? qgelu_grad(x) : gelu_grad(x)));
            a[k] += bf2f(os[k]);
        }
        *reinterpret_cast<uint4*>(out + o) = ov;
    };
    if (n < N) {
        int m = m0 + r4;
        for (; m + 4 < m1; m += 8) {          // two rows' loads in flight per lane
            const size_t o0 = (size_t)m * N + n, o1 = o0 + (size_t)4 * N;
            const uint4 p0 = *reinterpret_cast<const uint4*>(pre + o0), d0 = *reinterpret_cast<const uint4*>(dh + o0);
            const uint4 p1 = *reinterpret_cast<const uint4*>(pre + o1), d1 = *reinterpret_cast<const uint4*>(dh + o1);
            row(p0, d0, o0);
            row(p1, d1, o1);
        }
        if (m < m1) {
            const size_t o = (size_t)m * N + n;
            row(*reinterpret_cast<const uint4*>(pre + o), *reinterpret_cast<const uint4*>(dh + o), o);
        }
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) red[r4][c8 * 8 + k] = a[k];
    __syncthreads();
    for (int e = threadIdx.x; e < 512; e += 256) {
        const int nn = blockIdx.x * 512 + e;
        if (nn < N) part[(size_t)blockIdx.y * N + nn] = (red[0][e] + red[1][e]) + (red[2][e] + red[3][e]);
    }
}

// ---------------------------------------------------------------------------------------------
// Attention backward for one (batch, head) per workgroup, L <= 80 (the text context, 77), d = 64,
// on MFMA (v_mfma_f32_16x16x32_bf16).  q arrives pre-scaled (q' = q * log2(e)/8: the forward's
// convention, attention.hip), so S = q' k^T is in log2 units and, with the forward's row
// log-sum-exp lse (log2 units), P = exp2(S - lse) tile by tile -- no row pass.  delta_i = dO_i . O_i:
//   dP = dO V^T;  dS = ln2 * P o (dP - delta);  dq' = dS K;  dk = dS^T q';  dv = P^T dO
// dq' is the gradient w.r.t. the stored (pre-scaled) q; the in_proj chain rule is applied by the
// caller.  LDS (bf16): row-major q', k, v, dO [80][AB_LD]; transposed q'^T, k^T, dO^T [64][AB_LT];
// P^T, dS, dS^T [80][AB_LT] (contraction dims zero-padded to 96 = 3 x 32).  Row strides are padded
// (72 / 104 elements) so the 16 rows a ds_read_b128 lane group touches fall in distinct banks.
constexpr int AB_L = 80, AB_KP = 96, AB_LD = 72, AB_LT = 104;
__device__ __forceinline__ bf16x8 lds_frag(const bf16_t* base, int ld, int row, int k0) {
    return *reinterpret_cast<const bf16x8*>(base + row * ld + k0);
}
// C[16 x 16 tile (ti, tj)] = sum_k X[ti*16 + r][k] * Y[tj*16 + c][k], k < 32 * nk (both K-contiguous).
// Returns the lane's f32x4: rows ti*16 + 4*(lane>>4) + q (q = 0..3), column tj*16 + (lane&15).
__device__ __forceinline__ f32x4 mfma_tile(const bf16_t* X, int ldx, const bf16_t* Y, int ldy, int ti, int tj,
                                           int nk, int lane) {
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    const int r = lane & 15, kc = (lane >> 4) * 8;
    for (int k = 0; k < nk; ++k) {
        const bf16x8 a = lds_frag(X, ldx, ti * 16 + r, k * 32 + kc);
        const bf16x8 b = lds_frag(Y, ldy, tj * 16 + r, k * 32 + kc);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc, 0, 0, 0);
    }
    return acc;
}

__global__ __launch_bounds__(256) void attn_bwd_k(bf16_t* __restrict__ dqkv, const bf16_t* __restrict__ qkv,
                                                  const bf16_t* __restrict__ O, const bf16_t* __restrict__ dO,
                                                  const float* __restrict__ lse, int L, int H, int causal) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    bf16_t* Qs = reinterpret_cast<bf16_t*>(smem);            // [80][AB_LD]
    bf16_t* Ks = Qs + AB_L * AB_LD;
    bf16_t* Vs = Ks + AB_L * AB_LD;
    bf16_t* dOs = Vs + AB_L * AB_LD;
    bf16_t* QT = dOs + AB_L * AB_LD;                         // [64][AB_LT]
    bf16_t* KT = QT + 64 * AB_LT;
    bf16_t* dOT = KT + 64 * AB_LT;
    bf16_t* PT = dOT + 64 * AB_LT;                           // [80][AB_LT]
    bf16_t* dS = PT + AB_L * AB_LT;
    bf16_t* dST = dS + AB_L * AB_LT;
    float* delta = reinterpret_cast<float*>(dST + AB_L * AB_LT);   // [80]
    float* lrow = delta + AB_L;                                     // [80]

    const int bh = blockIdx.x, b = bh / H, h = bh - b * H;
    const int D = H * 64, ld = 3 * D;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    // zero the contraction padding of the transposed / P / dS images: columns 16 nt .. AB_KP - 1 of
    // their 3 x 64 + 3 x 80 rows (every column below 16 nt is written below: zero rows for i >= L,
    // p = dS = 0 for masked entries of the nt x nt score tiles); 16-B chunks
    {
        const int c0 = ((L + 15) / 16) * 16, nch = (AB_KP - c0) / 8;
        for (int e = tid; e < (3 * 64 + 3 * AB_L) * nch; e += 256)
            *reinterpret_cast<uint4*>(QT + (e / nch) * AB_LT + c0 + (e % nch) * 8) = make_uint4(0, 0, 0, 0);
    }
    if (tid < AB_L) lrow[tid] = tid < L ? lse[(size_t)bh * L + tid] : 0.f;
    __syncthreads();
    // load q', k, v, dO rows (16 B per thread-chunk) + delta_i = dO_i . O_i
    for (int e = tid; e < AB_L * 8; e += 256) {
        const int i = e >> 3, c = (e & 7) * 8;
        uint4 q = make_uint4(0, 0, 0, 0), k = q, v = q, g = q, o = q;
        if (i < L) {
            const size_t row = (size_t)(b * L + i);
            q = *reinterpret_cast<const uint4*>(qkv + row * ld + h * 64 + c);
            k = *reinterpret_cast<const uint4*>(qkv + row * ld + D + h * 64 + c);
            v = *reinterpret_cast<const uint4*>(qkv + row * ld + 2 * D + h * 64 + c);
            g = *reinterpret_cast<const uint4*>(dO + row * D + h * 64 + c);
            o = *reinterpret_cast<const uint4*>(O + row * D + h * 64 + c);
        }
        *reinterpret_cast<uint4*>(Qs + i * AB_LD + c) = q;
        *reinterpret_cast<uint4*>(Ks + i * AB_LD + c) = k;
        *reinterpret_cast<uint4*>(Vs + i * AB_LD + c) = v;
        *reinterpret_cast<uint4*>(dOs + i * AB_LD + c) = g;
        const bf16_t* qs = reinterpret_cast<const bf16_t*>(&q);
        const bf16_t* ks = reinterpret_cast<const bf16_t*>(&k);
        const bf16_t* gs = reinterpret_cast<const bf16_t*>(&g);
        const bf16_t* os = reinterpret_cast<const bf16_t*>(&o);
        float part = 0.f;
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            QT[(c + t) * AB_LT + i] = qs[t];
            KT[(c + t) * AB_LT + i] = ks[t];
            dOT[(c + t) * AB_LT + i] = gs[t];
            part += bf2f(gs[t]) * bf2f(os[t]);
        }
        // the 8 chunks of row i are 8 consecutive lanes of one wave (640 = 2.5 x 256: whole waves)
        part += __shfl_xor(part, 1, 64);
        part += __shfl_xor(part, 2, 64);
        part += __shfl_xor(part, 4, 64);
        if ((e & 7) == 0) delta[i] = part;
    }
    __syncthreads();
    const int nt = (L + 15) / 16;
    // per 16 x 16 tile: S = q' k^T -> P = exp2(S - lse) (masked) -> dP = dO V^T -> dS
    for (int t = wave; t < nt * nt; t += 4) {
        const int ti = t / nt, tj = t - ti * nt;
        const f32x4 sv = mfma_tile(Qs, AB_LD, Ks, AB_LD, ti, tj, 2, lane);
        const f32x4 dp = mfma_tile(dOs, AB_LD, Vs, AB_LD, ti, tj, 2, lane);
        const int j = tj * 16 + (lane & 15);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int i = ti * 16 + 4 * (lane >> 4) + q;
            const bool ok = i < L && j < L && !(causal && j > i);
            const float p = ok ? exp2f(sv[q] - lrow[i]) : 0.f;
            const float ds = ok ? 0.69314718055994531f * p * (dp[q] - delta[i]) : 0.f;
            PT[j * AB_LT + i] = f2bf(p);
            const bf16_t v = f2bf(ds);
            dS[i * AB_LT + j] = v;
            dST[j * AB_LT + i] = v;
        }
    }
    __syncthreads();
    // dq' = dS K (contract j: X = dS [i][j], Y = K^T [d][j]); dk = dS^T q' (X = dS^T, Y = q'^T);
    // dv = P^T dO (X = P^T [j][i], Y = dO^T [d][i]).  16 x 16 output tiles: nt x 4 per product.
    const int nkk = (L + 31) / 32;
    for (int t = wave; t < 3 * nt * 4; t += 4) {
        const int which = t / (nt * 4), tt = t - which * nt * 4;
        const int ti = tt >> 2, tj = tt & 3;
        const bf16_t* X = which == 0 ? dS : which == 1 ? dST : PT;
        const bf16_t* Y = which == 0 ? KT : which == 1 ? QT : dOT;
        const f32x4 r = mfma_tile(X, AB_LT, Y, AB_LT, ti, tj, nkk, lane);
        const int col = which * D + h * 64 + tj * 16 + (lane & 15);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int i = ti * 16 + 4 * (lane >> 4) + q;
            if (i < L) dqkv[(size_t)(b * L + i) * ld + col] = f2bf(r[q]);
        }
    }
}

// ---------------------------------------------------------------------------------------------
// Attention backward, v2 (default; CE_ATTN_BWD=1 / ce_set_attn_bwd_variant(1) keeps attn_bwd_k): the
// same arithmetic without the transposed LDS copies.  Every operand a product contracts over its
// image's ROW index comes from ds_read_b64_tr_b16 on the row-major image (guide T10: lane 4q+p of a
// 16-lane group addresses row r0 + q, columns c0 + 4p .. +3; lane i receives column c0 + i of the 4
// rows), so q', k, v, dO are staged once with 16-B stores and P, dS once each: 73 KB of LDS instead
// of 136 KB, two workgroups per CU.  Contractions over i / j run to K = 16 * ceil(L / 16) (80 at L = 77:
// two 16x16x32 steps + one 16x16x16 step; rows L .. K-1 of every image are zero).
constexpr int AB2_LP = 88;     // P / dS row stride (elements): K = 80 columns + pad
__device__ __forceinline__ s16x4 tr4(const bf16_t* img, int ld, int r0, int c0, int lane) {
    const int li = lane & 15;
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (CE_LDS s16x4*)(img + (size_t)(r0 + (li >> 2)) * ld + c0 + 4 * (li & 3)));
}
// operand fragments of a 16-row (or column) block m0 of a product contracting over k:
//   TR = false: image [m][k] (k contiguous);  TR = true: image [k][m] (m contiguous)
template <bool TR>
__device__ __forceinline__ bf16x8 frag8(const bf16_t* img, int ld, int m0, int k0, int lane) {
    const int g = lane >> 4;
    if constexpr (!TR) {
        return *reinterpret_cast<const bf16x8*>(img + (size_t)(m0 + (lane & 15)) * ld + k0 + 8 * g);
    } else {
        const s16x4 lo = tr4(img, ld, k0 + 8 * g, m0, lane), hi = tr4(img, ld, k0 + 8 * g + 4, m0, lane);
        typedef __attribute__((ext_vector_type(8))) short s16x8;
        return __builtin_bit_cast(bf16x8, (s16x8)__builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
    }
}
template <bool TR>
__device__ __forceinline__ s16x4 frag4(const bf16_t* img, int ld, int m0, int k0, int lane) {
    const int g = lane >> 4;
    if constexpr (!TR) return *reinterpret_cast<const s16x4*>(img + (size_t)(m0 + (lane & 15)) * ld + k0 + 4 * g);
    else return tr4(img, ld, k0 + 4 * g, m0, lane);
}
// C[16 x 16 tile at (m0, n0)] = sum_{k < K} Xop[m][k] Yop[n][k], K a multiple of 16; the lane's f32x4 =
// rows m0 + 4 * (lane >> 4) + q, column n0 + (lane & 15)
template <bool XT, bool YT>
__device__ __forceinline__ f32x4 mfma_tile2(const bf16_t* X, int ldx, const bf16_t* Y, int ldy, int m0, int n0, int K,
                                            int lane) {
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    int k0 = 0;
    for (; k0 + 32 <= K; k0 += 32)
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag8<XT>(X, ldx, m0, k0, lane), frag8<YT>(Y, ldy, n0, k0, lane),
                                                      acc, 0, 0, 0);
    if (k0 < K)
        acc = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(frag4<XT>(X, ldx, m0, k0, lane), frag4<YT>(Y, ldy, n0, k0, lane),
                                                        acc, 0, 0, 0);
    return acc;
}

// bpart (nullable): [B][3D] per-caption column sums of the bf16-rounded dq' | dk | dv (the in_proj
// bias gradient before the caller's sum over captions): wave w owns column block tj = w of every
// product (t = w, w + 4, ... walks ti for fixed tj), so each column is summed in one fixed order
__global__ __launch_bounds__(256, 2) void attn_bwd2_k(bf16_t* __restrict__ dqkv, const bf16_t* __restrict__ qkv,
                                                      const bf16_t* __restrict__ O, const bf16_t* __restrict__ dO,
                                                      const float* __restrict__ lse, int L, int H, int causal,
                                                      float* __restrict__ bpart) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    bf16_t* Qs = reinterpret_cast<bf16_t*>(smem);            // [80][AB_LD]
    bf16_t* Ks = Qs + AB_L * AB_LD;
    bf16_t* Vs = Ks + AB_L * AB_LD;
    bf16_t* dOs = Vs + AB_L * AB_LD;
    bf16_t* Ps = dOs + AB_L * AB_LD;                         // [80][AB2_LP]  P[i][j]
    bf16_t* dSs = Ps + AB_L * AB2_LP;                        // [80][AB2_LP]  dS[i][j]
    float* delta = reinterpret_cast<float*>(dSs + AB_L * AB2_LP);   // [80]
    float* lrow = delta + AB_L;                                      // [80]

    const int bh = blockIdx.x, b = bh / H, h = bh - b * H;
    const int D = H * 64, ld = 3 * D;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int nt = (L + 15) / 16, K = nt * 16;
    if (tid < AB_L) lrow[tid] = tid < L ? lse[(size_t)bh * L + tid] : 0.f;
    // q', k, v, dO rows (zero past L) + delta_i = dO_i . O_i
    for (int e = tid; e < AB_L * 8; e += 256) {
        const int i = e >> 3, c = (e & 7) * 8;
        uint4 q = make_uint4(0, 0, 0, 0), k = q, v = q, g = q, o = q;
        if (i < L) {
            const size_t row = (size_t)(b * L + i);
            q = *reinterpret_cast<const uint4*>(qkv + row * ld + h * 64 + c);
            k = *reinterpret_cast<const uint4*>(qkv + row * ld + D + h * 64 + c);
            v = *reinterpret_cast<const uint4*>(qkv + row * ld + 2 * D + h * 64 + c);
            g = *reinterpret_cast<const uint4*>(dO + row * D + h * 64 + c);
            o = *reinterpret_cast<const uint4*>(O + row * D + h * 64 + c);
        }
        *reinterpret_cast<uint4*>(Qs + i * AB_LD + c) = q;
        *reinterpret_cast<uint4*>(Ks + i * AB_LD + c) = k;
        *reinterpret_cast<uint4*>(Vs + i * AB_LD + c) = v;
        *reinterpret_cast<uint4*>(dOs + i * AB_LD + c) = g;
        const bf16_t* gs = reinterpret_cast<const bf16_t*>(&g);
        const bf16_t* os = reinterpret_cast<const bf16_t*>(&o);
        float part = 0.f;
#pragma unroll
        for (int t = 0; t < 8; ++t) part += bf2f(gs[t]) * bf2f(os[t]);
        part += __shfl_xor(part, 1, 64);
        part += __shfl_xor(part, 2, 64);
        part += __shfl_xor(part, 4, 64);
        if ((e & 7) == 0) delta[i] = part;
    }
    __syncthreads();
    // per 16 x 16 tile: S = q' k^T -> P = exp2(S - lse) (masked) -> dP = dO V^T -> dS
    for (int t = wave; t < nt * nt; t += 4) {
        const int ti = t / nt, tj = t - ti * nt;
        const f32x4 sv = mfma_tile2<false, false>(Qs, AB_LD, Ks, AB_LD, ti * 16, tj * 16, 64, lane);
        const f32x4 dp = mfma_tile2<false, false>(dOs, AB_LD, Vs, AB_LD, ti * 16, tj * 16, 64, lane);
        const int j = tj * 16 + (lane & 15);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int i = ti * 16 + 4 * (lane >> 4) + q;
            const bool ok = i < L && j < L && !(causal && j > i);
            const float p = ok ? exp2f(sv[q] - lrow[i]) : 0.f;
            const float ds = ok ? 0.69314718055994531f * p * (dp[q] - delta[i]) : 0.f;
            Ps[i * AB2_LP + j] = f2bf(p);
            dSs[i * AB2_LP + j] = f2bf(ds);
        }
    }
    __syncthreads();
    // dq'[i][d] = sum_j dS[i][j] k[j][d];  dk[j][d] = sum_i dS[i][j] q'[i][d];  dv[j][d] = sum_i P[i][j] dO[i][d]
    float csum = 0.f;
    for (int t = wave; t < 3 * nt * 4; t += 4) {
        const int which = t / (nt * 4), tt = t - which * nt * 4;
        const int m0 = (tt >> 2) * 16, n0 = (tt & 3) * 16;
        f32x4 r;
        if (which == 0) r = mfma_tile2<false, true>(dSs, AB2_LP, Ks, AB_LD, m0, n0, K, lane);
        else if (which == 1) r = mfma_tile2<true, true>(dSs, AB2_LP, Qs, AB_LD, m0, n0, K, lane);
        else r = mfma_tile2<true, true>(Ps, AB2_LP, dOs, AB_LD, m0, n0, K, lane);
        const int col = which * D + h * 64 + n0 + (lane & 15);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int i = m0 + 4 * (lane >> 4) + q;
            if (i < L) {
                const bf16_t v = f2bf(r[q]);
                dqkv[(size_t)(b * L + i) * ld + col] = v;
                csum += bf2f(v);
            }
        }
        if (bpart && (tt >> 2) == nt - 1) {       // last row tile of this column block: reduce, store
            csum += __shfl_xor(csum, 16, 64);
            csum += __shfl_xor(csum, 32, 64);
            if (lane < 16) bpart[(size_t)b * 3 * D + col] = csum;
            csum = 0.f;
        }
    }
}

// ---------------------------------------------------------------------------------------------
// Attention backward, v3 (default; ce_set_attn_bwd_variant(2) keeps v2): v2's arithmetic with
//  * the causal structure used: phase 1 runs only the score tiles on or below the diagonal (15 of 25
//    at L = 77), and each phase-2 product contracts only over the blocks that can be non-zero — dq'
//    row block ti over key blocks 0..ti, dk / dv key block tj over query blocks tj..nt-1 (180 instead
//    of 300 16-deep MFMA steps at L = 77); every skipped product term is an exact zero (P = dS = 0
//    above the diagonal), so the sums are v2's up to the MFMA step split;
//  * all 15 row loads of a thread issued before the first use (v2 waits per 5);
//  * the outputs staged in LDS and written as whole 128-B rows (16 B per lane) instead of 2-byte
//    stores of 4 rows x 32 B per wave instruction.
template <bool XT, bool YT>
__device__ __forceinline__ f32x4 mfma_tile3(const bf16_t* X, int ldx, const bf16_t* Y, int ldy, int m0, int n0, int k0,
                                            int k1, int lane) {
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (; k0 + 32 <= k1; k0 += 32)
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag8<XT>(X, ldx, m0, k0, lane), frag8<YT>(Y, ldy, n0, k0, lane),
                                                      acc, 0, 0, 0);
    if (k0 < k1)
        acc = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(frag4<XT>(X, ldx, m0, k0, lane), frag4<YT>(Y, ldy, n0, k0, lane),
                                                        acc, 0, 0, 0);
    return acc;
}

__global__ __launch_bounds__(256, 2) void attn_bwd3_k(bf16_t* __restrict__ dqkv, const bf16_t* __restrict__ qkv,
                                                      const bf16_t* __restrict__ O, const bf16_t* __restrict__ dO,
                                                      const float* __restrict__ lse, int L, int H, int causal,
                                                      float* __restrict__ bpart) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    bf16_t* Qs = reinterpret_cast<bf16_t*>(smem);            // [80][AB_LD]
    bf16_t* Ks = Qs + AB_L * AB_LD;
    bf16_t* Vs = Ks + AB_L * AB_LD;
    bf16_t* dOs = Vs + AB_L * AB_LD;
    bf16_t* Ps = dOs + AB_L * AB_LD;                         // [80][AB2_LP]  P[i][j]
    bf16_t* dSs = Ps + AB_L * AB2_LP;                        // [80][AB2_LP]  dS[i][j]
    float* delta = reinterpret_cast<float*>(dSs + AB_L * AB2_LP);   // [80]
    float* lrow = delta + AB_L;                                      // [80]
    bf16_t* Out = Qs;                                        // [3][80][64], after phase 2

    const int bh = blockIdx.x, b = bh / H, h = bh - b * H;
    const int D = H * 64, ld = 3 * D;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int nt = (L + 15) / 16, K = nt * 16;
    if (tid < AB_L) lrow[tid] = tid < L ? lse[(size_t)bh * L + tid] : 0.f;
    // q', k, v, dO rows (zero past L) + delta_i = dO_i . O_i; the 3 chunks of a thread loaded first
    {
        uint4 q[3], k[3], v[3], g[3], o[3];
#pragma unroll
        for (int u = 0; u < 3; ++u) {
            const int e = tid + 256 * u, i = e >> 3, c = (e & 7) * 8;
            q[u] = k[u] = v[u] = g[u] = o[u] = make_uint4(0, 0, 0, 0);
            if (e < AB_L * 8 && i < L) {
                const size_t row = (size_t)(b * L + i);
                q[u] = *reinterpret_cast<const uint4*>(qkv + row * ld + h * 64 + c);
                k[u] = *reinterpret_cast<const uint4*>(qkv + row * ld + D + h * 64 + c);
                v[u] = *reinterpret_cast<const uint4*>(qkv + row * ld + 2 * D + h * 64 + c);
                g[u] = *reinterpret_cast<const uint4*>(dO + row * D + h * 64 + c);
                o[u] = *reinterpret_cast<const uint4*>(O + row * D + h * 64 + c);
            }
        }
#pragma unroll
        for (int u = 0; u < 3; ++u) {
            const int e = tid + 256 * u, i = e >> 3, c = (e & 7) * 8;
            if (e >= AB_L * 8) break;       // (u = 2: lanes 128..255 of the block, whole waves)
            *reinterpret_cast<uint4*>(Qs + i * AB_LD + c) = q[u];
            *reinterpret_cast<uint4*>(Ks + i * AB_LD + c) = k[u];
            *reinterpret_cast<uint4*>(Vs + i * AB_LD + c) = v[u];
            *reinterpret_cast<uint4*>(dOs + i * AB_LD + c) = g[u];
            const bf16_t* gs = reinterpret_cast<const bf16_t*>(&g[u]);
            const bf16_t* os = reinterpret_cast<const bf16_t*>(&o[u]);
            float part = 0.f;
#pragma unroll
            for (int t = 0; t < 8; ++t) part += bf2f(gs[t]) * bf2f(os[t]);
            part += __shfl_xor(part, 1, 64);
            part += __shfl_xor(part, 2, 64);
            part += __shfl_xor(part, 4, 64);
            if ((e & 7) == 0) delta[i] = part;
        }
    }
    __syncthreads();
    // phase 1: S = q' k^T -> P = exp2(S - lse) (masked) -> dP = dO V^T -> dS, for the score tiles that
    // hold an unmasked entry (causal: tj <= ti; t enumerates the lower triangle row by row)
    const int ntile = causal ? nt * (nt + 1) / 2 : nt * nt;
    for (int t = wave; t < ntile; t += 4) {
        int ti, tj;
        if (causal) {
            ti = 0;
            while ((ti + 1) * (ti + 2) / 2 <= t) ++ti;
            tj = t - ti * (ti + 1) / 2;
        } else {
            ti = t / nt;
            tj = t - ti * nt;
        }
        const f32x4 sv = mfma_tile3<false, false>(Qs, AB_LD, Ks, AB_LD, ti * 16, tj * 16, 0, 64, lane);
        const f32x4 dp = mfma_tile3<false, false>(dOs, AB_LD, Vs, AB_LD, ti * 16, tj * 16, 0, 64, lane);
        const int j = tj * 16 + (lane & 15);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int i = ti * 16 + 4 * (lane >> 4) + q;
            const bool ok = i < L && j < L && !(causal && j > i);
            const float p = ok ? exp2f(sv[q] - lrow[i]) : 0.f;
            const float ds = ok ? 0.69314718055994531f * p * (dp[q] - delta[i]) : 0.f;
            Ps[i * AB2_LP + j] = f2bf(p);
            dSs[i * AB2_LP + j] = f2bf(ds);
        }
    }
    __syncthreads();
    // phase 2: dq'[i][d] = sum_j dS[i][j] k[j][d];  dk[j][d] = sum_i dS[i][j] q'[i][d];  dv[j][d] = sum_i
    // P[i][j] dO[i][d].  Wave w owns column block w of every product (fixed-order column sums for bpart);
    // results stay in registers (bf16 pairs) until every wave's LDS reads are done
    uint2 res[3][AB_L / 16];
    float csum[3] = {0.f, 0.f, 0.f};
    const int n0 = wave * 16;
#pragma unroll
    for (int which = 0; which < 3; ++which)
#pragma unroll
        for (int ti = 0; ti < AB_L / 16; ++ti) {
            res[which][ti] = make_uint2(0, 0);
            if (ti >= nt) continue;
            const int m0 = ti * 16;
            f32x4 r;
            if (which == 0) r = mfma_tile3<false, true>(dSs, AB2_LP, Ks, AB_LD, m0, n0, 0, causal ? m0 + 16 : K, lane);
            else if (which == 1) r = mfma_tile3<true, true>(dSs, AB2_LP, Qs, AB_LD, m0, n0, causal ? m0 : 0, K, lane);
            else r = mfma_tile3<true, true>(Ps, AB2_LP, dOs, AB_LD, m0, n0, causal ? m0 : 0, K, lane);
            const uint32_t p01 = pack_bf2(r[0], r[1]), p23 = pack_bf2(r[2], r[3]);
            res[which][ti] = make_uint2(p01, p23);
            // column sums of the bf16-rounded values of rows < L (the in_proj bias gradient)
            const int i0 = m0 + 4 * (lane >> 4);
            const float v0 = __uint_as_float(p01 << 16), v1 = __uint_as_float(p01 & 0xffff0000u);
            const float v2 = __uint_as_float(p23 << 16), v3 = __uint_as_float(p23 & 0xffff0000u);
            csum[which] += (i0 < L ? v0 : 0.f) + (i0 + 1 < L ? v1 : 0.f) + (i0 + 2 < L ? v2 : 0.f) +
                           (i0 + 3 < L ? v3 : 0.f);
        }
    if (bpart) {
#pragma unroll
        for (int which = 0; which < 3; ++which) {
            float c = csum[which];
            c += __shfl_xor(c, 16, 64);
            c += __shfl_xor(c, 32, 64);
            if (lane < 16) bpart[(size_t)b * 3 * D + which * D + h * 64 + n0 + lane] = c;
        }
    }
    __syncthreads();
    // stage the three [L][64] outputs in LDS, then write whole 128-B rows
#pragma unroll
    for (int which = 0; which < 3; ++which)
#pragma unroll
        for (int ti = 0; ti < AB_L / 16; ++ti) {
            if (ti >= nt) continue;
            const int i0 = ti * 16 + 4 * (lane >> 4), col = n0 + (lane & 15);
            bf16_t* op = Out + ((size_t)which * AB_L + i0) * 64 + col;
            const uint2 w = res[which][ti];
            op[0] = (bf16_t)(w.x & 0xffffu);
            op[64] = (bf16_t)(w.x >> 16);
            op[128] = (bf16_t)(w.y & 0xffffu);
            op[192] = (bf16_t)(w.y >> 16);
        }
    __syncthreads();
    for (int e = tid; e < 3 * L * 8; e += 256) {
        const int which = e / (L * 8), rem = e - which * L * 8, i = rem >> 3, c = (rem & 7) * 8;
        *reinterpret_cast<uint4*>(dqkv + (size_t)(b * L + i) * ld + which * D + h * 64 + c) =
            *reinterpret_cast<const uint4*>(Out + ((size_t)which * AB_L + i) * 64 + c);
    }
}

std::atomic<int> g_attn_bwd_var{kKnobUnset};     // A/B knob (knobs.h)
int attn_bwd_env() { const int v = env_int("CE_ATTN_BWD", 3); return v == 1 || v == 2 ? v : 3; }
int attn_bwd_variant() { return knob_get(g_attn_bwd_var, attn_bwd_env); }

// ---------------------------------------------------------------------------------------------
// Token-embedding gradient, deterministic: (id, row) pairs sorted by id (stable radix sort), one
// workgroup per run of equal ids sums its rows in row order.  Positional gradient: sum over batch.
__global__ __launch_bounds__(256) void iota_ids_k(int* __restrict__ keys, int* __restrict__ vals,
                                                  const int64_t* __restrict__ ids, int n) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < n) {
        keys[i] = (int)ids[i];
        vals[i] = i;
    }
}
// Runs of equal ids are summed chunk by chunk (ECH sorted positions per workgroup): a run that
// starts and ends inside a chunk is written to dtok directly; the pieces of runs crossing chunk
// boundaries go to first[c] (a run continued from before chunk c) / last[c] (a run starting in
// chunk c that continues), and embed_join_k sums each crossing run's pieces in chunk order.
constexpr int ECH = 64;
template <int NC>
__global__ __launch_bounds__(256) void embed_pieces_k(float* __restrict__ dtok, float* __restrict__ first,
                                                      float* __restrict__ last, const int* __restrict__ keys,
                                                      const int* __restrict__ rows, const float* __restrict__ dx,
                                                      int n) {
    constexpr int D = NC * 256;
    const int c = blockIdx.x, c0 = c * ECH, c1 = min(n, c0 + ECH);
    float acc[NC];
    int a = c0;
    while (a < c1) {
        const int id = keys[a];
        int b = a;
#pragma unroll
        for (int q = 0; q < NC; ++q) acc[q] = 0.f;
        for (; b < c1 && keys[b] == id; ++b) {
            const float* src = dx + (size_t)rows[b] * D + threadIdx.x;
#pragma unroll
            for (int q = 0; q < NC; ++q) acc[q] += src[q * 256];
        }
        const bool starts = a == 0 || keys[a - 1] != id;
        const bool ends = b >= n || keys[b] != id;
        float* dst = (starts && ends) ? dtok + (size_t)id * D : (!starts ? first : last) + (size_t)c * D;
#pragma unroll
        for (int q = 0; q < NC; ++q) dst[q * 256 + threadIdx.x] = acc[q];
        a = b;
    }
}
template <int NC>
__global__ __launch_bounds__(256) void embed_join_k(float* __restrict__ dtok, const float* __restrict__ first,
                                                    const float* __restrict__ last, const int* __restrict__ keys,
                                                    int n, int nch) {
    constexpr int D = NC * 256;
    const int c = blockIdx.x, c1 = min(n, (c + 1) * ECH);
    const int id = keys[c1 - 1];
    // owner: the chunk in which the run of its last position starts, when that run continues
    if (c1 >= n || keys[c1] != id) return;
    int a = c1 - 1;
    while (a > c * ECH && keys[a - 1] == id) --a;
    if (a == c * ECH && c > 0 && keys[a - 1] == id) return;   // run started in an earlier chunk
    float acc[NC];
#pragma unroll
    for (int q = 0; q < NC; ++q) acc[q] = last[(size_t)c * D + q * 256 + threadIdx.x];
    for (int cc = c + 1; cc < nch && keys[cc * ECH] == id; ++cc)
#pragma unroll
        for (int q = 0; q < NC; ++q) acc[q] += first[(size_t)cc * D + q * 256 + threadIdx.x];
#pragma unroll
    for (int q = 0; q < NC; ++q) dtok[(size_t)id * D + q * 256 + threadIdx.x] = acc[q];
}

// ---------------------------------------------------------------------------------------------
// F.normalize backward: f = u / max(|u|, 1e-12):  du = (df - f (f . df)) / |u|   (|u| > 1e-12)
__global__ __launch_bounds__(256) void l2norm_bwd_k(float* __restrict__ du, const float* __restrict__ u,
                                                    const float* __restrict__ df, int rows, int D) {
    const int lane = threadIdx.x & 63, r = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= rows) return;
    const float* ur = u + (size_t)r * D;
    const float* gr = df + (size_t)r * D;
    float nn = 0.f;
    for (int e = lane; e < D; e += 64) nn += ur[e] * ur[e];
    const float nrm = sqrtf(wave_sum(nn));
    const float inv = 1.0f / fmaxf(nrm, 1e-12f);
    float fd = 0.f;
    for (int e = lane; e < D; e += 64) fd += ur[e] * inv * gr[e];
    fd = wave_sum(fd);
    for (int e = lane; e < D; e += 64) {
        const float f = ur[e] * inv;
        du[(size_t)r * D + e] = nrm > 1e-12f ? (gr[e] - f * fd) * inv : gr[e] * inv;
    }
}

// ---------------------------------------------------------------------------------------------
// Cross entropy with gradient, one wave per row of logits z [R][C] (z already scaled):
//   valid row (label >= 0): g = wgt * inv_count * (softmax(z) - onehot(label)),
//   loss_row = wgt * inv_count * (logsumexp(z) - z[label]),  gz_row = sum_j g_j z_j
//   ignored row (label -100): g = 0, loss_row = gz_row = 0.
// g may alias z (in place).  Row partials go to rowstat[2][R] and are summed by ce_finish_k.
__global__ __launch_bounds__(256) void ce_grad_k(float* __restrict__ g, const float* __restrict__ z, int R, int C,
                                                 const int64_t* __restrict__ labels, float wgt_inv_count,
                                                 float* __restrict__ rowstat) {
    const int lane = threadIdx.x & 63, r = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= R) return;
    const float* zr = z + (size_t)r * C;
    float* gr = g + (size_t)r * C;
    const long lab = labels[r];
    if (lab == -100 || lab < 0 || lab >= C) {
        // -100 = ignore_index; any other label outside [0, C) (F.cross_entropy raises) poisons the
        // row's gradient and loss with NaN rather than reading past the row
        const float v = lab == -100 ? 0.f : NAN;
        for (int j = lane; j < C; j += 64) gr[j] = v;
        if (lane == 0) { rowstat[r] = v; rowstat[R + r] = v; }
        return;
    }
    float m = -INFINITY;
    for (int j = lane; j < C; j += 64) m = fmaxf(m, zr[j]);
    m = wave_max(m);
    float s = 0.f;
    for (int j = lane; j < C; j += 64) s += __expf(zr[j] - m);
    s = wave_sum(s);
    const float lse = m + __logf(s), is = 1.0f / s;
    const float zl = zr[lab];
    float gz = 0.f;
    for (int j = lane; j < C; j += 64) {
        const float zj = zr[j];
        const float gj = wgt_inv_count * (__expf(zj - m) * is - (j == lab ? 1.0f : 0.0f));
        gz += gj * zj;
        gr[j] = gj;
    }
    gz = wave_sum(gz);
    if (lane == 0) {
        rowstat[r] = wgt_inv_count * (lse - zl);
        rowstat[R + r] = gz;
    }
}
// out[0] += sum_r rowstat[r] (loss), out[1] += sum_r rowstat[R + r] (d loss / d logit_scale)
__global__ __launch_bounds__(256) void ce_finish_k(float* __restrict__ out, const float* __restrict__ rowstat, int R) {
    __shared__ float red[2][4];
    float a = 0.f, c = 0.f;
    for (int r = threadIdx.x; r < R; r += 256) {
        a += rowstat[r];
        c += rowstat[R + r];
    }
    a = wave_sum(a);
    c = wave_sum(c);
    if ((threadIdx.x & 63) == 0) { red[0][threadIdx.x >> 6] = a; red[1][threadIdx.x >> 6] = c; }
    __syncthreads();
    if (threadIdx.x == 0) {
        out[0] += (red[0][0] + red[0][1]) + (red[0][2] + red[0][3]);
        out[1] += (red[1][0] + red[1][1]) + (red[1][2] + red[1][3]);
    }
}

// ---------------------------------------------------------------------------------------------
// AdamW (torch.optim.AdamW, maximize=False, amsgrad=False), f32 master weights:
//   p *= 1 - lr*wd;  m = b1 m + (1-b1) g;  v = b2 v + (1-b2) g^2;
//   p -= lr/(1-b1^t) * m / (sqrt(v)/sqrt(1-b2^t) + eps)
__global__ __launch_bounds__(256) void adamw_k(float* __restrict__ p, const float* __restrict__ g,
                                               float* __restrict__ m, float* __restrict__ v, long n, float lr,
                                               float b1, float b2, float eps, float wd, float bc1, float bc2_sqrt) {
    const long i = (long)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const float gi = g[i];
    float pi = p[i] * (1.0f - lr * wd);
    const float mi = b1 * m[i] + (1.0f - b1) * gi;
    const float vi = b2 * v[i] + (1.0f - b2) * gi * gi;
    m[i] = mi;
    v[i] = vi;
    pi -= (lr / bc1) * mi / (sqrtf(vi) / bc2_sqrt + eps);
    p[i] = pi;
}

// Engine weight copy from an f32 master: rows < scale_rows are multiplied by `scale` (the q
// rows of in_proj carry the attention scale, capi.hip ce_load_weights), output f32 or bf16.
template <bool BF16>
__global__ __launch_bounds__(256) void weight_from_master_k(void* __restrict__ out, const float* __restrict__ src,
                                                            long n, long row_len, long scale_rows, float scale) {
    const long i = (long)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    float x = src[i];
    if (i / row_len < scale_rows) x *= scale;
    if constexpr (BF16) static_cast<bf16_t*>(out)[i] = f2bf(x);
    else static_cast<float*>(out)[i] = x;
}

__global__ __launch_bounds__(256) void scale_k(float* __restrict__ x, long n, float s) {
    const long i = (long)blockIdx.x * 256 + threadIdx.x;
    if (i < n) x[i] *= s;
}

__global__ __launch_bounds__(256) void axpy_k(float* __restrict__ y, const float* __restrict__ x, long n, float a) {
    const long i = (long)blockIdx.x * 256 + threadIdx.x;
    if (i < n) y[i] += a * x[i];
}

__global__ __launch_bounds__(256) void cast_f32_bf16_k(bf16_t* __restrict__ out, const float* __restrict__ in, long n) {
    const long i = (long)blockIdx.x * 256 + threadIdx.x;
    if (i < n) out[i] = f2bf(in[i]);
}

unsigned blocks(long n, int per = 256) { return (unsigned)((n + per - 1) / per); }

}  // namespace

// ============================================================================================
hipError_t launch_transpose_bf16(bf16_t* out, long ldo, const void* in, bool in_f32, long ldi, int R, int C, int Rpad,
                                 hipStream_t s) {
    if (R <= 0 || C <= 0) return hipSuccess;
    const dim3 grid((unsigned)((std::max(R, Rpad) + 63) / 64), (unsigned)((C + 63) / 64));
    const bool v8 = C % 8 == 0 && Rpad % 8 == 0 && Rpad >= R && ldi % 8 == 0 && ldo % 8 == 0 &&
                    (reinterpret_cast<uintptr_t>(in) & 15) == 0 && (reinterpret_cast<uintptr_t>(out) & 15) == 0;
    if (v8) {
        if (in_f32) hipLaunchKernelGGL((transpose_v8_k<float>), grid, dim3(256), 0, s, out, ldo, (const float*)in, ldi, R, C, Rpad);
        else hipLaunchKernelGGL((transpose_v8_k<bf16_t>), grid, dim3(256), 0, s, out, ldo, (const bf16_t*)in, ldi, R, C, Rpad);
        return hipGetLastError();
    }
    if (in_f32) hipLaunchKernelGGL((transpose_k<float, bf16_t>), grid, dim3(256), 0, s, out, ldo, (const float*)in, ldi, R, C, Rpad);
    else hipLaunchKernelGGL((transpose_k<bf16_t, bf16_t>), grid, dim3(256), 0, s, out, ldo, (const bf16_t*)in, ldi, R, C, Rpad);
    return hipGetLastError();
}
hipError_t launch_transpose_f32(float* out, long ldo, const float* in, long ldi, int R, int C, hipStream_t s) {
    if (R <= 0 || C <= 0) return hipSuccess;
    const dim3 grid((unsigned)((R + 63) / 64), (unsigned)((C + 63) / 64));
    hipLaunchKernelGGL((transpose_k<float, float>), grid, dim3(256), 0, s, out, ldo, in, ldi, R, C, R);
    return hipGetLastError();
}

int colsum_chunk(int M, int N) {
    const int colblocks = (N + 63) / 64;
    const int target = std::max(1, 2048 / colblocks);
    int cs = (M + target - 1) / target;
    cs = std::max(64, (cs + 7) / 8 * 8);
    return cs;
}
long colsum_scratch_floats(int M, int N) {
    const int cs = colsum_chunk(M, N);
    return (long)std::max(1, (M + cs - 1) / cs) * N;
}
hipError_t launch_colsum(float* out, const void* in, bool in_f32, long ld, int M, int N, float scale, bool accumulate,
                         float* scratch, hipStream_t s) {
    if (N <= 0) return hipSuccess;
    const int cs = colsum_chunk(M, N);
    const int nb = std::max(1, (M + cs - 1) / cs);
    const unsigned cb = (unsigned)((N + 63) / 64);
    if (M > 0) {
        const dim3 grid(cb, (unsigned)nb);
        if (in_f32) hipLaunchKernelGGL(colsum_part_k<float>, grid, dim3(256), 0, s, scratch, (const float*)in, ld, M, N, cs);
        else hipLaunchKernelGGL(colsum_part_k<bf16_t>, grid, dim3(256), 0, s, scratch, (const bf16_t*)in, ld, M, N, cs);
    } else {
        (void)hipMemsetAsync(scratch, 0, sizeof(float) * N, s);
    }
    hipLaunchKernelGGL(colsum_finish_k, dim3(cb), dim3(256), 0, s, out, scratch, nb, N, scale, accumulate ? 1 : 0);
    return hipGetLastError();
}

long ln_bwd_scratch_floats(int n, int D) {
    const int nb = (n + LNB_ROWS - 1) / LNB_ROWS;
    return 3L * nb * D + colsum_scratch_floats(nb, D);
}
hipError_t launch_ln_bwd(float* dres, const float* x, const float* dy, long ldy, const float* w, const int* rows, int n,
                         int D, float* dw, float* db, bool accumulate_dx, bool accumulate_dwb, float* scratch,
                         hipStream_t s, bf16_t* dres_b, float* dsum, const bf16_t* dy_b) {
    if (n <= 0) return hipSuccess;
    const int nb = (n + LNB_ROWS - 1) / LNB_ROWS;
    float* pw = scratch;
    float* pb = scratch + (size_t)nb * D;
    float* pr = dsum ? pb + (size_t)nb * D : nullptr;
    const int acc = accumulate_dx ? 1 : 0;
#define CE_LNB(NC) \
    if (dy_b) hipLaunchKernelGGL((ln_bwd_k<NC, true>), dim3(nb), dim3(256), 0, s, dres, x, (const void*)dy_b, ldy, w, rows, n, \
                                 pw, pb, acc, dres_b, pr); \
    else hipLaunchKernelGGL((ln_bwd_k<NC, false>), dim3(nb), dim3(256), 0, s, dres, x, (const void*)dy, ldy, w, rows, n, pw, \
                            pb, acc, dres_b, pr)
    if (D == 768) { CE_LNB(3); }
    else if (D == 1024) { CE_LNB(4); }
    else if (D == 512) { CE_LNB(2); }
    else return hipErrorInvalidValue;
#undef CE_LNB
    float* cscr = pb + 2 * (size_t)nb * D;
    hipError_t e = launch_colsum(dw, pw, true, D, nb, D, 1.0f, accumulate_dwb, cscr, s);
    if (e == hipSuccess) e = launch_colsum(db, pb, true, D, nb, D, 1.0f, accumulate_dwb, cscr, s);
    if (e == hipSuccess && dsum) e = launch_colsum(dsum, pr, true, D, nb, D, 1.0f, false, cscr, s);
    return e;
}

int act_colsum_chunk(int M, int N) {
    const int colblocks = (N + 511) / 512;
    const int target = std::max(1, 1536 / colblocks);
    return std::max(16, (M + target - 1) / target);
}
long act_bwd_colsum_scratch_floats(int M, int N) {
    const long unfused = (long)((M + act_colsum_chunk(M, N) - 1) / act_colsum_chunk(M, N)) * N;
    return std::max(unfused, (long)((M + 127) / 128) * N);
}
hipError_t launch_colsum_finish(float* out, const float* part, int nb, int N, hipStream_t s) {
    if (nb <= 0 || N <= 0) return hipErrorInvalidValue;
    hipLaunchKernelGGL(colsum_finish_k, dim3((unsigned)((N + 63) / 64)), dim3(256), 0, s, out, part, nb, N, 1.0f, 0);
    return hipGetLastError();
}
hipError_t launch_act_bwd_colsum(bf16_t* out, const bf16_t* pre, const bf16_t* dh, int M, int N, int act, float* dbias,
                                 float* scratch, hipStream_t s) {
    if (N % 8 || M <= 0) return hipErrorInvalidValue;
    const int cs = act_colsum_chunk(M, N);
    const int nb = (M + cs - 1) / cs;
    const dim3 grid((unsigned)((N + 511) / 512), (unsigned)nb);
    if (act == ACT_GELU) hipLaunchKernelGGL(act_bwd_colsum_k<ACT_GELU>, grid, dim3(256), 0, s, out, pre, dh, M, N, cs, scratch);
    else if (act == ACT_QGELU) hipLaunchKernelGGL(act_bwd_colsum_k<ACT_QGELU>, grid, dim3(256), 0, s, out, pre, dh, M, N, cs, scratch);
    else return hipErrorInvalidValue;
    hipLaunchKernelGGL(colsum_finish_k, dim3((unsigned)((N + 63) / 64)), dim3(256), 0, s, dbias, scratch, nb, N, 1.0f, 0);
    return hipGetLastError();
}

hipError_t launch_act(bf16_t* out, const bf16_t* pre, const bf16_t* dh, long n, int act, hipStream_t s) {
    if (n % 8) return hipErrorInvalidValue;
    const long n8 = n / 8;
    const dim3 grid(blocks(n8));
#define CE_ACT(A_) \
    if (act == A_) { \
        if (dh) hipLaunchKernelGGL((act_k<A_, true>), grid, dim3(256), 0, s, out, pre, dh, n8); \
        else hipLaunchKernelGGL((act_k<A_, false>), grid, dim3(256), 0, s, out, pre, dh, n8); \
        return hipGetLastError(); }
    CE_ACT(ACT_GELU) CE_ACT(ACT_QGELU)
#undef CE_ACT
    return hipErrorInvalidValue;
}

constexpr size_t kAttnBwd2Lds = (size_t)(4 * AB_L * AB_LD + 2 * AB_L * AB2_LP) * 2 + (size_t)(2 * AB_L) * 4;
constexpr size_t kAttnBwdLds = (size_t)(4 * AB_L * AB_LD + 3 * 64 * AB_LT + 3 * AB_L * AB_LT) * 2 + (size_t)(2 * AB_L) * 4;
hipError_t launch_attention_bwd(bf16_t* dqkv, const bf16_t* qkv, const bf16_t* O, const bf16_t* dO, const float* lse,
                                int B, int L, int H, bool causal, hipStream_t s, float* dbias, float* bpart,
                                float* scratch) {
    if (L <= 0 || L > AB_L || B <= 0 || !lse || (dbias && (!bpart || !scratch))) return hipErrorInvalidValue;
    // dynamic-LDS opt-in, once per device (several host threads may drive several devices)
    static std::atomic<bool> attr[kMaxDevices], attr2[kMaxDevices];
    const int dev = current_device();
    if (!attr[dev].load(std::memory_order_acquire)) {
        (void)hipFuncSetAttribute((const void*)attn_bwd_k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kAttnBwdLds);
        attr[dev].store(true, std::memory_order_release);
    }
    const int var = attn_bwd_variant();
    if (var >= 2) {
        if (!attr2[dev].load(std::memory_order_acquire)) {
            (void)hipFuncSetAttribute((const void*)attn_bwd2_k, hipFuncAttributeMaxDynamicSharedMemorySize,
                                      (int)kAttnBwd2Lds);
            (void)hipFuncSetAttribute((const void*)attn_bwd3_k, hipFuncAttributeMaxDynamicSharedMemorySize,
                                      (int)kAttnBwd2Lds);
            attr2[dev].store(true, std::memory_order_release);
        }
        if (var == 3)
            hipLaunchKernelGGL(attn_bwd3_k, dim3((unsigned)(B * H)), dim3(256), kAttnBwd2Lds, s, dqkv, qkv, O, dO, lse,
                               L, H, causal ? 1 : 0, dbias ? bpart : nullptr);
        else
            hipLaunchKernelGGL(attn_bwd2_k, dim3((unsigned)(B * H)), dim3(256), kAttnBwd2Lds, s, dqkv, qkv, O, dO, lse,
                               L, H, causal ? 1 : 0, dbias ? bpart : nullptr);
        if (dbias)   // in_proj bias gradient: the captions' column sums (two-stage, fixed order)
            return launch_colsum(dbias, bpart, true, 3 * H * 64, B, 3 * H * 64, 1.0f, false, scratch, s);
        return hipGetLastError();
    }
    hipLaunchKernelGGL(attn_bwd_k, dim3((unsigned)(B * H)), dim3(256), kAttnBwdLds, s, dqkv, qkv, O, dO, lse, L, H,
                       causal ? 1 : 0);
    if (dbias) return launch_colsum(dbias, dqkv, false, 3 * H * 64, B * L, 3 * H * 64, 1.0f, false, scratch, s);
    return hipGetLastError();
}

int set_attn_bwd_variant(int v) {
    const int prev = attn_bwd_variant();
    g_attn_bwd_var.store(v == 1 || v == 2 ? v : 3);
    return prev;
}

size_t embed_bwd_scratch_bytes(int B, int ctx, int D) {
    const int n = B * ctx, nch = (n + ECH - 1) / ECH;
    size_t tmp = 0;
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, tmp, (const int*)nullptr, (int*)nullptr, (const int*)nullptr,
                                             (int*)nullptr, n);
    return 4 * sizeof(int) * (size_t)n + 2 * sizeof(float) * (size_t)nch * D +
           sizeof(float) * (size_t)colsum_scratch_floats(B, ctx * D) + tmp + 1024;
}
hipError_t launch_embed_bwd(float* dtok, float* dpos, const float* dx, const int64_t* ids, int B, int ctx, int D,
                            int vocab, void* scratch, size_t scratch_bytes, hipStream_t s) {
    const int n = B * ctx;
    if (n <= 0) return hipSuccess;
    if (D != 512 && D != 768 && D != 1024) return hipErrorInvalidValue;
    const int nch = (n + ECH - 1) / ECH;
    int* k0 = static_cast<int*>(scratch);
    int* v0 = k0 + n;
    int* k1 = v0 + n;
    int* v1 = k1 + n;
    float* first = reinterpret_cast<float*>(v1 + n);
    float* last = first + (size_t)nch * D;
    float* cscr = last + (size_t)nch * D;
    void* tmp = cscr + colsum_scratch_floats(B, ctx * D);
    const size_t used = (size_t)((char*)tmp - (char*)scratch);
    size_t tmp_bytes = scratch_bytes - used;
    hipLaunchKernelGGL(iota_ids_k, dim3(blocks(n)), dim3(256), 0, s, k0, v0, ids, n);
    int bits = 1;
    while ((1 << bits) < vocab) ++bits;
    hipError_t e = hipcub::DeviceRadixSort::SortPairs(tmp, tmp_bytes, k0, k1, v0, v1, n, 0, bits, s);
    if (e != hipSuccess) return e;
    (void)hipMemsetAsync(dtok, 0, sizeof(float) * (size_t)vocab * D, s);
#define CE_EMB(NC_) \
    hipLaunchKernelGGL(embed_pieces_k<NC_>, dim3((unsigned)nch), dim3(256), 0, s, dtok, first, last, k1, v1, dx, n); \
    hipLaunchKernelGGL(embed_join_k<NC_>, dim3((unsigned)nch), dim3(256), 0, s, dtok, first, last, k1, n, nch);
    if (D == 768) { CE_EMB(3) } else if (D == 512) { CE_EMB(2) } else { CE_EMB(4) }
#undef CE_EMB
    // positional: column sums of dx viewed as [B][ctx * D]
    return launch_colsum(dpos, dx, true, (long)ctx * D, B, ctx * D, 1.0f, false, cscr, s);
}

hipError_t launch_l2norm_bwd(float* du, const float* u, const float* df, int rows, int D, hipStream_t s) {
    if (rows <= 0) return hipSuccess;
    hipLaunchKernelGGL(l2norm_bwd_k, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, s, du, u, df, rows, D);
    return hipGetLastError();
}

hipError_t launch_ce_grad(float* g, const float* z, int R, int C, const int64_t* labels, float wgt_inv_count,
                          float* rowstat, float* out2, hipStream_t s) {
    if (R <= 0) return hipSuccess;
    hipLaunchKernelGGL(ce_grad_k, dim3((unsigned)((R + 3) / 4)), dim3(256), 0, s, g, z, R, C, labels, wgt_inv_count,
                       rowstat);
    hipLaunchKernelGGL(ce_finish_k, dim3(1), dim3(256), 0, s, out2, rowstat, R);
    return hipGetLastError();
}

hipError_t launch_adamw(float* p, const float* g, float* m, float* v, long n, float lr, float b1, float b2, float eps,
                        float wd, int step, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    const float bc1 = 1.0f - powf(b1, (float)step);
    const float bc2s = sqrtf(1.0f - powf(b2, (float)step));
    hipLaunchKernelGGL(adamw_k, dim3(blocks(n)), dim3(256), 0, s, p, g, m, v, n, lr, b1, b2, eps, wd, bc1, bc2s);
    return hipGetLastError();
}

hipError_t launch_weight_from_master(void* out, bool bf16, const float* src, long n, long row_len, long scale_rows,
                                     float scale, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    if (bf16) hipLaunchKernelGGL(weight_from_master_k<true>, dim3(blocks(n)), dim3(256), 0, s, out, src, n, row_len, scale_rows, scale);
    else hipLaunchKernelGGL(weight_from_master_k<false>, dim3(blocks(n)), dim3(256), 0, s, out, src, n, row_len, scale_rows, scale);
    return hipGetLastError();
}

hipError_t launch_scale(float* x, long n, float sc, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(scale_k, dim3(blocks(n)), dim3(256), 0, s, x, n, sc);
    return hipGetLastError();
}

hipError_t launch_axpy(float* y, const float* x, long n, float a, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(axpy_k, dim3(blocks(n)), dim3(256), 0, s, y, x, n, a);
    return hipGetLastError();
}

hipError_t launch_cast_bf16(bf16_t* out, const float* in, long n, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(cast_f32_bf16_k, dim3(blocks(n)), dim3(256), 0, s, out, in, n);
    return hipGetLastError();
}

}  // namespace ce
