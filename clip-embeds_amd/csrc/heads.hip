// Small f32 contractions and the fused PACL / SPARC reductions for gfx950.
//
//  * fgemm: batched f32 GEMM on the f32-input matrix cores (64x64 tiles, 32x32x2 f32 MFMA).  Used where the
//    reference keeps f32 and the work is tiny next to the towers: pooled @ proj
//    (transformer.py:830-831, model.py:293-296), contrastive logits scale * I @ T^T
//    (model.py:303-310, loss.py:155-164), PACL text Linear (pacl.py:75-79), SPARC's two einsums
//    (pacl.py:460,472).
//  * pacl_pool: the fused PACL patch-alignment reduction (pacl.py:120-145,199-209): per output row
//    normalise the text vector, stream the image's P projected patches once, compute
//    w_p = 1 or sigmoid(10 * cos(t, [rope](v_p))), accumulate sum_p w_p v_p, L2-normalise.
//  * sparc_weights: per (b,t) row of the similarity: min-max normalise (eps 1e-8), zero entries
//    below sigma, divide by the row sum (+1e-8)  (pacl.py:462-471).
#include "ce_device.h"
#include "ce_kernels.h"

namespace ce {
namespace {

constexpr int FT = 64;    // tile
constexpr int FK = 16;    // k chunk

// 64 x 64 output tile per 256-thread block; wave w computes the 32 x 32 quadrant (w >> 1, w & 1)
// with v_mfma_f32_32x32x2_f32 (f32 in, f32 accumulate: bit-for-bit a k-ordered fmaf chain, i.e.
// the reference's f32 precision at the matrix-core rate; guide §3 'FP32-input MFMA').  LDS holds
// the K-chunk k-major (As[k][m], Bs[k][n]) so lane l reads A[m = l & 31][k = l >> 5] and
// B[k = l >> 5][n = l & 31] for the instruction with consecutive lanes on consecutive words.
// C/D: column = lane & 31, row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5) for register r.
template <bool B_NK>
__global__ __launch_bounds__(256) void fgemm_k(FGemmParams p) {
    __shared__ float As[FK][FT + 4];
    __shared__ float Bs[FK][FT + 4];
    const int z = blockIdx.z;
    const float* A = p.A + (size_t)z * p.sA;
    const float* Bm = p.B + (size_t)z * p.sB;
    float* C = p.C + (size_t)z * p.sC;
    const int i0 = blockIdx.y * FT, j0 = blockIdx.x * FT;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 1, wn = wave & 1;
    f32x16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
    for (int k0 = 0; k0 < p.K; k0 += FK) {
        for (int e = tid; e < FT * FK; e += 256) {
            const int rr = e / FK, kk = e % FK;
            const int gi = i0 + rr, gk = k0 + kk;
            As[kk][rr] = (gi < p.M && gk < p.K) ? A[(size_t)gi * p.lda + gk] : 0.f;
        }
        for (int e = tid; e < FT * FK; e += 256) {
            if constexpr (B_NK) {
                const int cc = e / FK, kk = e % FK;
                const int gj = j0 + cc, gk = k0 + kk;
                Bs[kk][cc] = (gj < p.N && gk < p.K) ? Bm[(size_t)gj * p.ldb + gk] : 0.f;
            } else {
                const int kk = e / FT, cc = e % FT;
                const int gj = j0 + cc, gk = k0 + kk;
                Bs[kk][cc] = (gj < p.N && gk < p.K) ? Bm[(size_t)gk * p.ldb + gj] : 0.f;
            }
        }
        __syncthreads();
#pragma unroll
        for (int kk = 0; kk < FK; kk += 2) {
            const float a = As[kk + (lane >> 5)][wm * 32 + (lane & 31)];
            const float b = Bs[kk + (lane >> 5)][wn * 32 + (lane & 31)];
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
        }
        __syncthreads();
    }
    const int gj = j0 + wn * 32 + (lane & 31);
    if (gj >= p.N) return;
    const float bj = p.bias ? p.bias[gj] : 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int gi = i0 + wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        if (gi >= p.M) continue;
        const float v = acc[r] * p.alpha + bj;
        C[(size_t)gi * p.ldc + gj] = v;
        if (p.Ct) p.Ct[(size_t)gj * p.ldct + gi] = v;
    }
}

// ---- fused PACL pooling -----------------------------------------------------------------
// One 256-thread block per output row; D <= 1024, D % 128 == 0 (768 for ViT-L-14-336).
template <bool VP_BF16, int MODE, bool ROPE>
__global__ __launch_bounds__(256) void pacl_pool_k(const void* __restrict__ vp, int Bi, int P,
                                                   const float* __restrict__ tp, int Bt, int D,
                                                   const float* __restrict__ rc,
                                                   const float* __restrict__ rs,
                                                   float* __restrict__ out_img,
                                                   float* __restrict__ out_txt) {
    __shared__ float tn[1024];
    __shared__ float part[4][1024];
    __shared__ float red[4];
    const int row = blockIdx.x;
    const int img = Bi == 1 ? 0 : row;
    const int txt = Bt == 1 ? 0 : row;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;

    // normalised text vector
    float ss = 0.f;
    for (int d = tid; d < D; d += 256) { const float t = tp[(size_t)txt * D + d]; tn[d] = t; ss += t * t; }
    ss = wave_sum(ss);
    if (lane == 0) red[wave] = ss;
    __syncthreads();
    const float tinv = 1.0f / fmaxf(sqrtf(red[0] + red[1] + red[2] + red[3]), 1e-12f);
    for (int d = tid; d < D; d += 256) tn[d] *= tinv;
    __syncthreads();
    if (row < Bt && out_txt)
        for (int d = tid; d < D; d += 256) out_txt[(size_t)row * D + d] = tn[d];

    // each lane owns NE = D/64 consecutive-pair elements: e = 2*(c*64 + lane) + {0,1}
    constexpr int MAXC = 8;    // D <= 1024
    const int NCH = D / 128;
    float acc[MAXC][2];
#pragma unroll
    for (int c = 0; c < MAXC; ++c) { acc[c][0] = 0.f; acc[c][1] = 0.f; }
    const int half = D / 2;
    for (int p = wave; p < P; p += 4) {
        const size_t rbase = ((size_t)img * P + p) * D;
        float x[MAXC][2];
#pragma unroll
        for (int c = 0; c < MAXC; ++c) {
            if (c < NCH) {
                const int e = 2 * (c * 64 + lane);
                if constexpr (VP_BF16) {
                    const uint32_t u = *reinterpret_cast<const uint32_t*>(static_cast<const bf16_t*>(vp) + rbase + e);
                    x[c][0] = bf2f((bf16_t)(u & 0xffff));
                    x[c][1] = bf2f((bf16_t)(u >> 16));
                } else {
                    const float2 f = *reinterpret_cast<const float2*>(static_cast<const float*>(vp) + rbase + e);
                    x[c][0] = f.x; x[c][1] = f.y;
                }
            }
        }
        float w = 1.0f;
        if constexpr (MODE == 1) {
            float dot = 0.f, nrm = 0.f;
#pragma unroll
            for (int c = 0; c < MAXC; ++c) {
                if (c < NCH) {
                    const int e = 2 * (c * 64 + lane);
                    if constexpr (ROPE) {
                        const int i = e / 2;   // pair index
                        const float cs = rc[(size_t)p * half + i], sn = rs[(size_t)p * half + i];
                        const float lo = x[c][0] * cs - x[c][1] * sn;
                        const float hi = x[c][0] * sn + x[c][1] * cs;
                        dot += lo * tn[i] + hi * tn[half + i];
                        nrm += lo * lo + hi * hi;
                    } else {
                        dot += x[c][0] * tn[e] + x[c][1] * tn[e + 1];
                        nrm += x[c][0] * x[c][0] + x[c][1] * x[c][1];
                    }
                }
            }
            dot = wave_sum(dot);
            nrm = wave_sum(nrm);
            const float cosv = dot / fmaxf(sqrtf(nrm), 1e-12f);
            w = 1.0f / (1.0f + expf(-10.0f * cosv));
        }
#pragma unroll
        for (int c = 0; c < MAXC; ++c)
            if (c < NCH) { acc[c][0] = fmaf(w, x[c][0], acc[c][0]); acc[c][1] = fmaf(w, x[c][1], acc[c][1]); }
    }
#pragma unroll
    for (int c = 0; c < MAXC; ++c)
        if (c < NCH) {
            const int e = 2 * (c * 64 + lane);
            part[wave][e] = acc[c][0];
            part[wave][e + 1] = acc[c][1];
        }
    __syncthreads();
    float s2 = 0.f;
    for (int d = tid; d < D; d += 256) {
        const float v = (part[0][d] + part[1][d]) + (part[2][d] + part[3][d]);
        part[0][d] = v;
        s2 += v * v;
    }
    s2 = wave_sum(s2);
    __syncthreads();
    if (lane == 0) red[wave] = s2;
    __syncthreads();
    const float inv = 1.0f / fmaxf(sqrtf(red[0] + red[1] + red[2] + red[3]), 1e-12f);
    for (int d = tid; d < D; d += 256) out_img[(size_t)row * D + d] = part[0][d] * inv;
}

// ---- SPARC row weights ---------------------------------------------------------------------
__global__ __launch_bounds__(256) void sparc_weights_k(float* sim, long rows, int P, float sigma) {
    const int lane = threadIdx.x & 63;
    const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= rows) return;
    float* r = sim + row * P;
    float mn = INFINITY, mx = -INFINITY;
    for (int p = lane; p < P; p += 64) { const float v = r[p]; mn = fminf(mn, v); mx = fmaxf(mx, v); }
    mn = wave_min(mn);
    mx = wave_max(mx);
    const float den = (mx - mn) + 1e-8f;
    float s = 0.f;
    for (int p = lane; p < P; p += 64) {
        float v = (r[p] - mn) / den;
        v = v < sigma ? 0.f : v;
        r[p] = v;
        s += v;
    }
    s = wave_sum(s) + 1e-8f;
    for (int p = lane; p < P; p += 64) r[p] = r[p] / s;
}

}  // namespace

hipError_t launch_fgemm(const FGemmParams& p, bool b_nk, hipStream_t s) {
    if (p.M <= 0 || p.N <= 0 || p.batch <= 0) return hipSuccess;
    const dim3 grid((p.N + FT - 1) / FT, (p.M + FT - 1) / FT, p.batch);
    if (b_nk) hipLaunchKernelGGL(fgemm_k<true>, grid, dim3(256), 0, s, p);
    else hipLaunchKernelGGL(fgemm_k<false>, grid, dim3(256), 0, s, p);
    return hipGetLastError();
}

hipError_t launch_pacl_pool(const void* vp, bool vp_bf16, int Bi, int P, const float* tp, int Bt, int D,
                            int weight_mode, const float* rope_cos, const float* rope_sin, float* out_img,
                            float* out_txt, hipStream_t s) {
    if (D % 128 != 0 || D > 1024) return hipErrorInvalidValue;
    const int R = Bi > Bt ? Bi : Bt;
    const bool rope = rope_cos != nullptr;
    const dim3 grid(R), block(256);
#define CE_PP(BF, MO, RO) \
    if (vp_bf16 == BF && weight_mode == MO && rope == RO) { \
        hipLaunchKernelGGL((pacl_pool_k<BF, MO, RO>), grid, block, 0, s, vp, Bi, P, tp, Bt, D, rope_cos, \
                           rope_sin, out_img, out_txt); \
        return hipGetLastError(); }
    CE_PP(true, 0, false) CE_PP(true, 1, false) CE_PP(true, 1, true)
    CE_PP(false, 0, false) CE_PP(false, 1, false) CE_PP(false, 1, true)
#undef CE_PP
    return hipErrorInvalidValue;
}

hipError_t launch_sparc_weights(float* sim, long rows, int P, float sigma, hipStream_t s) {
    if (rows <= 0) return hipSuccess;
    hipLaunchKernelGGL(sparc_weights_k, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, s, sim, rows, P, sigma);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// SparcLoss (pacl.py:516-584)

namespace {

// out[b][d] = mean_p x[b][p][d]   (torch.mean(dim=1), pacl.py:566-567)
__global__ __launch_bounds__(256) void mean_mid_k(const float* __restrict__ x, float* __restrict__ out, int P,
                                                  int D) {
    const int b = blockIdx.y;
    const int d = blockIdx.x * 256 + threadIdx.x;
    if (d >= D) return;
    const float* xp = x + (size_t)b * P * D + d;
    float acc = 0.f;
    for (int p = 0; p < P; ++p) acc += xp[(size_t)p * D];
    out[(size_t)b * D + d] = acc / (float)P;
}

// loss[i] = logsumexp_j L[i][j] - L[i][i]  (F.cross_entropy against arange labels, per row); wave per row
__global__ __launch_bounds__(256) void ce_diag_rows_k(const float* __restrict__ L, int R, int C,
                                                      float* __restrict__ loss) {
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (row >= R) return;
    const float* lr = L + (size_t)row * C;
    float m = -INFINITY;
    for (int j = lane; j < C; j += 64) m = fmaxf(m, lr[j]);
    m = wave_max(m);
    float sum = 0.f;
    for (int j = lane; j < C; j += 64) sum += __expf(lr[j] - m);
    sum = wave_sum(sum);
    if (lane == 0) loss[row] = logf(sum) + m - lr[row];
}

// Masked pairwise local loss, both directions, for one sample per block (pacl.py:527-562):
// S = scale * grouped l^T [T][T]; vl row i: logits S[i][j] + (1 - mask[j]) * -1e8; lv row i (the
// transposed product) = column i of S with the same column mask.  part[b] = {sum_i mask_i
// (lse_vl_i - S_ii), sum_i mask_i (lse_lv_i - S_ii), sum_i mask_i}.
__global__ __launch_bounds__(256) void sparc_local_k(const float* __restrict__ S, const float* __restrict__ mask,
                                                     int T, float* __restrict__ part) {
    const int b = blockIdx.x;
    const float* Sb = S + (size_t)b * T * T;
    const float* mb = mask + (size_t)b * T;
    float a0 = 0.f, a1 = 0.f, a2 = 0.f;
    for (int i = threadIdx.x; i < T; i += blockDim.x) {
        float mr = -INFINITY, mc = -INFINITY;
        for (int j = 0; j < T; ++j) {
            const float pen = (1.0f - mb[j]) * -1e8f;
            mr = fmaxf(mr, Sb[(size_t)i * T + j] + pen);
            mc = fmaxf(mc, Sb[(size_t)j * T + i] + pen);
        }
        float sr = 0.f, sc = 0.f;
        for (int j = 0; j < T; ++j) {
            const float pen = (1.0f - mb[j]) * -1e8f;
            sr += __expf(Sb[(size_t)i * T + j] + pen - mr);
            sc += __expf(Sb[(size_t)j * T + i] + pen - mc);
        }
        const float dg = Sb[(size_t)i * T + i] + (1.0f - mb[i]) * -1e8f;
        const float w = mb[i];
        a0 += w * (logf(sr) + mr - dg);
        a1 += w * (logf(sc) + mc - dg);
        a2 += w;
    }
    __shared__ float red[3][4];
    a0 = wave_sum(a0); a1 = wave_sum(a1); a2 = wave_sum(a2);
    const int wv = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) { red[0][wv] = a0; red[1][wv] = a1; red[2][wv] = a2; }
    __syncthreads();
    if (threadIdx.x < 3) {
        float t = 0.f;
        for (int w = 0; w < (int)(blockDim.x >> 6); ++w) t += red[threadIdx.x][w];
        part[(size_t)b * 3 + threadIdx.x] = t;
    }
}

// total = wg * (mean(lr) + mean(lc)) / 2 + wl * (P0 / M + P1 / M) / 2; fixed summation order
__global__ __launch_bounds__(256) void sparc_loss_finish_k(const float* __restrict__ lr, const float* __restrict__ lc,
                                                           const float* __restrict__ part, int B, float wg, float wl,
                                                           float* __restrict__ out) {
    float v[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
    for (int i = threadIdx.x; i < B; i += 256) {
        v[0] += lr[i]; v[1] += lc[i];
        v[2] += part[3 * i]; v[3] += part[3 * i + 1]; v[4] += part[3 * i + 2];
    }
    __shared__ float red[5][4];
    const int wv = threadIdx.x >> 6;
#pragma unroll
    for (int k = 0; k < 5; ++k) {
        const float t = wave_sum(v[k]);
        if ((threadIdx.x & 63) == 0) red[k][wv] = t;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        float t[5];
        for (int k = 0; k < 5; ++k) t[k] = red[k][0] + red[k][1] + red[k][2] + red[k][3];
        const float glob = (t[0] / (float)B + t[1] / (float)B) * 0.5f;
        const float local = (t[2] / t[4] + t[3] / t[4]) * 0.5f;
        out[0] = wg * glob + wl * local;
    }
}

}  // namespace

hipError_t launch_mean_mid(float* out, const float* x, int B, int P, int D, hipStream_t s) {
    hipLaunchKernelGGL(mean_mid_k, dim3((unsigned)((D + 255) / 256), (unsigned)B), dim3(256), 0, s, x, out, P, D);
    return hipGetLastError();
}
hipError_t launch_ce_diag_rows(float* loss, const float* L, int R, int C, hipStream_t s) {
    hipLaunchKernelGGL(ce_diag_rows_k, dim3((unsigned)((R + 3) / 4)), dim3(256), 0, s, L, R, C, loss);
    return hipGetLastError();
}
hipError_t launch_sparc_local(float* part, const float* S, const float* mask, int B, int T, hipStream_t s) {
    hipLaunchKernelGGL(sparc_local_k, dim3((unsigned)B), dim3(128), 0, s, S, mask, T, part);
    return hipGetLastError();
}
hipError_t launch_sparc_loss_finish(float* out, const float* lr, const float* lc, const float* part, int B,
                                    float global_weight, float local_weight, hipStream_t s) {
    hipLaunchKernelGGL(sparc_loss_finish_k, dim3(1), dim3(256), 0, s, lr, lc, part, B, global_weight, local_weight,
                       out);
    return hipGetLastError();
}

}  // namespace ce
