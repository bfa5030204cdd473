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
#include "knobs.h"

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
        float v = acc[r] * p.alpha + bj;
        if (p.accumulate) v += C[(size_t)gi * p.ldc + gj];
        C[(size_t)gi * p.ldc + gj] = v;
        if (p.Ct) p.Ct[(size_t)gj * p.ldct + gi] = v;
    }
}

// ---- register-blocked f32 GEMM (the SPARC einsums, projections, logits) ----------------------
// 96 x 128 output tile per 256-thread block: wave w owns columns 32w .. 32w+31 and all 96 rows as
// three 32 x 32 accumulators, so one B fragment feeds three v_mfma_f32_32x32x2_f32.  K chunks of 32
// are staged global -> registers (float4) -> LDS, the next chunk's loads in flight under the current
// chunk's MFMAs.  LDS image: [k parity][row][k / 2] with rows padded to 20 floats, so a lane's 4
// consecutive k-pairs come in one ds_read_b128 (lane l: row l & 31, parity l >> 5) and the 16 lanes
// of a read group hit distinct banks.  96 rows: M = 77 (SPARC's T) fills 80 % of the MFMA rows.
constexpr int G2_BM = 96, G2_BN = 128, G2_BK = 32, G2_LD = G2_BK / 2 + 4;

template <bool B_NK>
__global__ __launch_bounds__(256) void fgemm2_k(FGemmParams p) {
    __shared__ __attribute__((aligned(16))) float As[2][G2_BM][G2_LD];
    __shared__ __attribute__((aligned(16))) float Bs[2][G2_BN][G2_LD];
    const int z = blockIdx.z;
    const float* A = p.A + (size_t)z * p.sA;
    const float* Bm = p.B + (size_t)z * p.sB;
    float* C = p.C + (size_t)z * p.sC;
    const int i0 = blockIdx.y * G2_BM, j0 = blockIdx.x * G2_BN;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    f32x16 acc[3];
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[r][e] = 0.f;
    // staging: A chunk = 96 rows x 32 k = 768 float4 (3 per thread); B chunk = 128 x 32 = 1024
    // float4 (4 per thread), [n][k] rows when B_NK, else [k][n] rows
    float4 ra[3], rb[4];
    auto load = [&](int k0) {
#pragma unroll
        for (int u = 0; u < 3; ++u) {
            const int e = tid + 256 * u, row = e >> 3, kq = (e & 7) * 4;
            const int gi = i0 + row, gk = k0 + kq;
            ra[u] = (gi < p.M && gk < p.K) ? *reinterpret_cast<const float4*>(A + (size_t)gi * p.lda + gk)
                                          : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int e = tid + 256 * u;
            if constexpr (B_NK) {
                const int row = e >> 3, kq = (e & 7) * 4;
                const int gj = j0 + row, gk = k0 + kq;
                rb[u] = (gj < p.N && gk < p.K) ? *reinterpret_cast<const float4*>(Bm + (size_t)gj * p.ldb + gk)
                                              : make_float4(0.f, 0.f, 0.f, 0.f);
            } else {
                const int kk = e >> 5, nq = (e & 31) * 4;
                const int gj = j0 + nq, gk = k0 + kk;
                rb[u] = (gj < p.N && gk < p.K) ? *reinterpret_cast<const float4*>(Bm + (size_t)gk * p.ldb + gj)
                                              : make_float4(0.f, 0.f, 0.f, 0.f);
            }
        }
    };
    auto store = [&] {
#pragma unroll
        for (int u = 0; u < 3; ++u) {
            const int e = tid + 256 * u, row = e >> 3, kp = (e & 7) * 2;
            *reinterpret_cast<float2*>(&As[0][row][kp]) = make_float2(ra[u].x, ra[u].z);
            *reinterpret_cast<float2*>(&As[1][row][kp]) = make_float2(ra[u].y, ra[u].w);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int e = tid + 256 * u;
            if constexpr (B_NK) {
                const int row = e >> 3, kp = (e & 7) * 2;
                *reinterpret_cast<float2*>(&Bs[0][row][kp]) = make_float2(rb[u].x, rb[u].z);
                *reinterpret_cast<float2*>(&Bs[1][row][kp]) = make_float2(rb[u].y, rb[u].w);
            } else {
                const int kk = e >> 5, nq = (e & 31) * 4;
                float* d = &Bs[kk & 1][nq][kk >> 1];
                d[0] = rb[u].x; d[G2_LD] = rb[u].y; d[2 * G2_LD] = rb[u].z; d[3 * G2_LD] = rb[u].w;
            }
        }
    };
    const int h = lane >> 5, m = lane & 31;
    load(0);
    for (int k0 = 0; k0 < p.K; k0 += G2_BK) {
        store();
        __syncthreads();
        if (k0 + G2_BK < p.K) load(k0 + G2_BK);
#pragma unroll
        for (int q = 0; q < G2_BK / 8; ++q) {      // 4 k-pairs per ds_read_b128
            const float4 b4 = *reinterpret_cast<const float4*>(&Bs[h][wave * 32 + m][4 * q]);
            float4 a4[3];
#pragma unroll
            for (int r = 0; r < 3; ++r) a4[r] = *reinterpret_cast<const float4*>(&As[h][r * 32 + m][4 * q]);
            const float bq[4] = {b4.x, b4.y, b4.z, b4.w};
#pragma unroll
            for (int kk = 0; kk < 4; ++kk) {
#pragma unroll
                for (int r = 0; r < 3; ++r) {
                    const float aq[4] = {a4[r].x, a4[r].y, a4[r].z, a4[r].w};
                    acc[r] = __builtin_amdgcn_mfma_f32_32x32x2f32(aq[kk], bq[kk], acc[r], 0, 0, 0);
                }
            }
        }
        __syncthreads();
    }
    const int gj = j0 + wave * 32 + m;
    if (gj >= p.N) return;
    const float bj = p.bias ? p.bias[gj] : 0.f;
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            const int gi = i0 + r * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
            if (gi >= p.M) continue;
            float v = acc[r][e] * p.alpha + bj;
            if (p.accumulate) v += C[(size_t)gi * p.ldc + gj];
            C[(size_t)gi * p.ldc + gj] = v;
            if (p.Ct) p.Ct[(size_t)gj * p.ldct + gi] = v;
        }
}

// ---- short-M batched f32 GEMM (SPARC's einsums: M = T = 77 rows per sample) -------------------
// 80 x 192 output tile per 256-thread block on v_mfma_f32_16x16x4_f32: 16-row granularity, so
// M = 77 fills 96 % of the rows (32-row blocks: 80 % at 96 rows), and 192 columns divide both
// N = 576 (P) and N = 768 (D).  Wave w owns columns 48w .. 48w+47 and all 80 rows: 5 x 3
// accumulators, so per k-step 5 A and 3 B values feed 15 MFMAs.  Within a K chunk of 32 the
// k index of lane group g = lane >> 4 at k-step s is 8g + s (any k assignment works when A and B
// share it), so a lane's 8 k-values of a row are contiguous: two ds_read_b128 per row per chunk,
// and the LDS image is the natural [row][k] layout (rows padded to 36 floats: the 16 rows of a
// read group start on distinct 4-bank groups).  The next chunk's float4 global loads are in flight
// under the current chunk's MFMAs.
constexpr int G3_BM = 80, G3_BN = 192, G3_BK = 32, G3_LD = G3_BK + 4;
constexpr int G3_NA = (G3_BM * G3_BK / 4 + 255) / 256;        // float4 per thread: A 640 -> 3
constexpr int G3_NB = G3_BN * G3_BK / 4 / 256;                // B 1536 -> 6

template <bool B_NK>
__global__ __launch_bounds__(256) void fgemm3_k(FGemmParams p) {
    __shared__ __attribute__((aligned(16))) float As[G3_BM][G3_LD];
    __shared__ __attribute__((aligned(16))) float Bs[G3_BN][G3_LD];
    const int z = blockIdx.z;
    const float* A = p.A + (size_t)z * p.sA;
    const float* Bm = p.B + (size_t)z * p.sB;
    float* C = p.C + (size_t)z * p.sC;
    const int i0 = blockIdx.y * G3_BM, j0 = blockIdx.x * G3_BN;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    f32x4 acc[5][3];
#pragma unroll
    for (int a = 0; a < 5; ++a)
#pragma unroll
        for (int b = 0; b < 3; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
    float4 ra[G3_NA], rb[G3_NB];
    const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
    auto load = [&](int k0) {
#pragma unroll
        for (int u = 0; u < G3_NA; ++u) {
            const int e = tid + 256 * u, row = e >> 3, kq = (e & 7) * 4;
            const int gi = i0 + row, gk = k0 + kq;
            ra[u] = (row < G3_BM && gi < p.M && gk < p.K) ? *reinterpret_cast<const float4*>(A + (size_t)gi * p.lda + gk) : z4;
        }
#pragma unroll
        for (int u = 0; u < G3_NB; ++u) {
            const int e = tid + 256 * u;
            if constexpr (B_NK) {
                const int row = e >> 3, kq = (e & 7) * 4;
                const int gj = j0 + row, gk = k0 + kq;
                rb[u] = (gj < p.N && gk < p.K) ? *reinterpret_cast<const float4*>(Bm + (size_t)gj * p.ldb + gk) : z4;
            } else {
                const int kk = e / (G3_BN / 4), nq = (e % (G3_BN / 4)) * 4;
                const int gj = j0 + nq, gk = k0 + kk;
                rb[u] = (gj < p.N && gk < p.K) ? *reinterpret_cast<const float4*>(Bm + (size_t)gk * p.ldb + gj) : z4;
            }
        }
    };
    auto store = [&] {
#pragma unroll
        for (int u = 0; u < G3_NA; ++u) {
            const int e = tid + 256 * u, row = e >> 3, kq = (e & 7) * 4;
            if (row < G3_BM) *reinterpret_cast<float4*>(&As[row][kq]) = ra[u];
        }
#pragma unroll
        for (int u = 0; u < G3_NB; ++u) {
            const int e = tid + 256 * u;
            if constexpr (B_NK) {
                const int row = e >> 3, kq = (e & 7) * 4;
                *reinterpret_cast<float4*>(&Bs[row][kq]) = rb[u];
            } else {
                const int kk = e / (G3_BN / 4), nq = (e % (G3_BN / 4)) * 4;
                Bs[nq][kk] = rb[u].x; Bs[nq + 1][kk] = rb[u].y; Bs[nq + 2][kk] = rb[u].z; Bs[nq + 3][kk] = rb[u].w;
            }
        }
    };
    const int g = lane >> 4, m = lane & 15;
    load(0);
    for (int k0 = 0; k0 < p.K; k0 += G3_BK) {
        store();
        __syncthreads();
        if (k0 + G3_BK < p.K) load(k0 + G3_BK);
#pragma unroll
        for (int hq = 0; hq < 2; ++hq) {             // k-steps 4hq .. 4hq+3: one ds_read_b128 per row
            float4 a4[5], b4[3];
#pragma unroll
            for (int ib = 0; ib < 5; ++ib) a4[ib] = *reinterpret_cast<const float4*>(&As[ib * 16 + m][8 * g + 4 * hq]);
#pragma unroll
            for (int jb = 0; jb < 3; ++jb)
                b4[jb] = *reinterpret_cast<const float4*>(&Bs[wave * 48 + jb * 16 + m][8 * g + 4 * hq]);
#pragma unroll
            for (int s = 0; s < 4; ++s)
#pragma unroll
                for (int ib = 0; ib < 5; ++ib)
#pragma unroll
                    for (int jb = 0; jb < 3; ++jb) {
                        const float av = s == 0 ? a4[ib].x : s == 1 ? a4[ib].y : s == 2 ? a4[ib].z : a4[ib].w;
                        const float bv = s == 0 ? b4[jb].x : s == 1 ? b4[jb].y : s == 2 ? b4[jb].z : b4[jb].w;
                        acc[ib][jb] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc[ib][jb], 0, 0, 0);
                    }
        }
        __syncthreads();
    }
    // D: lane holds column m of its 16-column block, rows 4g .. 4g+3 of each 16-row block
#pragma unroll
    for (int jb = 0; jb < 3; ++jb) {
        const int gj = j0 + wave * 48 + jb * 16 + m;
        if (gj >= p.N) continue;
        const float bj = p.bias ? p.bias[gj] : 0.f;
#pragma unroll
        for (int ib = 0; ib < 5; ++ib)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int gi = i0 + ib * 16 + 4 * g + r;
                if (gi >= p.M) continue;
                float v = acc[ib][jb][r] * p.alpha + bj;
                if (p.accumulate) v += C[(size_t)gi * p.ldc + gj];
                C[(size_t)gi * p.ldc + gj] = v;
                if (p.Ct) p.Ct[(size_t)gj * p.ldct + gi] = v;
            }
    }
}

// ---- fused PACL pooling -----------------------------------------------------------------
// Two passes.  Pass 1 (pacl_pool_part_k): grid = R output rows x S patch splits; each 256-thread
// workgroup streams its P/S patches of one image, one patch row per wave at a time, every lane
// loading 16-B chunks (8 bf16) of the row (chunk q = c * 64 + lane, elements 8q .. 8q + 7, valid
// while 8q < D), two patches in flight per wave; MODE 1 forms the wave's dot(t_n, v_p) and |v_p|^2
// (after RoPE for ROPE) with two wave reductions and w_p = sigmoid(10 cos); the four waves' sums
// meet in LDS and leave as one f32 partial row part[row][split][D].  Pass 2 (pacl_pool_finish_k):
// per output row the S partials in a fixed order, L2-normalised; the normalised text rows.
// D <= 1024, D % 128 == 0 (768 for ViT-L-14-336).
constexpr int PP_NC = 2;           // 16-B chunks per lane per patch row (D <= 1024 bf16)

template <bool VP_BF16>
__device__ __forceinline__ void pp_load(const void* vp, size_t rbase, int q, float (&x)[8]) {
    if constexpr (VP_BF16) {
        const uint4 u = *reinterpret_cast<const uint4*>(static_cast<const bf16_t*>(vp) + rbase + 8 * q);
        const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            x[2 * k] = __uint_as_float(w[k] << 16);
            x[2 * k + 1] = __uint_as_float(w[k] & 0xffff0000u);
        }
    } else {
        const float4 a = *reinterpret_cast<const float4*>(static_cast<const float*>(vp) + rbase + 8 * q);
        const float4 b = *reinterpret_cast<const float4*>(static_cast<const float*>(vp) + rbase + 8 * q + 4);
        x[0] = a.x; x[1] = a.y; x[2] = a.z; x[3] = a.w; x[4] = b.x; x[5] = b.y; x[6] = b.z; x[7] = b.w;
    }
}

template <bool VP_BF16, int MODE, bool ROPE>
__global__ __launch_bounds__(256) void pacl_pool_part_k(const void* __restrict__ vp, int Bi, int P,
                                                        const float* __restrict__ tp, int Bt, int D,
                                                        const float* __restrict__ rc,
                                                        const float* __restrict__ rs, int S,
                                                        float* __restrict__ part) {
    __shared__ __attribute__((aligned(16))) float tn[1024];
    __shared__ __attribute__((aligned(16))) float red[4][1024];
    const int row = blockIdx.x / S, split = blockIdx.x - row * S;
    const int img = Bi == 1 ? 0 : row;
    const int txt = Bt == 1 ? 0 : row;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int half = D / 2;
    if constexpr (MODE == 1) {
        // normalised text vector (F.normalize, pacl.py:123)
        float ss = 0.f;
        for (int d = tid; d < D; d += 256) { const float t = tp[(size_t)txt * D + d]; tn[d] = t; ss = fmaf(t, t, ss); }
        ss = wave_sum(ss);
        if (lane == 0) red[0][wave] = ss;
        __syncthreads();
        const float tinv = 1.0f / fmaxf(sqrtf((red[0][0] + red[0][1]) + (red[0][2] + red[0][3])), 1e-12f);
        for (int d = tid; d < D; d += 256) tn[d] *= tinv;
        __syncthreads();
    }
    const int p0 = (int)((long)split * P / S), p1 = (int)((long)(split + 1) * P / S);
    float acc[PP_NC][8];
#pragma unroll
    for (int c = 0; c < PP_NC; ++c)
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[c][k] = 0.f;
    // weight of one patch row (MODE 1): sigmoid(10 cos(t_n, [rope](v_p)))  (pacl.py:120-127,199-209)
    auto weight = [&](int p, const float (&x)[PP_NC][8]) -> float {
        if constexpr (MODE == 0) {
            return 1.0f;
        } else {
            float dot = 0.f, nrm = 0.f;
#pragma unroll
            for (int c = 0; c < PP_NC; ++c) {
                const int q = c * 64 + lane;
                if (8 * q < D) {
                    if constexpr (ROPE) {
                        // pairs (8q + 2k, 8q + 2k + 1) -> positions i = 4q + k and half + i (Q7)
                        const float4 cs = *reinterpret_cast<const float4*>(rc + (size_t)p * half + 4 * q);
                        const float4 sn = *reinterpret_cast<const float4*>(rs + (size_t)p * half + 4 * q);
                        const float4 tl = *reinterpret_cast<const float4*>(tn + 4 * q);
                        const float4 th = *reinterpret_cast<const float4*>(tn + half + 4 * q);
                        const float c4[4] = {cs.x, cs.y, cs.z, cs.w}, s4[4] = {sn.x, sn.y, sn.z, sn.w};
                        const float l4[4] = {tl.x, tl.y, tl.z, tl.w}, h4[4] = {th.x, th.y, th.z, th.w};
#pragma unroll
                        for (int k = 0; k < 4; ++k) {
                            const float lo = x[c][2 * k] * c4[k] - x[c][2 * k + 1] * s4[k];
                            const float hi = x[c][2 * k] * s4[k] + x[c][2 * k + 1] * c4[k];
                            dot += lo * l4[k] + hi * h4[k];
                            nrm += lo * lo + hi * hi;
                        }
                    } else {
                        const float4 ta = *reinterpret_cast<const float4*>(tn + 8 * q);
                        const float4 tb = *reinterpret_cast<const float4*>(tn + 8 * q + 4);
                        const float t8[8] = {ta.x, ta.y, ta.z, ta.w, tb.x, tb.y, tb.z, tb.w};
#pragma unroll
                        for (int k = 0; k < 8; ++k) {
                            dot = fmaf(x[c][k], t8[k], dot);
                            nrm = fmaf(x[c][k], x[c][k], nrm);
                        }
                    }
                }
            }
            dot = wave_sum(dot);
            nrm = wave_sum(nrm);
            const float cosv = dot / fmaxf(sqrtf(nrm), 1e-12f);
            return 1.0f / (1.0f + expf(-10.0f * cosv));
        }
    };
    auto load_row = [&](int p, float (&x)[PP_NC][8]) {
        const size_t rbase = ((size_t)img * P + p) * D;
#pragma unroll
        for (int c = 0; c < PP_NC; ++c) {
            const int q = c * 64 + lane;
            if (8 * q < D) pp_load<VP_BF16>(vp, rbase, q, x[c]);
            else {
#pragma unroll
                for (int k = 0; k < 8; ++k) x[c][k] = 0.f;
            }
        }
    };
    int p = p0 + wave;
    // two patch rows in flight per wave
    for (; p + 4 < p1; p += 8) {
        float xa[PP_NC][8], xb[PP_NC][8];
        load_row(p, xa);
        load_row(p + 4, xb);
        const float wa = weight(p, xa), wb = weight(p + 4, xb);
#pragma unroll
        for (int c = 0; c < PP_NC; ++c)
#pragma unroll
            for (int k = 0; k < 8; ++k) acc[c][k] = fmaf(wb, xb[c][k], fmaf(wa, xa[c][k], acc[c][k]));
    }
    if (p < p1) {
        float xa[PP_NC][8];
        load_row(p, xa);
        const float wa = weight(p, xa);
#pragma unroll
        for (int c = 0; c < PP_NC; ++c)
#pragma unroll
            for (int k = 0; k < 8; ++k) acc[c][k] = fmaf(wa, xa[c][k], acc[c][k]);
    }
    // the four waves' sums, fixed order, one partial row
#pragma unroll
    for (int c = 0; c < PP_NC; ++c) {
        const int q = c * 64 + lane;
        if (8 * q < D) {
            *reinterpret_cast<float4*>(&red[wave][8 * q]) = make_float4(acc[c][0], acc[c][1], acc[c][2], acc[c][3]);
            *reinterpret_cast<float4*>(&red[wave][8 * q + 4]) = make_float4(acc[c][4], acc[c][5], acc[c][6], acc[c][7]);
        }
    }
    __syncthreads();
    float* dst = part + (size_t)blockIdx.x * D;
    for (int d4 = tid; d4 < D / 4; d4 += 256) {
        const float4 a = *reinterpret_cast<const float4*>(&red[0][4 * d4]);
        const float4 b = *reinterpret_cast<const float4*>(&red[1][4 * d4]);
        const float4 c = *reinterpret_cast<const float4*>(&red[2][4 * d4]);
        const float4 e = *reinterpret_cast<const float4*>(&red[3][4 * d4]);
        *reinterpret_cast<float4*>(dst + 4 * d4) =
            make_float4((a.x + b.x) + (c.x + e.x), (a.y + b.y) + (c.y + e.y), (a.z + b.z) + (c.z + e.z),
                        (a.w + b.w) + (c.w + e.w));
    }
}

// Pass 2: out_img[row] = normalize(sum_split part[row][split]); out_txt[row] = normalize(tp[row])
__global__ __launch_bounds__(256) void pacl_pool_finish_k(const float* __restrict__ part, int S, int D,
                                                          const float* __restrict__ tp, int Bt,
                                                          float* __restrict__ out_img,
                                                          float* __restrict__ out_txt) {
    __shared__ float red[2][4];
    const int row = blockIdx.x;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    float v[4] = {0.f, 0.f, 0.f, 0.f};     // D <= 1024: elements tid + 256 k
    float s2 = 0.f, st = 0.f;
    const float* pr = part + (size_t)row * S * D;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int d = tid + 256 * k;
        if (d < D) {
            float a = 0.f;
            for (int sp = 0; sp < S; ++sp) a += pr[(size_t)sp * D + d];
            v[k] = a;
            s2 = fmaf(a, a, s2);
            if (out_txt && row < Bt) { const float t = tp[(size_t)row * D + d]; st = fmaf(t, t, st); }
        }
    }
    s2 = wave_sum(s2);
    st = wave_sum(st);
    if (lane == 0) { red[0][wave] = s2; red[1][wave] = st; }
    __syncthreads();
    const float inv = 1.0f / fmaxf(sqrtf((red[0][0] + red[0][1]) + (red[0][2] + red[0][3])), 1e-12f);
    const float tinv = 1.0f / fmaxf(sqrtf((red[1][0] + red[1][1]) + (red[1][2] + red[1][3])), 1e-12f);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int d = tid + 256 * k;
        if (d < D) {
            out_img[(size_t)row * D + d] = v[k] * inv;
            if (out_txt && row < Bt) out_txt[(size_t)row * D + d] = tp[(size_t)row * D + d] * tinv;
        }
    }
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

// f32 GEMM variant: 0 = the 64 x 64 scalar-staged kernel; 1 (default) = the register-blocked 96 x 128
// kernel; 2 = as 1, with the short-M 80 x 192 kernel for batched products of M <= 80 rows (measured
// slower at the C5 shapes: sparc_sim 51.5 vs 62.9 TF/s, sparc_group 59.3 vs 71.1; kept for A/B)
std::atomic<int> g_fgemm2{1};     // A/B knob (knobs.h: process-wide atomic)

}  // namespace

int set_fgemm_variant(int v) {
    const int prev = g_fgemm2.load();
    g_fgemm2 = v < 0 ? 0 : v > 2 ? 2 : v;
    return prev;
}

hipError_t launch_fgemm(const FGemmParams& p, bool b_nk, hipStream_t s) {
    if (p.M <= 0 || p.N <= 0 || p.batch <= 0) return hipSuccess;
    // float4 staging needs 16-B aligned rows and K chunks: every operand base, stride and K a
    // multiple of 4 floats; anything else takes the scalar-staged 64 x 64 kernel
    auto al = [](const void* q) { return ((uintptr_t)q & 15) == 0; };
    const bool vec = p.K % 4 == 0 && p.lda % 4 == 0 && p.ldb % 4 == 0 && p.sA % 4 == 0 && p.sB % 4 == 0 &&
                     al(p.A) && al(p.B) && (b_nk || p.N % 4 == 0);
    const int fv = g_fgemm2.load(std::memory_order_acquire);
    if (vec && fv == 2 && p.M <= G3_BM && p.N >= G3_BN && p.batch > 1) {
        const dim3 grid((p.N + G3_BN - 1) / G3_BN, 1, p.batch);
        if (b_nk) hipLaunchKernelGGL(fgemm3_k<true>, grid, dim3(256), 0, s, p);
        else hipLaunchKernelGGL(fgemm3_k<false>, grid, dim3(256), 0, s, p);
        return hipGetLastError();
    }
    if (vec && fv) {
        const dim3 grid((p.N + G2_BN - 1) / G2_BN, (p.M + G2_BM - 1) / G2_BM, p.batch);
        if (b_nk) hipLaunchKernelGGL(fgemm2_k<true>, grid, dim3(256), 0, s, p);
        else hipLaunchKernelGGL(fgemm2_k<false>, grid, dim3(256), 0, s, p);
        return hipGetLastError();
    }
    const dim3 grid((p.N + FT - 1) / FT, (p.M + FT - 1) / FT, p.batch);
    if (b_nk) hipLaunchKernelGGL(fgemm_k<true>, grid, dim3(256), 0, s, p);
    else hipLaunchKernelGGL(fgemm_k<false>, grid, dim3(256), 0, s, p);
    return hipGetLastError();
}

int pacl_pool_splits(int R, int P) {
    // >= 4096 workgroups (16 per CU) where the rows allow, >= 16 patches per workgroup
    int S = (4096 + R - 1) / R;
    const int smax = P / 16 > 1 ? P / 16 : 1;
    return S < 1 ? 1 : S > smax ? smax : S;
}

size_t pacl_pool_part_bytes(int R, int P, int D) { return (size_t)R * pacl_pool_splits(R, P) * D * 4; }

hipError_t launch_pacl_pool(const void* vp, bool vp_bf16, int Bi, int P, const float* tp, int Bt, int D,
                            int weight_mode, const float* rope_cos, const float* rope_sin, float* out_img,
                            float* out_txt, float* part, hipStream_t s) {
    if (D % 128 != 0 || D > 1024 || !part) return hipErrorInvalidValue;
    const int R = Bi > Bt ? Bi : Bt;
    const int S = pacl_pool_splits(R, P);
    const bool rope = rope_cos != nullptr;
    const dim3 grid((unsigned)(R * S)), block(256);
    bool launched = false;
#define CE_PP(BF, MO, RO) \
    if (!launched && vp_bf16 == BF && weight_mode == MO && rope == RO) { \
        hipLaunchKernelGGL((pacl_pool_part_k<BF, MO, RO>), grid, block, 0, s, vp, Bi, P, tp, Bt, D, rope_cos, \
                           rope_sin, S, part); \
        launched = true; }
    CE_PP(true, 0, false) CE_PP(true, 1, false) CE_PP(true, 1, true)
    CE_PP(false, 0, false) CE_PP(false, 1, false) CE_PP(false, 1, true)
#undef CE_PP
    if (!launched) return hipErrorInvalidValue;
    hipLaunchKernelGGL(pacl_pool_finish_k, dim3((unsigned)R), block, 0, s, part, S, D, tp, Bt, out_img, out_txt);
    return hipGetLastError();
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

// loss[i] = logsumexp_j L[i][j] - L[i][off + i]  (F.cross_entropy against labels arange + off, per row;
// off = the first global row of this rank's shard, loss.py:113-117 local-loss labels); wave per row
__global__ __launch_bounds__(256) void ce_diag_rows_k(const float* __restrict__ L, int R, int C, int off,
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
    if (lane == 0) loss[row] = logf(sum) + m - lr[off + row];
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

// Partial sums of one shard, fixed summation order: parts = {sum_i lr_i, sum_i lc_i, sum_b part[b][0],
// sum_b part[b][1], sum_b part[b][2]} (lr / lc / part may be null: those sums are 0).  The shards' parts
// add up (caller's all-reduce) to the sums over the whole batch.
__global__ __launch_bounds__(256) void loss_parts_k(const float* __restrict__ lr, const float* __restrict__ lc,
                                                    int R, const float* __restrict__ part, int B,
                                                    float* __restrict__ parts) {
    float v[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
    if (lr)
        for (int i = threadIdx.x; i < R; i += 256) { v[0] += lr[i]; v[1] += lc[i]; }
    if (part)
        for (int i = threadIdx.x; i < B; i += 256) {
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
    if (threadIdx.x < 5) {
        const int k = threadIdx.x;
        parts[k] = red[k][0] + red[k][1] + red[k][2] + red[k][3];
    }
}

// total = wg * (P0 / N + P1 / N) / 2 + wl * (P2 / P4 + P3 / P4) / 2   (pacl.py:567-583; wl == 0: the
// PACL ClipLoss, pacl.py:509-512, no local term)
__global__ void loss_combine_k(const float* __restrict__ parts, int N, float wg, float wl, float* __restrict__ out) {
    if (threadIdx.x != 0) return;
    const float glob = (parts[0] / (float)N + parts[1] / (float)N) * 0.5f;
    float total = wg * glob;
    if (wl != 0.f) total += wl * ((parts[2] / parts[4] + parts[3] / parts[4]) * 0.5f);
    out[0] = total;
}

}  // namespace

hipError_t launch_mean_mid(float* out, const float* x, int B, int P, int D, hipStream_t s) {
    hipLaunchKernelGGL(mean_mid_k, dim3((unsigned)((D + 255) / 256), (unsigned)B), dim3(256), 0, s, x, out, P, D);
    return hipGetLastError();
}
hipError_t launch_ce_diag_rows(float* loss, const float* L, int R, int C, int off, hipStream_t s) {
    if (R <= 0) return hipSuccess;
    hipLaunchKernelGGL(ce_diag_rows_k, dim3((unsigned)((R + 3) / 4)), dim3(256), 0, s, L, R, C, off, loss);
    return hipGetLastError();
}
hipError_t launch_sparc_local(float* part, const float* S, const float* mask, int B, int T, hipStream_t s) {
    hipLaunchKernelGGL(sparc_local_k, dim3((unsigned)B), dim3(128), 0, s, S, mask, T, part);
    return hipGetLastError();
}
hipError_t launch_loss_parts(float* parts, const float* lr, const float* lc, int R, const float* part, int B,
                             hipStream_t s) {
    hipLaunchKernelGGL(loss_parts_k, dim3(1), dim3(256), 0, s, lr, lc, R, part, B, parts);
    return hipGetLastError();
}
hipError_t launch_loss_combine(float* out, const float* parts, int N, float global_weight, float local_weight,
                               hipStream_t s) {
    hipLaunchKernelGGL(loss_combine_k, dim3(1), dim3(64), 0, s, parts, N, global_weight, local_weight, out);
    return hipGetLastError();
}

}  // namespace ce
