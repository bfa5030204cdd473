// SPARC head training kernels for gfx950 (train_sparc.py:29-37 on Patch-Aligned-Contrastive-Learning/
// model/pacl.py:380-584): the row kernels of the heads' forward with dropout, of the alignment's
// backward and of SparcLoss's gradients.  The GEMMs of the heads and of the batched einsums are the
// engine's (gemm.hip, gemm_tn.hip, heads.hip fgemm); capi.hip orchestrates (ce_sparc_train_*).
#include "ce_device.h"
#include "ce_kernels.h"

namespace ce {
namespace {

// nn.Dropout(p) keep decision: counter-based, so the backward recomputes the forward's mask.
// keep(seed, i) = top 24 bits of splitmix64(seed + (i + 1) * gamma) >= p * 2^24 (the generator's
// n-th output for state seed).  i counts elements over the GLOBAL batch (row offset roff = the rank's
// first sample x rows per sample), so a data-parallel step draws the masks of the single-device step.
// tests/test_gpu_sparc_train.py restates it in NumPy.
__device__ __forceinline__ bool drop_keep(uint64_t seed, uint64_t i, uint32_t thresh) {
    uint64_t z = seed + (i + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    return (uint32_t)(z >> 40) >= thresh;
}
__host__ __device__ inline uint32_t drop_thresh(float p) {
    const double t = (double)p * 16777216.0;
    return t <= 0.0 ? 0u : t >= 16777216.0 ? 16777216u : (uint32_t)t;
}

// LayerNorm (eps 1e-5, affine) then Dropout(p) of one row per wave (nn.Sequential(LayerNorm, Dropout),
// pacl.py:397-406): x f32 [R][D] -> out (bf16 for the bf16 GEMMs of the visual head, f32 for the text
// head's f32 GEMM), stats[r] = (mu, rstd) for the backward.  D % 256 == 0, D <= 1024.
template <bool OUT_BF16>
__global__ __launch_bounds__(256) void ln_drop_k(const float* __restrict__ x, const float* __restrict__ w,
                                                 const float* __restrict__ b, long R, int D, uint32_t thresh,
                                                 float inv_keep, uint64_t seed, long roff, void* __restrict__ out,
                                                 float2* __restrict__ stats) {
    const int lane = threadIdx.x & 63;
    const long r = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= R) return;
    const int nq = D / 256;                      // float4 chunks per lane
    const float* xr = x + r * D;
    float4 v[4];
    float s = 0.f;
    for (int q = 0; q < nq; ++q) {
        v[q] = *reinterpret_cast<const float4*>(xr + 256 * q + 4 * lane);
        s += (v[q].x + v[q].y) + (v[q].z + v[q].w);
    }
    const float mu = wave_sum(s) / (float)D;
    float ss = 0.f;
    for (int q = 0; q < nq; ++q) {
        const float a = v[q].x - mu, c = v[q].y - mu, d = v[q].z - mu, e = v[q].w - mu;
        ss += (a * a + c * c) + (d * d + e * e);
    }
    const float rstd = rsqrtf(wave_sum(ss) / (float)D + 1e-5f);
    if (lane == 0) stats[r] = make_float2(mu, rstd);
    for (int q = 0; q < nq; ++q) {
        const int c0 = 256 * q + 4 * lane;
        const float4 g = *reinterpret_cast<const float4*>(w + c0), bb = *reinterpret_cast<const float4*>(b + c0);
        float y[4] = {(v[q].x - mu) * rstd * g.x + bb.x, (v[q].y - mu) * rstd * g.y + bb.y,
                      (v[q].z - mu) * rstd * g.z + bb.z, (v[q].w - mu) * rstd * g.w + bb.w};
        if (thresh) {
#pragma unroll
            for (int e = 0; e < 4; ++e)
                y[e] = drop_keep(seed, (uint64_t)(roff + r) * D + c0 + e, thresh) ? y[e] * inv_keep : 0.f;
        }
        if constexpr (OUT_BF16) {
            *reinterpret_cast<uint2*>(static_cast<bf16_t*>(out) + r * D + c0) =
                make_uint2(pack_bf2(y[0], y[1]), pack_bf2(y[2], y[3]));
        } else {
            *reinterpret_cast<float4*>(static_cast<float*>(out) + r * D + c0) = make_float4(y[0], y[1], y[2], y[3]);
        }
    }
}

// LayerNorm weight / bias gradients through the dropout (the LN input is a frozen tower's output: no dx):
// dy' = dy * keep / (1 - p), xhat = (x - mu) rstd, part[chunk][0][c] = sum_r dy' xhat, part[chunk][1][c] =
// sum_r dy' over the chunk's rows (fixed order); ln_grad_finish_k sums the chunks in order.
constexpr int LNG_ROWS = 128;
__global__ __launch_bounds__(256) void ln_grad_part_k(const float* __restrict__ dy, const float* __restrict__ x,
                                                      const float2* __restrict__ stats, long R, int D, uint32_t thresh,
                                                      float inv_keep, uint64_t seed, long roff, float* __restrict__ part) {
    const long r0 = (long)blockIdx.x * LNG_ROWS;
    const long r1 = min(R, r0 + LNG_ROWS);
    for (int c = threadIdx.x; c < D; c += 256) {
        float ag = 0.f, ab = 0.f;
        for (long r = r0; r < r1; ++r) {
            float g = dy[r * D + c];
            if (thresh) g = drop_keep(seed, (uint64_t)(roff + r) * D + c, thresh) ? g * inv_keep : 0.f;
            const float2 st = stats[r];
            ag = fmaf(g, (x[r * D + c] - st.x) * st.y, ag);
            ab += g;
        }
        part[(size_t)blockIdx.x * 2 * D + c] = ag;
        part[(size_t)blockIdx.x * 2 * D + D + c] = ab;
    }
}
__global__ __launch_bounds__(256) void ln_grad_finish_k(const float* __restrict__ part, int nchunk, int D,
                                                        float* __restrict__ dw, float* __restrict__ db) {
    const int c = blockIdx.x * 256 + threadIdx.x;
    if (c >= 2 * D) return;
    float a = 0.f;
    for (int k = 0; k < nchunk; ++k) a += part[(size_t)k * 2 * D + c];
    if (c < D) dw[c] = a;
    else db[c - D] = a;
}

// Backward of sparc.forward's alignment weights (pacl.py:460-470) for one (sample, token) row per wave:
// N = (S - min) / (max - min + 1e-8), Th = N where N >= sigma else 0, W = Th / (sum Th + 1e-8).
// In: S (the raw similarity row) and dW (d loss / d W, in io); out: d loss / d S in io.  The min / max
// gradients go to the first minimal / maximal patch (torch.min / max along a dim return one index).
__global__ __launch_bounds__(256) void align_bwd_k(const float* __restrict__ S, float* __restrict__ io, long rows,
                                                   int P, float sigma) {
    const int lane = threadIdx.x & 63;
    const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= rows) return;
    const float* sr = S + row * P;
    float* dr = io + row * P;
    float mn = INFINITY, mx = -INFINITY;
    int imn = P, imx = P;
    for (int p = lane; p < P; p += 64) {
        const float v = sr[p];
        if (v < mn) { mn = v; imn = p; }
        if (v > mx) { mx = v; imx = p; }
    }
    // wave argmin / argmax (first index on ties)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const float omn = __shfl_xor(mn, o, 64), omx = __shfl_xor(mx, o, 64);
        const int oin = __shfl_xor(imn, o, 64), oix = __shfl_xor(imx, o, 64);
        if (omn < mn || (omn == mn && oin < imn)) { mn = omn; imn = oin; }
        if (omx > mx || (omx == mx && oix < imx)) { mx = omx; imx = oix; }
    }
    const float den = (mx - mn) + 1e-8f, iden = 1.0f / den;
    float s = 0.f;
    for (int p = lane; p < P; p += 64) {
        const float n = (sr[p] - mn) / den;
        s += n < sigma ? 0.f : n;
    }
    s = wave_sum(s) + 1e-8f;
    float dot = 0.f;
    for (int p = lane; p < P; p += 64) {
        const float n = (sr[p] - mn) / den;
        dot += dr[p] * ((n < sigma ? 0.f : n) / s);
    }
    dot = wave_sum(dot);
    float dmn = 0.f, dmx = 0.f;
    const float is = 1.0f / s;
    for (int p = lane; p < P; p += 64) {
        const float n = (sr[p] - mn) / den;
        const float dn = n < sigma ? 0.f : (dr[p] - dot) * is;
        dmn = fmaf(dn, (n - 1.0f) * iden, dmn);
        dmx = fmaf(-dn, n * iden, dmx);
        dr[p] = dn * iden;
    }
    dmn = wave_sum(dmn);
    dmx = wave_sum(dmx);
    if (lane == 0) {
        // (separate adds: imn == imx only for a constant row, whose gradients are 0 anyway)
        dr[imn] += dmn;
        dr[imx] += dmx;
    }
}

// Gradient of SparcLoss's masked pairwise local losses (pacl.py:522-556, 575-580) for one sample per
// block: R = scale Gn Ln^T [T][T] (Gn = grouped, Ln = tokens, both normalised); vl row i: z = R[i][.] +
// pen, lv row i: z = R[.][i] + pen (pen_j = (1 - mask_j) * -1e8), each row's CE against label i
// weighted w * mask_i (w = local_weight / 2 / sum of the mask over the global batch).  Writes
// dR = d loss / d R and its transpose (the B operands of dGn = scale dR Ln, dLn = scale dR^T Gn) and
// the loss sums part[b] = {sum_i mask_i (lse_vl_i - z_ii), sum_i mask_i (lse_lv_i - z_ii), sum_i mask_i}
// (sparc_local_k's).  T <= 80 (51 KB of LDS).
__global__ __launch_bounds__(128) void local_grad_k(const float* __restrict__ R, const float* __restrict__ mask, int T,
                                                    float w, float* __restrict__ dR, float* __restrict__ dRT,
                                                    float* __restrict__ part) {
    __shared__ float a1[80 * 81];                            // [T][T + 1]: row contributions
    __shared__ float a2[80 * 81];                            // [T][T + 1]: column contributions, transposed
    __shared__ float red[3][2];
    const int b = blockIdx.x, i = threadIdx.x;
    const float* Rb = R + (size_t)b * T * T;
    const float* mb = mask + (size_t)b * T;
    const int L = T + 1;
    float c0 = 0.f, c1 = 0.f, c2 = 0.f;
    if (i < T) {
        const float mi = mb[i];
        float mr = -INFINITY, mc = -INFINITY;
        for (int j = 0; j < T; ++j) {
            const float pen = (1.0f - mb[j]) * -1e8f;
            mr = fmaxf(mr, Rb[(size_t)i * T + j] + pen);
            mc = fmaxf(mc, Rb[(size_t)j * T + i] + pen);
        }
        float sr = 0.f, sc = 0.f;
        for (int j = 0; j < T; ++j) {
            const float pen = (1.0f - mb[j]) * -1e8f;
            sr += __expf(Rb[(size_t)i * T + j] + pen - mr);
            sc += __expf(Rb[(size_t)j * T + i] + pen - mc);
        }
        const float dg = Rb[(size_t)i * T + i] + (1.0f - mi) * -1e8f;
        c0 = mi * (logf(sr) + mr - dg);
        c1 = mi * (logf(sc) + mc - dg);
        c2 = mi;
        const float gw = w * mi, isr = 1.0f / sr, isc = 1.0f / sc;
        for (int j = 0; j < T; ++j) {
            const float pen = (1.0f - mb[j]) * -1e8f;
            const float pr = __expf(Rb[(size_t)i * T + j] + pen - mr) * isr;
            const float pc = __expf(Rb[(size_t)j * T + i] + pen - mc) * isc;
            a1[i * L + j] = gw * (pr - (j == i ? 1.0f : 0.0f));      // d / d R[i][j]
            a2[i * L + j] = gw * (pc - (j == i ? 1.0f : 0.0f));      // d / d R[j][i]
        }
    }
    const float s0 = wave_sum(c0), s1 = wave_sum(c1), s2 = wave_sum(c2);
    if ((i & 63) == 0) { red[0][i >> 6] = s0; red[1][i >> 6] = s1; red[2][i >> 6] = s2; }
    __syncthreads();
    if (i < 3) part[(size_t)b * 3 + i] = red[i][0] + red[i][1];
    if (i < T) {
        float* o = dR + (size_t)b * T * T + (size_t)i * T;
        float* ot = dRT + (size_t)b * T * T + (size_t)i * T;
        for (int j = 0; j < T; ++j) {
            o[j] = a1[i * L + j] + a2[j * L + i];
            ot[j] = a1[j * L + i] + a2[i * L + j];
        }
    }
}

// Softmax-CE gradient rows against the diagonal labels (F.cross_entropy(logits, arange), pacl.py:574-577):
// g = w (softmax(z) - onehot(row)), loss[row] = logsumexp(z) - z[row] (unweighted).  One wave per row.
__global__ __launch_bounds__(256) void ce_diag_grad_k(const float* __restrict__ z, int R, int C, float w,
                                                      float* __restrict__ g, float* __restrict__ loss) {
    const int lane = threadIdx.x & 63, r = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= R) return;
    const float* zr = z + (size_t)r * C;
    float m = -INFINITY;
    for (int j = lane; j < C; j += 64) m = fmaxf(m, zr[j]);
    m = wave_max(m);
    float s = 0.f;
    for (int j = lane; j < C; j += 64) s += __expf(zr[j] - m);
    s = wave_sum(s);
    const float is = 1.0f / s;
    for (int j = lane; j < C; j += 64) g[(size_t)r * C + j] = w * (__expf(zr[j] - m) * is - (j == r ? 1.0f : 0.0f));
    if (lane == 0) loss[r] = logf(s) + m - zr[r];
}

// out[z][c][r] = in[z][r][c] (+ add[z][c][r] when add is given): 32 x 32 tiles through LDS
__global__ __launch_bounds__(256) void transpose_add_k(const float* __restrict__ in, const float* __restrict__ add,
                                                       float* __restrict__ out, int R, int C) {
    __shared__ float t[32][33];
    const size_t zoff = (size_t)blockIdx.z * R * C;
    const int r0 = blockIdx.y * 32, c0 = blockIdx.x * 32;
    const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;     // 8 rows of 32 per pass
    for (int k = ty; k < 32; k += 8) {
        const int r = r0 + k, c = c0 + tx;
        t[k][tx] = (r < R && c < C) ? in[zoff + (size_t)r * C + c] : 0.f;
    }
    __syncthreads();
    for (int k = ty; k < 32; k += 8) {
        const int c = c0 + k, r = r0 + tx;
        if (c < C && r < R) {
            const size_t o = zoff + (size_t)c * R + r;
            out[o] = t[tx][k] + (add ? add[o] : 0.f);
        }
    }
}

// x[b][p][d] += s * v[b][d]   (the backward of a mean over dim 1, pacl.py:566-567)
__global__ __launch_bounds__(256) void bcast_add_mid_k(float* __restrict__ x, const float* __restrict__ v, int P, int D,
                                                       float s) {
    const int b = blockIdx.z, p = blockIdx.y;
    const int d = blockIdx.x * 256 + threadIdx.x;
    if (d >= D) return;
    x[((size_t)b * P + p) * D + d] += s * v[(size_t)b * D + d];
}

}  // namespace

hipError_t launch_ln_drop(const float* x, const float* w, const float* b, long R, int D, float p, uint64_t seed,
                          long roff, void* out, bool out_bf16, float2* stats, hipStream_t s) {
    if (R <= 0) return hipSuccess;
    if (D % 256 != 0 || D > 1024 || !(p >= 0.f && p < 1.f)) return hipErrorInvalidValue;
    const uint32_t th = drop_thresh(p);
    const float ik = 1.0f / (1.0f - p);
    const dim3 grid((unsigned)((R + 3) / 4));
    if (out_bf16) hipLaunchKernelGGL(ln_drop_k<true>, grid, dim3(256), 0, s, x, w, b, R, D, th, ik, seed, roff, out, stats);
    else hipLaunchKernelGGL(ln_drop_k<false>, grid, dim3(256), 0, s, x, w, b, R, D, th, ik, seed, roff, out, stats);
    return hipGetLastError();
}

long ln_grad_scratch_floats(long R, int D) { return ((R + LNG_ROWS - 1) / LNG_ROWS) * 2L * D; }

hipError_t launch_ln_grad(const float* dy, const float* x, const float2* stats, long R, int D, float p, uint64_t seed,
                          long roff, float* dw, float* db, float* scratch, hipStream_t s) {
    if (R <= 0) return hipSuccess;
    const int nch = (int)((R + LNG_ROWS - 1) / LNG_ROWS);
    hipLaunchKernelGGL(ln_grad_part_k, dim3((unsigned)nch), dim3(256), 0, s, dy, x, stats, R, D, drop_thresh(p),
                       1.0f / (1.0f - p), seed, roff, scratch);
    hipLaunchKernelGGL(ln_grad_finish_k, dim3((unsigned)((2 * D + 255) / 256)), dim3(256), 0, s, scratch, nch, D, dw, db);
    return hipGetLastError();
}

hipError_t launch_align_bwd(const float* S, float* io, long rows, int P, float sigma, hipStream_t s) {
    if (rows <= 0) return hipSuccess;
    hipLaunchKernelGGL(align_bwd_k, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, s, S, io, rows, P, sigma);
    return hipGetLastError();
}

hipError_t launch_local_grad(const float* R, const float* mask, int B, int T, float w, float* dR, float* dRT,
                             float* part, hipStream_t s) {
    if (T > 80) return hipErrorInvalidValue;
    hipLaunchKernelGGL(local_grad_k, dim3((unsigned)B), dim3(128), 0, s, R, mask, T, w, dR, dRT, part);
    return hipGetLastError();
}

hipError_t launch_ce_diag_grad(const float* z, int R, int C, float w, float* g, float* loss, hipStream_t s) {
    if (R <= 0) return hipSuccess;
    hipLaunchKernelGGL(ce_diag_grad_k, dim3((unsigned)((R + 3) / 4)), dim3(256), 0, s, z, R, C, w, g, loss);
    return hipGetLastError();
}

hipError_t launch_transpose_add(const float* in, const float* add, float* out, int batch, int R, int C, hipStream_t s) {
    if (batch <= 0 || R <= 0 || C <= 0) return hipSuccess;
    hipLaunchKernelGGL(transpose_add_k, dim3((unsigned)((C + 31) / 32), (unsigned)((R + 31) / 32), (unsigned)batch),
                       dim3(256), 0, s, in, add, out, R, C);
    return hipGetLastError();
}

hipError_t launch_bcast_add_mid(float* x, const float* v, int B, int P, int D, float scale, hipStream_t s) {
    if (B <= 0 || P <= 0) return hipSuccess;
    hipLaunchKernelGGL(bcast_add_mid_k, dim3((unsigned)((D + 255) / 256), (unsigned)P, (unsigned)B), dim3(256), 0, s, x,
                       v, P, D, scale);
    return hipGetLastError();
}

}  // namespace ce
