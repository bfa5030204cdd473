// Row-wise HBM-bound kernels of the CLIP towers for gfx950: LayerNorm (optionally LN -> RoPE ->
// LN for the PACL head), patchify (im2col), class/positional embeddings, token embedding
// gather, EOT pooling, L2 normalisation, cross-entropy.
//
// Reference semantics:
//   LayerNorm          open_clip/src/open_clip/transformer.py:23-29 (eps 1e-5, biased var)
//   conv1 patchify     transformer.py:549-555,702-704 (14x14/14, no bias; flatten c,ky,kx)
//   cls + pos          transformer.py:707-709
//   token embedding    model.py:286-288
//   argmax pooling     transformer.py:848-851 (torch.argmax -> first maximal index)
//   F.normalize        model.py:281,300 (x / max(||x||, 1e-12))
//   apply_rope         Patch-Aligned-Contrastive-Learning/model/pacl.py:147-181
//   cross_entropy      loss.py:188-191 (mean over rows, ignore_index -100)
#include "ce_device.h"
#include "ce_kernels.h"

namespace ce {
namespace {

__device__ __forceinline__ int map_row(int r, int grp, int gs, int go) {
    if (grp == 0) return r;
    const int g = r / grp;
    return g * gs + go + (r - g * grp);
}

template <int NC>
__device__ __forceinline__ void ln_inplace(float4 (&v)[NC], int D, const float* __restrict__ w,
                                           const float* __restrict__ b, int lane) {
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < NC; ++c) s += (v[c].x + v[c].y) + (v[c].z + v[c].w);
    const float mean = wave_sum(s) / (float)D;
    float q = 0.f;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        v[c].x -= mean; v[c].y -= mean; v[c].z -= mean; v[c].w -= mean;
        q += (v[c].x * v[c].x + v[c].y * v[c].y) + (v[c].z * v[c].z + v[c].w * v[c].w);
    }
    const float rstd = rsqrtf(wave_sum(q) / (float)D + 1e-5f);
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        const int e = c * 256 + lane * 4;
        const float4 ww = *reinterpret_cast<const float4*>(w + e);
        const float4 bb = *reinterpret_cast<const float4*>(b + e);
        v[c].x = v[c].x * rstd * ww.x + bb.x;
        v[c].y = v[c].y * rstd * ww.y + bb.y;
        v[c].z = v[c].z * rstd * ww.z + bb.z;
        v[c].w = v[c].w * rstd * ww.w + bb.w;
    }
}

// One wave per row; 4 rows per 256-thread block.  D = NC * 256.
template <int NC, bool OUT_BF16, bool DOUBLE, bool ROPE, bool STATS = false>
__global__ __launch_bounds__(256) void layernorm_k(LNParams p) {
    __shared__ float rbuf[ROPE ? 4 * NC * 256 : 1];
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int row = blockIdx.x * 4 + wave;
    if (row >= p.rows) return;
    const int D = NC * 256;
    const int irow = map_row(row, p.grp, p.i_gs, p.i_go);
    const int orow = map_row(row, p.grp, p.o_gs, p.o_go);
    const float* x = p.in + (size_t)irow * p.ldi;
    float4 v[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) v[c] = *reinterpret_cast<const float4*>(x + c * 256 + lane * 4);
    ln_inplace<NC>(v, D, p.w, p.b, lane);
    if constexpr (ROPE) {
        // de-interleave rotate: out[i] = x[2i]c_i - x[2i+1]s_i ; out[D/2+i] = x[2i]s_i + x[2i+1]c_i
        float* rb = rbuf + wave * NC * 256;
        const int pos = row % p.rope_P;
        const float* ct = p.rope_cos + (size_t)pos * (D / 2);
        const float* st = p.rope_sin + (size_t)pos * (D / 2);
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            const int i0 = c * 128 + lane * 2;
            const float c0 = ct[i0], s0 = st[i0], c1 = ct[i0 + 1], s1 = st[i0 + 1];
            rb[i0] = v[c].x * c0 - v[c].y * s0;
            rb[D / 2 + i0] = v[c].x * s0 + v[c].y * c0;
            rb[i0 + 1] = v[c].z * c1 - v[c].w * s1;
            rb[D / 2 + i0 + 1] = v[c].z * s1 + v[c].w * c1;
        }
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int c = 0; c < NC; ++c) v[c] = *reinterpret_cast<const float4*>(rb + c * 256 + lane * 4);
    }
    if constexpr (DOUBLE) ln_inplace<NC>(v, D, p.w2, p.b2, lane);
    if constexpr (STATS) {
        // the output row is the next block's residual stream: its bf16 copy and (mu, rstd) feed an
        // LN-folded GEMM (EPI_LN_FOLD) in place of that block's LayerNorm launch
        float sm = 0.f;
#pragma unroll
        for (int c = 0; c < NC; ++c) sm += (v[c].x + v[c].y) + (v[c].z + v[c].w);
        const float mean = wave_sum(sm) / (float)D;
        float q = 0.f;
#pragma unroll
        for (int c = 0; c < NC; ++c)
            q += ((v[c].x - mean) * (v[c].x - mean) + (v[c].y - mean) * (v[c].y - mean)) +
                 ((v[c].z - mean) * (v[c].z - mean) + (v[c].w - mean) * (v[c].w - mean));
        const float rstd = rsqrtf(wave_sum(q) / (float)D + 1e-5f);
        if (lane == 0) p.stats[orow] = make_float2(mean, rstd);
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            uint2 hi, lo;
            split_hl(v[c].x, v[c].y, hi.x, lo.x);
            split_hl(v[c].z, v[c].w, hi.y, lo.y);
            const size_t o = (size_t)orow * p.ldo + c * 256 + lane * 4;
            *reinterpret_cast<uint2*>(p.xb + o) = hi;
            if (p.xlo) *reinterpret_cast<uint2*>(p.xlo + o) = lo;
        }
    }
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        const int e = c * 256 + lane * 4;
        if constexpr (OUT_BF16) {
            uint2 o;
            o.x = pack_bf2(v[c].x, v[c].y);
            o.y = pack_bf2(v[c].z, v[c].w);
            *reinterpret_cast<uint2*>(static_cast<bf16_t*>(p.out) + (size_t)orow * p.ldo + e) = o;
        } else {
            *reinterpret_cast<float4*>(static_cast<float*>(p.out) + (size_t)orow * p.ldo + e) = v[c];
        }
    }
}

template <int NC>
hipError_t ln_dispatch_nc(const LNParams& p, bool out_bf16, hipStream_t s) {
    const dim3 grid((p.rows + 3) / 4);
    const bool dbl = p.w2 != nullptr;
    const bool rope = p.rope_cos != nullptr;
    if (rope && !dbl) return hipErrorInvalidValue;
    if (p.stats || p.xb) {
        if (!p.stats || !p.xb || out_bf16 || dbl || rope) return hipErrorInvalidValue;
        hipLaunchKernelGGL((layernorm_k<NC, false, false, false, true>), grid, dim3(256), 0, s, p);
        return hipGetLastError();
    }
    if (out_bf16) {
        if (rope) hipLaunchKernelGGL((layernorm_k<NC, true, true, true>), grid, dim3(256), 0, s, p);
        else if (dbl) hipLaunchKernelGGL((layernorm_k<NC, true, true, false>), grid, dim3(256), 0, s, p);
        else hipLaunchKernelGGL((layernorm_k<NC, true, false, false>), grid, dim3(256), 0, s, p);
    } else {
        if (rope) hipLaunchKernelGGL((layernorm_k<NC, false, true, true>), grid, dim3(256), 0, s, p);
        else if (dbl) hipLaunchKernelGGL((layernorm_k<NC, false, true, false>), grid, dim3(256), 0, s, p);
        else hipLaunchKernelGGL((layernorm_k<NC, false, false, false>), grid, dim3(256), 0, s, p);
    }
    return hipGetLastError();
}

// ---- patchify ---------------------------------------------------------------------------
template <bool PIX_BF16>
__global__ __launch_bounds__(256) void im2col_k(const void* __restrict__ pix, bf16_t* __restrict__ cols,
                                                int B, int S, int patch, int Kp) {
    const int G = S / patch;
    const long total = (long)B * G * G * Kp;
    const long idx = (long)blockIdx.x * 256 + threadIdx.x;
    if (idx >= total) return;
    const int col = (int)(idx % Kp);
    const long row = idx / Kp;
    const int pp2 = patch * patch;
    float val = 0.f;
    if (col < 3 * pp2) {
        const int b = (int)(row / (G * G));
        const int pidx = (int)(row % (G * G));
        const int py = pidx / G, px = pidx % G;
        const int c = col / pp2, rem = col % pp2;
        const int ky = rem / patch, kx = rem % patch;
        const size_t off = (((size_t)b * 3 + c) * S + (size_t)(py * patch + ky)) * S + px * patch + kx;
        if constexpr (PIX_BF16) val = bf2f(static_cast<const bf16_t*>(pix)[off]);
        else val = static_cast<const float*>(pix)[off];
    }
    cols[idx] = f2bf(val);
}

// Patchify with one wave per patch row for patch 14 (ViT-L/14): lane (c, ky) = (lane / 14, lane % 14),
// lanes 0..41, moves one 14-pixel run of channel c, image row py * 14 + ky (f32: 7 x 8-B loads;
// bf16: 7 x 4-B loads) to columns c * 196 + ky * 14 .. + 13 (7 x 4-B stores of bf16 pairs); lanes
// 42..63 zero the K padding (588 .. Kp - 1, in bf16 pairs).  4 patch rows per 256-thread block.
template <bool PIX_BF16>
__global__ __launch_bounds__(256) void im2col14_k(const void* __restrict__ pix, bf16_t* __restrict__ cols, int rows,
                                                  int S, int Kp) {
    const int lane = threadIdx.x & 63;
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= rows) return;
    const int G = S / 14;
    const int b = row / (G * G), pidx = row - b * (G * G);
    const int py = pidx / G, px = pidx - py * G;
    uint32_t* out = reinterpret_cast<uint32_t*>(cols + (size_t)row * Kp);
    if (lane < 42) {
        const int c = lane / 14, ky = lane - c * 14;
        const size_t off = (((size_t)b * 3 + c) * S + (size_t)(py * 14 + ky)) * S + px * 14;
        uint32_t w[7];
        if constexpr (PIX_BF16) {
            const uint32_t* src = reinterpret_cast<const uint32_t*>(static_cast<const bf16_t*>(pix) + off);
#pragma unroll
            for (int k = 0; k < 7; ++k) w[k] = src[k];
        } else {
            const float2* src = reinterpret_cast<const float2*>(static_cast<const float*>(pix) + off);
#pragma unroll
            for (int k = 0; k < 7; ++k) {
                const float2 v = src[k];
                w[k] = pack_bf2(v.x, v.y);
            }
        }
        uint32_t* dst = out + (c * 196 + ky * 14) / 2;
#pragma unroll
        for (int k = 0; k < 7; ++k) dst[k] = w[k];
    } else {
        for (int q = 294 + (lane - 42); q < Kp / 2; q += 22) out[q] = 0u;
    }
}

__global__ __launch_bounds__(256) void cls_rows_k(float* x, const float* cls, const float* pos, int B,
                                                  int Lv, int D) {
    const int b = blockIdx.y;
    const int d = blockIdx.x * 256 + threadIdx.x;
    if (d < D) x[(size_t)b * Lv * D + d] = cls[d] + pos[d];
}

__global__ __launch_bounds__(256) void text_embed_k(float* x, const int64_t* ids, const float* tok,
                                                    const float* pos, int B, int ctx, int D, int vocab) {
    const int row = blockIdx.x;   // b*ctx + t
    const int t = row % ctx;
    int64_t id = ids[row];
    id = id < 0 ? 0 : (id >= vocab ? vocab - 1 : id);
    const float* tr = tok + (size_t)id * D;
    const float* pr = pos + (size_t)t * D;
    float* xr = x + (size_t)row * D;
    for (int d = threadIdx.x * 4; d < D; d += 1024) {
        const float4 a = *reinterpret_cast<const float4*>(tr + d);
        const float4 c = *reinterpret_cast<const float4*>(pr + d);
        *reinterpret_cast<float4*>(xr + d) = make_float4(a.x + c.x, a.y + c.y, a.z + c.z, a.w + c.w);
    }
}

// Text embedding as the LN-folded text tower's entry state (the tower has no ln_pre): x = tok[id] +
// pos (f32), its hi/lo bf16 planes (xb = hi, xlo = lo, optional) and the row (mu, rstd) that block
// 0's folded QKV GEMM needs in place of ln_1.  One wave per row, D = NC * 256.
template <int NC>
__global__ __launch_bounds__(256) void text_embed_stats_k(float* __restrict__ x, bf16_t* __restrict__ xb,
                                                          bf16_t* __restrict__ xlo, float2* __restrict__ stats,
                                                          const int64_t* __restrict__ ids,
                                                          const float* __restrict__ tok,
                                                          const float* __restrict__ pos, int rows, int ctx,
                                                          int vocab, const int* __restrict__ seg) {
    constexpr int D = NC * 256;
    const int lane = threadIdx.x & 63;
    const int prow = blockIdx.x * 4 + (threadIdx.x >> 6);     // padded row b * ctx + t
    if (prow >= rows) return;
    const int t = prow % ctx;
    int row = prow;
    if (seg) {                                                 // packed: caption b's rows from seg[b]
        const int b = prow / ctx;
        if (t >= seg[b + 1] - seg[b]) return;
        row = seg[b] + t;
    }
    int64_t id = ids[prow];
    id = id < 0 ? 0 : (id >= vocab ? vocab - 1 : id);
    const float* tr = tok + (size_t)id * D;
    const float* pr = pos + (size_t)t * D;
    float4 v[NC];
    float sm = 0.f;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        const int e = c * 256 + lane * 4;
        const float4 a = *reinterpret_cast<const float4*>(tr + e);
        const float4 b = *reinterpret_cast<const float4*>(pr + e);
        v[c] = make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
        sm += (v[c].x + v[c].y) + (v[c].z + v[c].w);
    }
    const float mean = wave_sum(sm) / (float)D;
    float q = 0.f;
#pragma unroll
    for (int c = 0; c < NC; ++c)
        q += ((v[c].x - mean) * (v[c].x - mean) + (v[c].y - mean) * (v[c].y - mean)) +
             ((v[c].z - mean) * (v[c].z - mean) + (v[c].w - mean) * (v[c].w - mean));
    const float rstd = rsqrtf(wave_sum(q) / (float)D + 1e-5f);
    if (lane == 0) stats[row] = make_float2(mean, rstd);
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        const size_t o = (size_t)row * D + c * 256 + lane * 4;
        *reinterpret_cast<float4*>(x + o) = v[c];
        uint2 hi, lo;
        split_hl(v[c].x, v[c].y, hi.x, lo.x);
        split_hl(v[c].z, v[c].w, hi.y, lo.y);
        *reinterpret_cast<uint2*>(xb + o) = hi;
        if (xlo) *reinterpret_cast<uint2*>(xlo + o) = lo;
    }
}

// Packed text rows for pooled-only calls: caption b keeps its rows up to the EOT
// token (the argmax id, ties to the first, as argmax_rows_k) — under the causal mask no later row
// reaches the EOT row — at packed rows seg[b] .. seg[b + 1] - 1; seg[B] = the live row count and
// sel[b] = the packed EOT row.  One workgroup, chunks of 256 captions, block-wide exclusive scan.
__global__ __launch_bounds__(256) void text_pack_k(int* __restrict__ sel, int* __restrict__ seg,
                                                   const int64_t* __restrict__ ids, int B, int ctx) {
    __shared__ int wsum[4];
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    int carry = 0;
    for (int b0 = 0; b0 < B; b0 += 256) {
        const int b = b0 + t;
        int len = 0;
        if (b < B) {
            const int64_t* r = ids + (size_t)b * ctx;
            int64_t best = r[0];
            int bi = 0;
            for (int k = 1; k < ctx; ++k) {
                const int64_t v = r[k];
                if (v > best) { best = v; bi = k; }
            }
            len = bi + 1;
        }
        int inc = len;                                   // inclusive scan inside the wave
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int v = __shfl_up(inc, o, 64);
            if (lane >= o) inc += v;
        }
        if (lane == 63) wsum[wave] = inc;
        __syncthreads();
        int before = carry;
        for (int w = 0; w < wave; ++w) before += wsum[w];
        const int total = wsum[0] + wsum[1] + wsum[2] + wsum[3];
        if (b < B) {
            const int off = before + inc - len;
            seg[b] = off;
            sel[b] = off + len - 1;
        }
        carry += total;
        __syncthreads();
    }
    if (t == 0) seg[B] = carry;
}

__global__ __launch_bounds__(64) void argmax_rows_k(int* rows, const int64_t* ids, int B, int ctx) {
    const int b = blockIdx.x;
    const int lane = threadIdx.x;
    int64_t best = INT64_MIN;
    int bidx = ctx;
    for (int t = lane; t < ctx; t += 64) {
        const int64_t v = ids[(size_t)b * ctx + t];
        if (v > best) { best = v; bidx = t; }
    }
    // reduce: larger value wins, ties -> smaller index
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const int64_t ov = __shfl_xor(best, o, 64);
        const int oi = __shfl_xor(bidx, o, 64);
        if (ov > best || (ov == best && oi < bidx)) { best = ov; bidx = oi; }
    }
    if (lane == 0) rows[b] = b * ctx + bidx;
}

// LayerNorm of gathered rows into a compact f32 buffer (pooled tokens), any D % 4 == 0, D <= 4096.
__global__ __launch_bounds__(256) void ln_gather_k(float* out, const float* x, const int* rows,
                                                   long row_stride, int n, int D, const float* w,
                                                   const float* b) {
    __shared__ float red[2][4];
    const int i = blockIdx.x;
    if (i >= n) return;
    const float* src = x + (size_t)(rows ? rows[i] : i) * row_stride;
    float s = 0.f;
    for (int d = threadIdx.x; d < D; d += 256) s += src[d];
    s = wave_sum(s);
    if ((threadIdx.x & 63) == 0) red[0][threadIdx.x >> 6] = s;
    __syncthreads();
    const float mean = (red[0][0] + red[0][1] + red[0][2] + red[0][3]) / (float)D;
    float q = 0.f;
    for (int d = threadIdx.x; d < D; d += 256) { const float t = src[d] - mean; q += t * t; }
    q = wave_sum(q);
    if ((threadIdx.x & 63) == 0) red[1][threadIdx.x >> 6] = q;
    __syncthreads();
    const float rstd = rsqrtf((red[1][0] + red[1][1] + red[1][2] + red[1][3]) / (float)D + 1e-5f);
    for (int d = threadIdx.x; d < D; d += 256) out[(size_t)i * D + d] = (src[d] - mean) * rstd * w[d] + b[d];
}

__global__ __launch_bounds__(256) void l2norm_k(float* out, const float* x, int rows, int D) {
    const int lane = threadIdx.x & 63;
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= rows) return;
    const float* xr = x + (size_t)row * D;
    float s = 0.f;
    for (int d = lane; d < D; d += 64) s += xr[d] * xr[d];
    s = wave_sum(s);
    const float inv = 1.0f / fmaxf(sqrtf(s), 1e-12f);
    for (int d = lane; d < D; d += 64) out[(size_t)row * D + d] = xr[d] * inv;
}

// per-row CE: accum[0] += lse - logit[label], accum[1] += 1 (rows with label != -100)
__global__ __launch_bounds__(256) void ce_rows_k(float* accum, const float* logits, int R, int C,
                                                 const int64_t* labels) {
    const int lane = threadIdx.x & 63;
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= R) return;
    const int64_t lab = labels[row];
    if (lab == -100) return;
    if (lab < 0 || lab >= C) {
        // F.cross_entropy raises on a label outside [0, C): poison the loss instead of reading
        // past the row (no host sync on the label values)
        if (lane == 0) atomicAdd(&accum[0], NAN);
        return;
    }
    const float* lr = logits + (size_t)row * C;
    float mx = -INFINITY;
    for (int c = lane; c < C; c += 64) mx = fmaxf(mx, lr[c]);
    mx = wave_max(mx);
    float s = 0.f;
    for (int c = lane; c < C; c += 64) s += expf(lr[c] - mx);
    s = wave_sum(s);
    if (lane == 0) {
        const float loss = (logf(s) + mx) - lr[lab];
        atomicAdd(&accum[0], loss);
        atomicAdd(&accum[1], 1.0f);
    }
}
__global__ void ce_finish_k(float* loss, const float* accum) {
    loss[0] = accum[1] > 0.f ? accum[0] / accum[1] : NAN;
}

__global__ __launch_bounds__(256) void rope_k(float* out, const float* x, int B, int P, int D,
                                              const float* ct, const float* st) {
    const long row = blockIdx.x;         // b*P + p
    const int p = (int)(row % P);
    const float* xr = x + row * D;
    const int half = D / 2;
    float lo[8], hi[8];
    int cnt = 0;
    for (int i = threadIdx.x; i < half && cnt < 8; i += 256, ++cnt) {
        const float a = xr[2 * i], bb = xr[2 * i + 1];
        const float c = ct[(size_t)p * half + i], s = st[(size_t)p * half + i];
        lo[cnt] = a * c - bb * s;
        hi[cnt] = a * s + bb * c;
    }
    __syncthreads();   // x and out may alias
    cnt = 0;
    for (int i = threadIdx.x; i < half && cnt < 8; i += 256, ++cnt) {
        out[row * D + i] = lo[cnt];
        out[row * D + half + i] = hi[cnt];
    }
}

__global__ __launch_bounds__(256) void f32_to_bf16_k(bf16_t* out, const float* in, long n) {
    const long i = (long)blockIdx.x * 256 + threadIdx.x;
    if (i < n) out[i] = f2bf(in[i]);
}

// (mu, rstd) of a row from equal-count (64-column) slab statistics (mean_s, M2_s):
// mu = mean of the means, M2 = sum M2_s + 64 sum (mean_s - mu)^2 (Chan et al.), var = M2 / (64 n)
// 16 lanes per row, lane k reading slab k (k, k+16, ...): the row's partials are one coalesced
// 128-B read for D = 1024; Chan's combine of equal-size (64-column) slabs
__global__ __launch_bounds__(256) void ln_stats_finalize_k(float2* __restrict__ stats, const float2* __restrict__ part,
                                                           int rows, int nslab, const int* __restrict__ m_dev) {
    const int r = blockIdx.x * 16 + (threadIdx.x >> 4), k0 = threadIdx.x & 15;
    if (m_dev) rows = min(rows, *m_dev);                 // packed rows: the live count
    const bool live = r < rows;
    const float2* pr = part + (size_t)(live ? r : 0) * nslab;
    float2 v[4];
    float sm = 0.f;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        const int k = k0 + 16 * t;
        v[t] = (live && k < nslab) ? pr[k] : make_float2(0.f, 0.f);
        sm += v[t].x;
    }
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) sm += __shfl_xor(sm, o, 64);
    const float mu = sm / (float)nslab;
    float m2 = 0.f;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        if (k0 + 16 * t < nslab) {
            const float d = v[t].x - mu;
            m2 += v[t].y + 64.0f * d * d;
        }
    }
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) m2 += __shfl_xor(m2, o, 64);
    if (live && k0 == 0) stats[r] = make_float2(mu, rsqrtf(m2 / (64.0f * nslab) + 1e-5f));
}

// The same for an even nslab <= 16 (D = 1024 / 768): 8 lanes per row, lane k holding slabs 2k and
// 2k + 1 (one 16-B load), two rows 32 apart per lane, so every lane has two loads in flight (the
// one-8-B-load-per-lane form above was latency-bound: 71 % of its wave cycles parked in s_waitcnt)
__global__ __launch_bounds__(256) void ln_stats_finalize16_k(float2* __restrict__ stats, const float2* __restrict__ part,
                                                             int rows, int nslab, const int* __restrict__ m_dev) {
    if (m_dev) rows = min(rows, *m_dev);
    const int k0 = threadIdx.x & 7;
    const int rb = blockIdx.x * 64 + (threadIdx.x >> 3);
    const bool has = 2 * k0 < nslab;
    float4 v[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        const int r = rb + 32 * u;
        v[u] = (r < rows && has) ? *reinterpret_cast<const float4*>(part + (size_t)r * nslab + 2 * k0)
                                 : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        float sm = v[u].x + v[u].z;
#pragma unroll
        for (int o = 1; o < 8; o <<= 1) sm += __shfl_xor(sm, o, 64);
        const float mu = sm / (float)nslab;
        const float d0 = v[u].x - mu, d1 = v[u].z - mu;
        float m2 = has ? (v[u].y + 64.0f * d0 * d0) + (v[u].w + 64.0f * d1 * d1) : 0.f;
#pragma unroll
        for (int o = 1; o < 8; o <<= 1) m2 += __shfl_xor(m2, o, 64);
        const int r = rb + 32 * u;
        if (r < rows && k0 == 0) stats[r] = make_float2(mu, rsqrtf(m2 / (64.0f * nslab) + 1e-5f));
    }
}

}  // namespace

hipError_t launch_ln_stats_finalize(float2* stats, const float2* part, int rows, int nslab, hipStream_t s,
                                    const int* m_dev) {
    if (rows <= 0) return hipSuccess;
    if (nslab <= 0 || nslab > 64) return hipErrorInvalidValue;
    if (nslab <= 16 && nslab % 2 == 0 && ((uintptr_t)part & 15) == 0) {
        hipLaunchKernelGGL(ln_stats_finalize16_k, dim3((unsigned)((rows + 63) / 64)), dim3(256), 0, s, stats, part,
                           rows, nslab, m_dev);
        return hipGetLastError();
    }
    hipLaunchKernelGGL(ln_stats_finalize_k, dim3((unsigned)((rows + 15) / 16)), dim3(256), 0, s, stats, part, rows,
                       nslab, m_dev);
    return hipGetLastError();
}

hipError_t launch_layernorm(const LNParams& p, bool out_bf16, hipStream_t s) {
    if (p.rows <= 0) return hipSuccess;
    if (p.D % 256 != 0) return hipErrorInvalidValue;
    switch (p.D / 256) {
        case 2: return ln_dispatch_nc<2>(p, out_bf16, s);
        case 3: return ln_dispatch_nc<3>(p, out_bf16, s);
        case 4: return ln_dispatch_nc<4>(p, out_bf16, s);
        case 5: return ln_dispatch_nc<5>(p, out_bf16, s);
        case 6: return ln_dispatch_nc<6>(p, out_bf16, s);
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_im2col(const void* pix, bool pix_bf16, bf16_t* cols, int B, int S, int patch,
                         int Kp, hipStream_t s) {
    const int G = S / patch;
    if (patch == 14 && Kp % 2 == 0 && Kp >= 588 && S % 2 == 0) {
        const int rows = B * G * G;
        const dim3 g4((unsigned)((rows + 3) / 4));
        if (pix_bf16) hipLaunchKernelGGL(im2col14_k<true>, g4, dim3(256), 0, s, pix, cols, rows, S, Kp);
        else hipLaunchKernelGGL(im2col14_k<false>, g4, dim3(256), 0, s, pix, cols, rows, S, Kp);
        return hipGetLastError();
    }
    const long total = (long)B * G * G * Kp;
    const dim3 grid((unsigned)((total + 255) / 256));
    if (pix_bf16) hipLaunchKernelGGL(im2col_k<true>, grid, dim3(256), 0, s, pix, cols, B, S, patch, Kp);
    else hipLaunchKernelGGL(im2col_k<false>, grid, dim3(256), 0, s, pix, cols, B, S, patch, Kp);
    return hipGetLastError();
}

hipError_t launch_cls_rows(float* x, const float* cls, const float* pos, int B, int Lv, int D,
                           hipStream_t s) {
    hipLaunchKernelGGL(cls_rows_k, dim3((D + 255) / 256, B), dim3(256), 0, s, x, cls, pos, B, Lv, D);
    return hipGetLastError();
}

hipError_t launch_text_embed(float* x, const int64_t* ids, const float* tok, const float* pos, int B,
                             int ctx, int D, int vocab, hipStream_t s) {
    if (D % 4) return hipErrorInvalidValue;
    hipLaunchKernelGGL(text_embed_k, dim3(B * ctx), dim3(256), 0, s, x, ids, tok, pos, B, ctx, D, vocab);
    return hipGetLastError();
}

hipError_t launch_text_embed_stats(float* x, bf16_t* xb, bf16_t* xlo, float2* stats, const int64_t* ids,
                                   const float* tok, const float* pos, int B, int ctx, int D, int vocab,
                                   hipStream_t s, const int* seg) {
    const int rows = B * ctx;
    const dim3 grid((unsigned)((rows + 3) / 4));
    if (!x || !xb || !stats) return hipErrorInvalidValue;
    if (D == 768) hipLaunchKernelGGL(text_embed_stats_k<3>, grid, dim3(256), 0, s, x, xb, xlo, stats, ids, tok, pos, rows, ctx, vocab, seg);
    else if (D == 512) hipLaunchKernelGGL(text_embed_stats_k<2>, grid, dim3(256), 0, s, x, xb, xlo, stats, ids, tok, pos, rows, ctx, vocab, seg);
    else if (D == 1024) hipLaunchKernelGGL(text_embed_stats_k<4>, grid, dim3(256), 0, s, x, xb, xlo, stats, ids, tok, pos, rows, ctx, vocab, seg);
    else if (D == 1280) hipLaunchKernelGGL(text_embed_stats_k<5>, grid, dim3(256), 0, s, x, xb, xlo, stats, ids, tok, pos, rows, ctx, vocab, seg);
    else if (D == 256) hipLaunchKernelGGL(text_embed_stats_k<1>, grid, dim3(256), 0, s, x, xb, xlo, stats, ids, tok, pos, rows, ctx, vocab, seg);
    else return hipErrorInvalidValue;
    return hipGetLastError();
}

hipError_t launch_text_pack(int* sel, int* seg, const int64_t* ids, int B, int ctx, hipStream_t s) {
    if (B <= 0 || ctx <= 0) return hipErrorInvalidValue;
    hipLaunchKernelGGL(text_pack_k, dim3(1), dim3(256), 0, s, sel, seg, ids, B, ctx);
    return hipGetLastError();
}

hipError_t launch_argmax_rows(int* rows, const int64_t* ids, int B, int ctx, hipStream_t s) {
    hipLaunchKernelGGL(argmax_rows_k, dim3(B), dim3(64), 0, s, rows, ids, B, ctx);
    return hipGetLastError();
}

hipError_t launch_ln_gather(float* out, const float* x, const int* rows, long row_stride, int n, int D,
                            const float* w, const float* b, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(ln_gather_k, dim3(n), dim3(256), 0, s, out, x, rows, row_stride, n, D, w, b);
    return hipGetLastError();
}

hipError_t launch_l2norm(float* out, const float* x, int rows, int D, hipStream_t s) {
    if (rows <= 0) return hipSuccess;
    hipLaunchKernelGGL(l2norm_k, dim3((rows + 3) / 4), dim3(256), 0, s, out, x, rows, D);
    return hipGetLastError();
}

hipError_t launch_cross_entropy_rows(float* accum, const float* logits, int R, int C,
                                     const int64_t* labels, hipStream_t s) {
    hipLaunchKernelGGL(ce_rows_k, dim3((R + 3) / 4), dim3(256), 0, s, accum, logits, R, C, labels);
    return hipGetLastError();
}
hipError_t launch_cross_entropy_finish(float* loss, const float* accum, hipStream_t s) {
    hipLaunchKernelGGL(ce_finish_k, dim3(1), dim3(1), 0, s, loss, accum);
    return hipGetLastError();
}

hipError_t launch_rope(float* out, const float* x, int B, int P, int D, const float* cos_t,
                       const float* sin_t, hipStream_t s) {
    if (D % 2 || D / 2 > 8 * 256) return hipErrorInvalidValue;
    hipLaunchKernelGGL(rope_k, dim3(B * P), dim3(256), 0, s, out, x, B, P, D, cos_t, sin_t);
    return hipGetLastError();
}

hipError_t launch_f32_to_bf16(bf16_t* out, const float* in, long n, hipStream_t s) {
    hipLaunchKernelGGL(f32_to_bf16_k, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, out, in, n);
    return hipGetLastError();
}

}  // namespace ce
