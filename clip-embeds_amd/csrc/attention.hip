// Fused multi-head attention forward (flash-style, online softmax) for gfx950.
//
// Replaces the nn.MultiheadAttention core inside ResidualAttentionBlock.attention
// (open_clip/src/open_clip/transformer.py:242-255): softmax(q k^T / sqrt(64) + mask) v per head,
// with the additive causal -inf mask of the text tower (transformer.py:960-966).
//
// Layout: qkv [B*L][3D] bf16 as produced by the in_proj GEMM (q | k | v, head h at columns
// h*64..h*64+63 of each third, nn.MultiheadAttention packing); out [B*L][D] bf16.
//
// Design:
//  * workgroup = 4 waves = 128 queries of one (batch, head); each wave owns 32 queries.
//  * K/V tiles of 64 keys staged global->LDS with global_load_lds_dwordx4 into a 2-deep ring
//    (next tile issued before the current one is consumed, counted vmcnt).
//  * "Swapped" QK^T: S^T = K Q^T with v_mfma_f32_32x32x16_bf16 so each lane holds one query
//    (lane&31) and 32 of the tile's keys in registers — the row max/sum are in-lane plus one
//    cross-half exchange (lanes l, l^32).
//  * P stays in registers: the S^T accumulator, packed to bf16, is directly the B operand of
//    O^T = V^T P^T (no LDS round trip); V^T fragments come from ds_read_b64_tr_b16 on the
//    row-major V tile.  O^T keeps the query on the lane, so the online-softmax rescale is a
//    per-lane scalar.
//  * K tile LDS image swizzled (16-B chunk c of row r at c ^ ((r>>1)&7)) for conflict-free
//    ds_read_b128; ragged tails (L = 577 = 9*64 + 1, L = 77) are clamped on load and masked
//    with -inf in the scores.
#include <cstdio>
#include <type_traits>

#include "ce_device.h"
#include "ce_kernels.h"
#include "knobs.h"

namespace ce {
namespace {

typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2_t;

constexpr int QBLK = 128;
constexpr int KBLK = 64;
constexpr int TILE_KV_BYTES = KBLK * 64 * 2;       // 8 KB per K or V tile
constexpr int STAGE_BYTES = 2 * TILE_KV_BYTES;      // K + V

__device__ __forceinline__ s16x4 ds_read_tr16(const char* p) {
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16((CE_LDS s16x4*)(p));
}
// The same read as inline asm: with the builtin, hipcc waits vmcnt(0) before it (it cannot tell the
// V tile being read from the next tile's LDS-DMA in flight), so every key tile waited for its
// successor's K/V transfer in the middle of its P.V MFMAs.  The caller waits lgkmcnt itself.
__device__ __forceinline__ s16x4 ds_read_tr16_asm(const char* p) {
    s16x4 r;
    asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(r) : "v"((unsigned)(uintptr_t)(CE_LDS void*)p));
    return r;
}

// buffer descriptor from wave-uniform inputs (readfirstlane: no waterfall loops, guide T20)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t attn_srd(const void* base, int nbytes) {
    const uint64_t b = reinterpret_cast<uint64_t>(base);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)b);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32));
    const int n = __builtin_amdgcn_readfirstlane(nbytes);
    return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(((uint64_t)hi << 32) | lo), (short)0, n,
                                             0x00020000);
}

__device__ __forceinline__ void barrier() {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

// Variants (the VAR bits; set_attn_variant selects among the instantiated ones, DESIGN.md §6.6,
// §6.9, §6.12): MODE (bits 0-1) 0 = every tile on the general online-softmax path; 1 = "fixed-offset"
// tiles: once tile 0 has shown every row max of the wave within +-64 (log2 units), the softmax offset
// stays 0 and full tiles skip the row max, the accumulator moves and the subtraction (p = exp2(q.k)
// directly; bf16 P has the f32 exponent range, O and l the same factor), with an overflow check on
// the row sums (any p > 2^64 or inf/NaN: the tile is redone with the exact max and the wave returns
// to the general path).  Every instantiation has the 16-B output stores (bit 8), the inline-asm V^T
// reads (bit 16) and the buffer-descriptor K/V DMAs (bit 64).  Instantiated: 381 (non-causal
// L = 64k + 1, default), 125 (non-causal, other L), 88 (causal).  (Measured and removed in round 6:
// MFMA row sums, a three-slot ring, early prologue loads, per-wave timelines and the persistent
// variants)
template <bool CAUSAL, int VAR>
__global__ __launch_bounds__(256, 2) void attn_fwd(const bf16_t* __restrict__ qkv,
                                                    bf16_t* __restrict__ out, int Lp, int H,
                                                    float qscale, float* __restrict__ lse,
                                                    const int* __restrict__ seg) {
    static_assert((VAR & (8 | 16 | 64)) == (8 | 16 | 64) && (VAR & 3) <= 1, "attn_fwd: instantiated variant set");
    __shared__ __attribute__((aligned(16))) char smem[2 * STAGE_BYTES];
    constexpr int MODE = VAR & 3;            // softmax: 0 general, 1 fixed offset
    constexpr bool ONEBAR = (VAR & 4) != 0;  // one barrier per key tile (next tile staged after it)
    constexpr bool FAST0 = (VAR & 32) != 0;  // tile 0 on the fixed offset too (two-sided check)
    // CLSK (bit 256, non-causal, (L - 1) % 64 == 0): key 0 (the CLS token) enters the softmax up
    // front (one 64-d dot product per query on the VALU, O and l initialised with its term) and the
    // key tiles cover keys 1..L-1: L = 577 runs 9 full tiles instead of 9 + one single-key tile on the
    // masked general path
    constexpr bool CLSK = !CAUSAL && (VAR & 256) != 0;
    // XCD-aware bijective remap (as the GEMM): consecutive wgids = the q-blocks of one head, so
    // every workgroup that re-reads a head's K/V runs on the same XCD and shares its L2.
    const int nqb = (Lp + QBLK - 1) / QBLK;
    const int nwg = gridDim.x;
    const int bid = blockIdx.x;
    const int xcd = bid & 7, qn = nwg >> 3, rn = nwg & 7;
    const int wgid = (xcd < rn ? xcd * (qn + 1) : rn * (qn + 1) + (xcd - rn) * qn) + (bid >> 3);
    const int bh = wgid / nqb;
    const int qb = wgid - bh * nqb;
    const int b = bh / H, h = bh - b * H;
    const int D = H * 64;
    const long ld = 3L * D;
    // packed sequences (seg: the text tower's pooled-only rows, launch_text_pack): sequence b is
    // rows seg[b] .. seg[b + 1] - 1; q-blocks past its end exit
    int L = Lp;
    long row0 = (long)b * Lp;
    if (seg) {
        row0 = seg[b];
        L = seg[b + 1] - seg[b];
        if (qb * QBLK >= L) return;
    }
    const bf16_t* base = qkv + (size_t)row0 * ld;

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int r = lane & 31;
    const int h2 = lane >> 5;
    const int qrow = qb * QBLK + wave * 32 + r;
    const int q_wave0 = qb * QBLK + wave * 32;        // first query of this wave (wave-uniform)

    // Q fragments: B operand of S^T = K Q^T; lane holds Q[qrow][16ks + 8h2 .. +7]
    bf16x8 qf[4];
    {
        const bf16_t* qp = base + (size_t)min(qrow, L - 1) * ld + h * 64 + 8 * h2;
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) qf[ks] = *reinterpret_cast<const bf16x8*>(qp + 16 * ks);
        // scores in log2 units: q is pre-multiplied by log2(e)/sqrt(64), either here (qscale != 1,
        // the raw-qkv kernel entry) or already by the in_proj weights the engine uploads
        if (qscale != 1.0f) {
#pragma unroll
            for (int ks = 0; ks < 4; ++ks)
#pragma unroll
                for (int e = 0; e < 8; ++e) qf[ks][e] = (__bf16)((float)qf[ks][e] * qscale);
        }
    }

    // staging: thread -> row tid>>3 of a 32-row pass, 16-B chunk tid&7
    const int srow = tid >> 3;
    const int spos = tid & 7;
    const int kchunk = spos ^ ((tid >> 4) & 7);
    const int vchunk = spos ^ (((srow >> 1) & 1) << 2);   // V image swizzle (conflict-free tr reads)
    const int Lk = CLSK ? L - 1 : L;                     // keys covered by the tiles
    const int kv_end = CAUSAL ? min(L, qb * QBLK + QBLK) : Lk;
    const int nkt = (kv_end + KBLK - 1) / KBLK;
    const bf16_t* kbase = base + D + h * 64 + (CLSK ? ld : 0);
    const bf16_t* vbase = base + 2 * D + h * 64 + (CLSK ? ld : 0);

    // the K / V columns of this (b, h) as buffer descriptors clipped after row L - 1 (rows past the
    // end read zeros: masked keys), per-lane row/chunk offsets computed once, the tile's row offset
    // one scalar add per DMA (the flat form rebuilt 64-bit addresses with 64-bit multiplies for
    // every DMA)
    const int ld2 = (int)ld * 2;
    const int nrec = (Lk - 1) * ld2 + 128;
    const __amdgpu_buffer_rsrc_t ksrd = attn_srd(kbase, nrec);
    const __amdgpu_buffer_rsrc_t vsrd = attn_srd(vbase, nrec);
    int kvo[2], vvo[2];
#pragma unroll
    for (int ps = 0; ps < 2; ++ps) {
        kvo[ps] = (ps * 32 + srow) * ld2 + kchunk * 16;
        vvo[ps] = (ps * 32 + srow) * ld2 + vchunk * 16;
    }
    auto stage = [&](int t, int buf) {
        char* dst = smem + buf * STAGE_BYTES + wave * 1024;
        const int ro = t * KBLK * ld2;
#pragma unroll
        for (int ps = 0; ps < 2; ++ps) {
            __builtin_amdgcn_raw_ptr_buffer_load_lds(ksrd, (CE_LDS void*)(dst + ps * 4096), 16, kvo[ps] + ro, 0, 0, 0);
            __builtin_amdgcn_raw_ptr_buffer_load_lds(vsrd, (CE_LDS void*)(dst + TILE_KV_BYTES + ps * 4096), 16,
                                                     vvo[ps] + ro, 0, 0, 0);
        }
    };

    // per-lane LDS read offsets
    int koff[2][4];
#pragma unroll
    for (int kt2 = 0; kt2 < 2; ++kt2)
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
            const int row = kt2 * 32 + r;
            koff[kt2][ks] = row * 128 + (((2 * ks + h2) ^ ((row >> 1) & 7)) << 4);
        }
    // V^T via ds_read_b64_tr_b16: 16-lane group G supplies rows (keys) kb + 4*(G>>1) + q,
    // columns dt*32 + 16*(G&1) + 4*p (q = i>>2, p = i&3); the 16-B chunk of that address is
    // XOR-ed with 4*((row>>1)&1) = 4*((q>>1)&1) (rows kb + 4*(G>>1) are multiples of 4).
    const int G = lane >> 4, gi = lane & 15;
    const int vq = gi >> 2, vp = gi & 3;
    int voff[2];
#pragma unroll
    for (int dt = 0; dt < 2; ++dt) {
        const int chunk = dt * 4 + 2 * (G & 1) + (vp >> 1);
        voff[dt] = (4 * (G >> 1) + vq) * 128 + ((chunk ^ (((vq >> 1) & 1) << 2)) << 4) + (vp & 1) * 8;
    }

    f32x16 o[2];
#pragma unroll
    for (int i = 0; i < 16; ++i) { o[0][i] = 0.f; o[1][i] = 0.f; }
    float m_run = 0.f;   // running row max (log2 units); set exactly by the first tile
    float l_run = 0.f;   // partial (this half's keys)
    // wave-uniform: softmax offset fixed at 0 (MODE >= 1).  FAST0 (bit 32): tile 0 too starts on the
    // fixed offset, its row sums checked from both sides (2^-64 <= sum <= 2^64: no row can underflow
    // to l = 0 later); a row outside sends tile 0 to the general path, which sets the exact max
    bool fast = MODE >= 1 && FAST0;
    const f32x16 zero16 = {};
    // CLSK: key 0's score (log2 units, both lane halves) and its term in O / l.  Offset 0 (the fixed
    // offset) when every query of the wave has |s0| <= 64, else the exact s0 (general path)
    float s0v = 0.f;
    bool fix_ok = true;                      // wave-uniform: the offset may stay fixed at 0
    if constexpr (CLSK) {
        const bf16_t* k0 = base + D + h * 64 + 8 * h2;
        float a = 0.f;
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
            const bf16x8 kv = *reinterpret_cast<const bf16x8*>(k0 + 16 * ks);
            // (f32 FMAs: v_dot2_f32_bf16 here, with the packed multiplies below, took the kernel to 126
            // VGPRs and four waves per SIMD, 1 % slower than three in a same-box A/B)
#pragma unroll
            for (int e = 0; e < 8; ++e) a = fmaf((float)qf[ks][e], (float)kv[e], a);
        }
        s0v = a + __shfl_xor(a, 32, 64);
        fix_ok = MODE >= 1 && __all(s0v <= 64.0f && s0v >= -64.0f);
        float p0 = 1.0f;
        if (fix_ok) p0 = __builtin_amdgcn_exp2f(s0v);
        else { m_run = s0v; fast = false; }
        if (h2 == 0) l_run = p0;
        const bf16_t* v0 = base + 2 * D + h * 64;
#pragma unroll
        for (int dt = 0; dt < 2; ++dt)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const uint2 w = *reinterpret_cast<const uint2*>(v0 + dt * 32 + 8 * g + 4 * h2);
                o[dt][4 * g + 0] = p0 * __uint_as_float(w.x << 16);
                o[dt][4 * g + 1] = p0 * __uint_as_float(w.x & 0xffff0000u);
                o[dt][4 * g + 2] = p0 * __uint_as_float(w.y << 16);
                o[dt][4 * g + 3] = p0 * __uint_as_float(w.y & 0xffff0000u);
            }
    }

    // O^T += V^T P^T with the V^T fragments read by inline asm (no wait on the LDS-DMA in flight):
    // the reads of 16-key group q + 1 are issued before the MFMAs of group q, counted lgkmcnt.
    // Addresses: one lane base per dt (smem + voff[dt]) plus compile-time immediates (VB = the V
    // tile of ring slot BUF), so the reads need no address VGPRs of their own.
    unsigned vaddr[2];
#pragma unroll
    for (int dt = 0; dt < 2; ++dt) vaddr[dt] = (unsigned)(uintptr_t)(CE_LDS void*)(smem + voff[dt]);
    auto pv_asm = [&](auto vbc, const bf16x8 (&pf)[2][2], bool with_half2) {
        constexpr int VB = decltype(vbc)::value;
        typedef __attribute__((ext_vector_type(8))) short s16x8;
        s16x4 vr[2][2][2];        // [ring][dt][lo, hi]
#define CE_TRV(R, DT, H, OFF) \
    asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(vr[R][DT][H]) : "v"(vaddr[DT]), "n"(OFF))
#define CE_ISSUE(Q) \
    CE_TRV((Q) & 1, 0, 0, VB + (((Q) >> 1) * 32 + 16 * ((Q) & 1)) * 128); \
    CE_TRV((Q) & 1, 0, 1, VB + (((Q) >> 1) * 32 + 16 * ((Q) & 1)) * 128 + 1024); \
    CE_TRV((Q) & 1, 1, 0, VB + (((Q) >> 1) * 32 + 16 * ((Q) & 1)) * 128); \
    CE_TRV((Q) & 1, 1, 1, VB + (((Q) >> 1) * 32 + 16 * ((Q) & 1)) * 128 + 1024)
        auto mf = [&](int q) {
#pragma unroll
            for (int dt = 0; dt < 2; ++dt) {
                const s16x8 v8 = __builtin_shufflevector(vr[q & 1][dt][0], vr[q & 1][dt][1], 0, 1, 2, 3, 4, 5, 6, 7);
                o[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, v8), pf[q >> 1][q & 1],
                                                               o[dt], 0, 0, 0);
            }
        };
        // one 16-key group at a time (issuing the next group ahead holds 16 more VGPRs: 156 > 128,
        // three waves per SIMD instead of four); the other waves on the SIMD cover the LDS latency
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            if (q >= 2 && !with_half2) break;
            if (q == 0) { CE_ISSUE(0); }
            else if (q == 1) { CE_ISSUE(1); }
            else if (q == 2) { CE_ISSUE(2); }
            else { CE_ISSUE(3); }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_sched_barrier(0);
            mf(q);
        }
#undef CE_ISSUE
#undef CE_TRV
    };

    // rescale of O and l by 2^-delta (delta per lane, equal on lanes l and l^32)
    auto rescale = [&](float delta) {
        const float alpha = __builtin_amdgcn_exp2f(-delta);
        l_run *= alpha;
#pragma unroll
        for (int i = 0; i < 16; ++i) { o[0][i] *= alpha; o[1][i] *= alpha; }
        m_run += delta;
    };

    stage(0, 0);
    // one key tile; BUF (the ring slot, t & 1) is a compile-time constant so every LDS address is a
    // per-lane offset plus an immediate (the loop is unrolled by two)
    auto tile = [&](const int t, auto bufc) {
        constexpr int BUF = decltype(bufc)::value;
        if (ONEBAR) {
            // tile t landed (the only DMA in flight) and every wave is done with tile t-1, whose
            // slot BUF^1 then takes tile t+1
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
            barrier();
            if (t + 1 < nkt) stage(t + 1, BUF ^ 1);
        } else {
            if (t + 1 < nkt) {
                stage(t + 1, BUF ^ 1);
                asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
            } else {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            barrier();
        }
        const char* kb = smem + BUF * STAGE_BYTES;
        const char* vb = kb + TILE_KV_BYTES;

        // waves whose queries are all padding, or (causal) whose queries all precede this key
        // tile, skip the math but keep the workgroup barriers
        const bool active = q_wave0 < L && !(CAUSAL && t * KBLK > q_wave0 + 31);
        // second 32-key subtile entirely past the sequence end (L = 577: the last tile holds one
        // key) or (causal) entirely above this wave's diagonal: skip its MFMAs and exponentials
        const bool half2 = (t * KBLK + 32 < Lk) && !(CAUSAL && t * KBLK + 32 > q_wave0 + 31);
        const int key0 = t * KBLK;
        // masking only on the ragged last tile and (causal) on tiles that cross the diagonal
        const bool need_mask = (key0 + KBLK > Lk) || (CAUSAL && key0 + KBLK - 1 > q_wave0);
        const bool fast_tile = MODE >= 1 && fast && half2 && !need_mask;   // wave-uniform
        bool redo = false;
        if (active && fast_tile) {
            // ---- fixed-offset tile: S^T = K Q^T from a zero accumulator, p = exp2(s) ----
            f32x16 s[2];
#pragma unroll
            for (int kt2 = 0; kt2 < 2; ++kt2)
#pragma unroll
                for (int ks = 0; ks < 4; ++ks) {
                    const bf16x8 kf = *reinterpret_cast<const bf16x8*>(kb + koff[kt2][ks]);
                    s[kt2] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[ks], ks == 0 ? zero16 : s[kt2], 0, 0, 0);
                }
            float ps[4] = {0.f, 0.f, 0.f, 0.f};
            bf16x8 pf[2][2];
#pragma unroll
            for (int kt2 = 0; kt2 < 2; ++kt2)
#pragma unroll
                for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        const float pv_ = __builtin_amdgcn_exp2f(s[kt2][8 * s2 + j]);
                        ps[j & 3] += pv_;
                        pf[kt2][s2][j] = (__bf16)pv_;
                    }
            const float psum = (ps[0] + ps[1]) + (ps[2] + ps[3]);
            // (!(x <= 2^64) also catches NaN)
            const bool overflow = __any(!(psum <= 0x1p64f)) || (FAST0 && t == 0 && __any(!(psum >= 0x1p-64f)));
            if (!overflow) {
                l_run += psum;
                __builtin_amdgcn_sched_barrier(0);
                pv_asm(std::integral_constant<int, BUF * STAGE_BYTES + TILE_KV_BYTES>{}, pf, true);
            } else {
                // rare: the tile is redone on the general path below (exact row max, rescale),
                // and the wave stays there
                fast = false;
                redo = true;
            }
        }
        if (active && (redo || !(MODE >= 1 && fast_tile))) {
            // ---- S^T = K Q^T (two 32-key subtiles) ----
            f32x16 s[2];
    #pragma unroll
            for (int kt2 = 0; kt2 < 2; ++kt2) {
    #pragma unroll
                for (int i = 0; i < 16; ++i) s[kt2][i] = kt2 == 1 && !half2 ? -INFINITY : -m_run;
                if (kt2 == 1 && !half2) continue;
    #pragma unroll
                for (int ks = 0; ks < 4; ++ks) {
                    const bf16x8 kf = *reinterpret_cast<const bf16x8*>(kb + koff[kt2][ks]);
                    s[kt2] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[ks], s[kt2], 0, 0, 0);
                }
            }

            // ---- online softmax, log2 domain.  The S accumulator starts at -m_run, so the MFMA
            // leaves s = q.k - m_run (q pre-scaled): p = exp2(s) needs no per-score FMA ----
            if (need_mask) {
    #pragma unroll
                for (int kt2 = 0; kt2 < 2; ++kt2)
    #pragma unroll
                    for (int i = 0; i < 16; ++i) {
                        const int key = key0 + kt2 * 32 + (i & 3) + 8 * (i >> 2) + 4 * h2;
                        const bool masked = (key >= Lk) || (CAUSAL && key > qrow);
                        s[kt2][i] = masked ? -INFINITY : s[kt2][i];
                    }
            }
            float tmax = s[0][0];
    #pragma unroll
            for (int kt2 = 0; kt2 < 2; ++kt2)
    #pragma unroll
                for (int i = (kt2 == 0 ? 1 : 0); i < 16; ++i) tmax = fmaxf(tmax, s[kt2][i]);
            tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));    // relative to m_run
            // Deferred rescale (guide T13): m_run moves on the first tile (to the exact row max:
            // key 0 is never masked, so it is finite) and afterwards only when a row max exceeds
            // it by more than the threshold (8, or 64 with the offset fixed at 0), so p stays far
            // from the f32 / bf16 overflow and O / l are rarely rescaled.  O and l always see the
            // same factor, and the decision precedes this tile's P, so no P.V product straddles it.
            // VARs >= 1: when tile 0's row maxima all lie within +-64, the offset stays 0.
            // (CLSK: O / l already hold key 0's term, so the first move rescales them, and the exact
            // max includes key 0; the fixed offset needs key 0 on it too)
            const bool fix0 = MODE >= 1 && t == 0 && fix_ok && __all(tmax <= 64.0f && tmax >= -64.0f);
            if (fix0) fast = true;
            if (!fix0 && (t == 0 || __any(tmax > (fast ? 64.0f : 8.0f)))) {
                const float delta = t == 0 ? (CLSK ? fmaxf(tmax, s0v - m_run) : tmax) : fmaxf(tmax, 0.f);
                if (t != 0 || CLSK) rescale(delta);
                else m_run += delta;
                fast = false;
    #pragma unroll
                for (int kt2 = 0; kt2 < 2; ++kt2)
    #pragma unroll
                    for (int i = 0; i < 16; ++i) s[kt2][i] -= delta;
            }
            float psum = 0.f;
            bf16x8 pf[2][2];
    #pragma unroll
            for (int kt2 = 0; kt2 < 2; ++kt2)
    #pragma unroll
                for (int s2 = 0; s2 < 2; ++s2)
    #pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        if (kt2 == 1 && !half2) { pf[kt2][s2][j] = (__bf16)0.f; continue; }
                        const float pv_ = __builtin_amdgcn_exp2f(s[kt2][8 * s2 + j]);
                        psum += pv_;
                        pf[kt2][s2][j] = (__bf16)pv_;
                    }
            l_run += psum;
            pv_asm(std::integral_constant<int, BUF * STAGE_BYTES + TILE_KV_BYTES>{}, pf, half2);
        }
        if (!ONEBAR) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            barrier();
        }
    };
    for (int t = 0; t < nkt; t += 2) {
        tile(t, std::integral_constant<int, 0>{});
        if (t + 1 < nkt) tile(t + 1, std::integral_constant<int, 1>{});
    }

    // ---- epilogue: O = O^T / l, lane holds query qrow, d = dt*32 + 8g + 4h2 + (0..3) ----
    const float l_tot = l_run + __shfl_xor(l_run, 32, 64);
    const float inv = 1.0f / l_tot;
    // training: log2-domain log-sum-exp of the row (P = exp2(S - lse) in the attention backward)
    if (lse && qrow < L && h2 == 0) lse[((size_t)b * H + h) * Lp + qrow] = m_run + __log2f(l_tot);
    bf16_t* op = out + ((size_t)row0 + min(qrow, L - 1)) * D + h * 64;
    {
        // 16-B stores: lane h2 = 0 holds d = 8g + 0..3 and its partner l^32 d = 8g + 4..7: v_permlane32_swap
        // trades the lower lane's odd-g words for the upper lane's even-g words, so each lane
        // stores 8 consecutive d (16 B): the lower lane d = 16gp + 0..7, the upper 16gp + 8..15
#pragma unroll
        for (int dt = 0; dt < 2; ++dt)
#pragma unroll
            for (int gp = 0; gp < 2; ++gp) {
                const int g0 = 2 * gp, g1 = 2 * gp + 1;
                const uint32_t ax = pack_bf2(o[dt][4 * g0 + 0] * inv, o[dt][4 * g0 + 1] * inv);
                const uint32_t ay = pack_bf2(o[dt][4 * g0 + 2] * inv, o[dt][4 * g0 + 3] * inv);
                const uint32_t bx = pack_bf2(o[dt][4 * g1 + 0] * inv, o[dt][4 * g1 + 1] * inv);
                const uint32_t by = pack_bf2(o[dt][4 * g1 + 2] * inv, o[dt][4 * g1 + 3] * inv);
                const auto x = __builtin_amdgcn_permlane32_swap(ax, bx, false, false);
                const auto y = __builtin_amdgcn_permlane32_swap(ay, by, false, false);
                if (qrow < L)
                    *reinterpret_cast<uint4*>(op + dt * 32 + 16 * gp + 8 * h2) = make_uint4(x[0], y[0], x[1], y[1]);
            }
    }
}

std::atomic<int> g_attn_var{381};     // A/B knob (knobs.h: process-wide atomic)

// One query row per (batch, head) against all of its sequence's keys (keys 0..pos with the causal
// mask): the attention of a tower's last block when only the pooled row is consumed (CLS row b*L
// of the image tower, the EOT row qrows[b] of the text tower).  Workgroup =
// (head, batch), 256 threads: scores with four lanes per key (32 B each, two lane-pair sums),
// block max / sum, then P.V with 16 key slots x 16 four-column groups and a fixed-order slot sum.
// Same arithmetic as attn_fwd where it matters: q pre-scaled by log2(e)/8 (the engine's in_proj
// weights), scores in log2 units, p = exp2(s - max); P stays f32 here.
// wq (optional): the pooled row's q is computed here instead of read from qkv (the QKV GEMM then
// covers only K and V): the LN-folded in_proj of that row, q = rstd (x W'^T - mu c) + d rounded to
// bf16 as the GEMM's output, with x = the hi plane row (src), (mu, rstd) = stats[row].
// src/dst (optional): copies the pooled row's 64 columns of the hi/lo residual planes to compact
// planes (the residual of the pruned out-projection).
__global__ __launch_bounds__(256) void attn_rows_k(const bf16_t* __restrict__ qkv, const int* __restrict__ qrows,
                                                   int L, int H, int causal, bf16_t* __restrict__ out,
                                                   const bf16_t* __restrict__ src, long splane,
                                                   bf16_t* __restrict__ dst, long dplane, const int* __restrict__ seg,
                                                   const bf16_t* __restrict__ wq, const float* __restrict__ cq,
                                                   const float* __restrict__ dq, const float2* __restrict__ stats) {
    extern __shared__ float sc[];                 // [L]: scores, then probabilities
    __shared__ float qs[64];
    __shared__ float red[2][4];
    __shared__ float pv[16][68];
    const int h = blockIdx.x, b = blockIdx.y;
    const int D = H * 64;
    const long ld = 3L * D;
    const long row0 = seg ? (long)seg[b] : (long)b * L;
    const long qr = qrows ? (long)qrows[b] : row0;
    const int nk = causal ? (int)(qr - row0) + 1 : L;
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    if (wq) {
        // q[j]: wave w takes columns j = 16w .. 16w + 15, each a dot product of the whole row over
        // the wave (lane l: 16-B chunks l, l + 64, ... of x and of W' row j: coalesced 1-KB loads)
        const int nch = D / 8;
        const uint4* xr = reinterpret_cast<const uint4*>(src + qr * D);
        uint4 xv[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) xv[c] = (lane + 64 * c < nch) ? xr[lane + 64 * c] : make_uint4(0u, 0u, 0u, 0u);
        for (int jj = 0; jj < 16; ++jj) {
            const int j = wave * 16 + jj;
            const uint4* wr = reinterpret_cast<const uint4*>(wq + (long)(h * 64 + j) * D);
            float a = 0.f;
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                if (lane + 64 * c < nch) {
                    const uint4 w = wr[lane + 64 * c], x = xv[c];
                    const uint32_t xs[4] = {x.x, x.y, x.z, x.w}, ws[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        a = fmaf(__uint_as_float(xs[e] << 16), __uint_as_float(ws[e] << 16), a);
                        a = fmaf(__uint_as_float(xs[e] & 0xffff0000u), __uint_as_float(ws[e] & 0xffff0000u), a);
                    }
                }
            }
            a = wave_sum(a);
            if (lane == 0) {
                const float2 st = stats[qr];
                const int n = h * 64 + j;
                qs[j] = bf2f(f2bf(fmaf(st.y, fmaf(-st.x, cq[n], a), dq[n])));
            }
        }
    } else if (t < 64) {
        qs[t] = bf2f(qkv[qr * ld + h * 64 + t]);
    }
    if (src && t < 128) {
        const int pl = t >> 6;
        dst[pl * dplane + (long)b * D + h * 64 + lane] = src[pl * splane + qr * D + h * 64 + lane];
    }
    __syncthreads();
    // scores: key j = t / 4 + 64 i, dims (t & 3) * 16 .. + 15 of it per lane
    float m = -INFINITY;
    const int part = t & 3;
    float qp[16];
#pragma unroll
    for (int e = 0; e < 16; ++e) qp[e] = qs[part * 16 + e];
    for (int j = t >> 2; j < nk; j += 64) {
        const uint4* kp = reinterpret_cast<const uint4*>(qkv + (row0 + j) * ld + D + h * 64 + part * 16);
        const uint4 u0 = kp[0], u1 = kp[1];
        const uint32_t w[8] = {u0.x, u0.y, u0.z, u0.w, u1.x, u1.y, u1.z, u1.w};
        float s = 0.f;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            s = fmaf(qp[2 * e], __uint_as_float(w[e] << 16), s);
            s = fmaf(qp[2 * e + 1], __uint_as_float(w[e] & 0xffff0000u), s);
        }
        s += __shfl_xor(s, 1, 64);
        s += __shfl_xor(s, 2, 64);
        if (part == 0) sc[j] = s;
        m = fmaxf(m, s);
    }
    m = wave_max(m);
    if (lane == 0) red[0][wave] = m;
    __syncthreads();
    m = fmaxf(fmaxf(red[0][0], red[0][1]), fmaxf(red[0][2], red[0][3]));
    float l = 0.f;
    for (int j = t; j < nk; j += 256) {
        const float p = exp2f(sc[j] - m);
        sc[j] = p;
        l += p;
    }
    l = wave_sum(l);
    if (lane == 0) red[1][wave] = l;
    __syncthreads();
    l = (red[1][0] + red[1][1]) + (red[1][2] + red[1][3]);
    const int ks = t >> 4, d0 = (t & 15) * 4;
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
    const bf16_t* vb = qkv + row0 * ld + 2 * D + h * 64 + d0;
    for (int j = ks; j < nk; j += 16) {
        const uint2 v = *reinterpret_cast<const uint2*>(vb + j * ld);
        const float p = sc[j];
        a0 = fmaf(p, __uint_as_float(v.x << 16), a0);
        a1 = fmaf(p, __uint_as_float(v.x & 0xffff0000u), a1);
        a2 = fmaf(p, __uint_as_float(v.y << 16), a2);
        a3 = fmaf(p, __uint_as_float(v.y & 0xffff0000u), a3);
    }
    pv[ks][d0] = a0; pv[ks][d0 + 1] = a1; pv[ks][d0 + 2] = a2; pv[ks][d0 + 3] = a3;
    __syncthreads();
    if (t < 64) {
        float o = 0.f;
#pragma unroll
        for (int k2 = 0; k2 < 16; ++k2) o += pv[k2][t];
        out[(long)b * D + h * 64 + t] = f2bf(o / l);
    }
}

}  // namespace

hipError_t launch_attention_rows(const bf16_t* qkv, const int* qrows, bf16_t* out, int B, int L, int H, bool causal,
                                 const bf16_t* src, long splane, bf16_t* dst, long dplane, hipStream_t s,
                                 const int* seg, const bf16_t* wq, const float* cq, const float* dq,
                                 const float2* stats) {
    if (B <= 0 || L <= 0) return hipSuccess;
    if ((size_t)L * 4 > 96 * 1024 || B > 65535) return hipErrorInvalidValue;
    if (seg && (!qrows || !causal)) return hipErrorInvalidValue;
    if (wq && (!src || !cq || !dq || !stats || H * 64 > 4 * 64 * 8)) return hipErrorInvalidValue;
    hipLaunchKernelGGL(attn_rows_k, dim3(H, B), dim3(256), (size_t)L * 4, s, qkv, qrows, L, H, causal ? 1 : 0, out,
                       src, splane, dst, dplane, seg, wq, cq, dq, stats);
    return hipGetLastError();
}

hipError_t launch_attention(const bf16_t* qkv, bf16_t* out, int B, int L, int H, bool causal, bool q_prescaled,
                            hipStream_t s, float* lse, const int* seg) {
    if (B <= 0 || L <= 0) return hipSuccess;
    const dim3 grid((unsigned)(((L + QBLK - 1) / QBLK) * H * B));
    const float qscale = q_prescaled ? 1.0f : kAttnQScale;
#define CE_ATTN_LAUNCH(C, V) hipLaunchKernelGGL((attn_fwd<C, V>), grid, dim3(256), 0, s, qkv, out, L, H, qscale, lse, seg)
    // the text tower's causal tiles all cross the diagonal or the ragged end: general softmax
    const int v = g_attn_var.load(std::memory_order_acquire);
    if (causal) {
        CE_ATTN_LAUNCH(true, 88);
    } else if (v == 381 && (L - 1) % KBLK == 0 && L > 1) {
        // key 0 first (CLSK) needs the keys after the first to fill whole tiles
        CE_ATTN_LAUNCH(false, 381);
    } else {
        CE_ATTN_LAUNCH(false, 125);
    }
#undef CE_ATTN_LAUNCH
    return hipGetLastError();
}

int set_attn_variant(int var) {
    // 381: key 0 ahead of the key tiles where (L - 1) % 64 == 0 (default); 125: the key tiles only
    return g_attn_var.exchange(var == 125 ? 125 : 381);
}

}  // namespace ce
