// bf16 MFMA GEMM with fused epilogues for gfx950 (CDNA4).
//
// Computes every nn.Linear / patch-conv of the CLIP towers (open_clip transformer.py:228,235-239,
// 549-555 — in_proj, out_proj, c_fc, c_proj, conv1) as  out = act(A W^T + bias) + resid
// with A = activations [M][K] and W = nn.Linear weight [N][K], both K-contiguous.
//
// Design:
//  * 256x256 output tile per 512-thread workgroup (8 waves, 2 along M x 4 along N, each wave
//    128(M) x 64(N) = 8x4 MFMA tiles of v_mfma_f32_16x16x32_bf16, 128 f32 accumulators/lane).
//  * BK = 64; A and W tiles (32 KB each) are staged global->LDS with global_load_lds_dwordx4
//    into a 2-stage ring (128 KB LDS, one workgroup per CU); the stage for tile t+2 is issued
//    right after tile t is consumed, so each load has a full tile of MFMA work to land.
//    Waits are counted (vmcnt(8) = one stage in flight) around raw s_barriers.
//  * LDS image: 128-B rows, 16-B chunk c of row r stored at chunk c ^ ((r>>1)&7) — makes the
//    16-lane ds_read_b128 groups bank-conflict free.  The global source address carries the
//    inverse permutation (glds writes lane-linearly).
//  * Operands are swapped in the MFMA (W fragment as A, activation fragment as B) so each lane
//    ends with 4 consecutive output columns of one row: the epilogue does 16-B f32 / 8-B bf16
//    stores and float4 bias/residual loads.
//  * Workgroup -> tile map is XCD-aware (bijective round-robin remap): consecutive tiles of one
//    A row-panel land on the same XCD and share its L2.
#include "ce_device.h"
#include "ce_kernels.h"
#include "knobs.h"

#include <algorithm>
#include <type_traits>
#include <utility>
#include <atomic>
#include <cstdlib>
#include <mutex>

#ifndef CE_RESID_RING
#define CE_RESID_RING 4
#endif

namespace ce {

namespace {

constexpr int BM = 256, BN = 256, BK = 64;
constexpr int NTHREADS = 512;
constexpr int TILE_BYTES = BM * BK * 2;        // 32 KB per operand tile (BM == BN)
constexpr int STAGE_BYTES = 2 * TILE_BYTES;    // A + W

__device__ __forceinline__ void compiler_fence() { asm volatile("" ::: "memory"); }
__device__ __forceinline__ void barrier() {
    compiler_fence();
    __builtin_amdgcn_s_barrier();
    compiler_fence();
}

__device__ __forceinline__ int map_row(int m, int grp, int gs, int go) {
    if (grp == 0) return m;
    const int g = m / grp;
    return g * gs + go + (m - g * grp);
}

__device__ __forceinline__ void wait_vm(int n) {
    // n is a small compile-time constant after inlining/unrolling
    if (n <= 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else if (n == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    else if (n == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
}


// Epilogue: lane holds C[m = mbase + 16i + (lane&15)][n = nbase + 16j + 4(lane>>4) .. +3].
// vmcnt counts stores as well as loads and retires in order, so a residual/bias load issued after
// earlier stores waits for those stores too: bias is loaded once up front and the residual rows of
// fragment row i+1 are issued before the stores of row i (two-deep register ring), so each store
// batch has a full row of work to drain behind it.
// Buffer descriptor from provably wave-uniform inputs: without the readfirstlanes hipcc keeps the
// words in VGPRs and wraps every buffer op in a waterfall loop (guide T20).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_srd(const void* base, int nbytes) {
    const uint64_t b = reinterpret_cast<uint64_t>(base);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)b);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32));
    const int n = __builtin_amdgcn_readfirstlane(nbytes);
    return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(((uint64_t)hi << 32) | lo), (short)0, n,
                                             0x00020000);
}

// LN-folded consumer operands of one wave's 128 x 16*NJ output block: per-column c_n and per-row
// (mu, rstd).  CE_FOLD_PREFETCH=1 loads them at kernel start instead of at the epilogue; measured
// 8% slower on the c_fc shape (registers held across the main loop), so off.
template <int NJ>
struct FoldOps {
    float4 c[NJ];
    float2 st[8];
    __device__ __forceinline__ void load(const GemmParams& p, int mbase, int nbase, int lane) {
        const int fr = lane & 15, fq = lane >> 4;
#pragma unroll
        for (int j = 0; j < NJ; ++j) c[j] = *reinterpret_cast<const float4*>(p.fold_c + nbase + j * 16 + fq * 4);
#pragma unroll
        for (int i = 0; i < 8; ++i) st[i] = p.fold_stats[min(mbase + i * 16 + fr, p.M - 1)];
    }
};

// cache policy of the GEMM epilogues' output stores (buffer-store aux bits; gfx950: 1 = sc0, 2 = nt,
// 16 = sc1).  0 = plain (the line stays in the XCD's L2); an A/B build with 16 (sc1: written through
// and dropped from the L2) leaves the L2 to the operand panels
#ifndef CE_STORE_AUX
#define CE_STORE_AUX 0
#endif

#ifndef CE_FOLD_PREFETCH
#define CE_FOLD_PREFETCH 0
#endif

// kernel-variant bits (set_gemm_variant / env CE_GEMM_VARIANT), default GEMM_VAR_DEFAULT.  Bit values
// are kept from earlier rounds; the bits of the schedules measured and removed in round 6 (ablations,
// DMA-split alternatives, SCHED 13 / 14 routing) are gone, and the two DMA-spread bits are always on.
enum { GEMM_VAR_W4PP_NOWAIT = 1,
       // the four-wave kernels' epilogues for one wave per SIMD (operands in an LDS side area); off: the
       // residual-free and LN-statistics GEMMs stay on SCHED 1
       GEMM_VAR_W4_EPI2 = 2,
       // the four-wave schedule with one tile per workgroup (grid = tiles): an exiting workgroup's
       // stores drain while the next one on the CU starts, instead of ahead of the next tile's DMAs
       GEMM_VAR_W4_ONETILE = 16,
       // split-K tail on the four-wave persistent schedule (a last round of <= 1/8 of the grid).
       // Off by default; on a GELU GEMM its tail tiles finish in gemm_splitk_fixup with the
       // polynomial GELU (gelu_pair, <= 2.5e-6) while the main tiles use gelu_fast4 (<= 6.2e-5):
       // both far inside the bf16 output rounding, but A/B timings of this bit mix two epilogues
       GEMM_VAR_W4_TAIL = 32,
       // the hi/lo residual GEMMs (EPI_LN_STATS_HL) on the staged-residual four-wave kernel
       GEMM_VAR_W4_RHL = 128,
       // (always on since round 6) a K-tile's 16 operand DMAs spread over B2 and B3
       GEMM_VAR_W4_DMA_SPREAD = 256, GEMM_VAR_RHL_DMA_SPREAD = 512,
       // honour GemmParams::onetile: the caller's small grids (text tower) on the four-wave kernels
       // with one tile per workgroup instead of the 8-wave 4-phase kernel
       GEMM_VAR_SMALL_ONETILE = 8192 };
#ifndef CE_GEMM_VAR_DEFAULT
#define CE_GEMM_VAR_DEFAULT \
    (GEMM_VAR_W4PP_NOWAIT | GEMM_VAR_W4_EPI2 | GEMM_VAR_W4_RHL | GEMM_VAR_W4_DMA_SPREAD | GEMM_VAR_RHL_DMA_SPREAD | \
     GEMM_VAR_SMALL_ONETILE)
#endif

template <int ACT, bool HAS_RESID, bool OUT_BF16, bool CHECK_M, int NJ, int RING, int EPI = EPI_PLAIN>
__device__ __forceinline__ void gemm_epilogue_rows(const GemmParams& p, const f32x4 (&acc)[8][NJ], int mbase,
                                                   int nbase, int lane, const FoldOps<NJ>* pre = nullptr) {
    const int fr = lane & 15, fq = lane >> 4;
    // LN statistics of the output (x of the residual stream) and the hi/lo bf16 residual planes
    constexpr bool STATS = EPI == EPI_LN_STATS || EPI == EPI_LN_STATS_HL;
    constexpr bool HL_IN = EPI == EPI_LN_STATS_HL || EPI == EPI_HL_F32;
    constexpr bool HL_OUT = EPI == EPI_LN_STATS_HL;
    // LN-folded consumer: per-column c_n and per-row (mu, rstd), loaded before any store is issued
    FoldOps<NJ> fo;
    if constexpr (EPI == EPI_LN_FOLD) {
        if (pre) fo = *pre;
        else fo.load(p, mbase, nbase, lane);
    }
    const float4 (&foldc)[NJ] = fo.c;
    const float2 (&fst)[8] = fo.st;
    // bias through a buffer descriptor: a null bias gets num_records 0 and reads zeros, with no branch
    const __amdgpu_buffer_rsrc_t bsrd = make_srd(p.bias ? (const void*)p.bias : (const void*)p.A, p.bias ? p.N * 4 : 0);
    float4 bias[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
        const int n = nbase + j * 16 + fq * 4;
        bias[j] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(bsrd, n * 4, 0, 0));
    }
    // 16-column blocks inside N (wave-uniform; N % 64 == 0, so a 64-column slab is whole and only
    // the 128-column slabs of SCHED 2 can be cut)
    const int jmax = NJ > 4 ? min(NJ, (p.N - nbase) / 16) : NJ;
    // residual rows are prefetched RD-1 fragment rows ahead (RD-deep register ring): one HBM latency
    // per RD-1 rows instead of one per row
    constexpr int RD = NJ > 4 ? 2 : RING;
    float4 rbuf[RD][NJ];
    auto load_resid = [&](int i, float4 (&r)[NJ]) {
        int m = mbase + i * 16 + fr;
        if constexpr (CHECK_M) m = m < p.M ? m : p.M - 1;     // clamp: a valid row, result unused
        const size_t ro = (size_t)map_row(m, p.grp, p.r_gs, p.r_go) * p.ldr + nbase + fq * 4;
        if constexpr (HL_IN) {
            uint2 hi[NJ], lo[NJ];
#pragma unroll
            for (int j = 0; j < NJ; ++j)
                if (j < jmax) {
                    hi[j] = *reinterpret_cast<const uint2*>(p.rhl + ro + j * 16);
                    lo[j] = *reinterpret_cast<const uint2*>(p.rhl + p.hl_plane + ro + j * 16);
                }
#pragma unroll
            for (int j = 0; j < NJ; ++j)
                if (j < jmax) {
                    const float2 a = join_hl(hi[j].x, lo[j].x), c = join_hl(hi[j].y, lo[j].y);
                    r[j] = make_float4(a.x, a.y, c.x, c.y);
                }
        } else {
            const float* rp = p.resid + ro;
#pragma unroll
            for (int j = 0; j < NJ; ++j)
                if (j < jmax) r[j] = *reinterpret_cast<const float4*>(rp + j * 16);
        }
    };
    if constexpr (HAS_RESID) {
#pragma unroll
        for (int i = 0; i < RD - 1; ++i) load_resid(i, rbuf[i]);
    }
    uint2 pend[NJ];      // bf16 output: packed values of the even fragment row, awaiting its partner
    uint2 pxb[NJ];       // EPI_LN_STATS: bf16 copy of the even fragment row (16-B stores as for pend)
    uint2 plo[NJ];       // EPI_LN_STATS_HL: lo plane of the even fragment row
    // EPI_LN_STATS, per 64-column slab (NJ/4 of them): (mean, M2) of fragment rows fq and fq + 4
    // (this lane stores them) and the running (mean, M2) of this lane's values of the current row
    constexpr int NS = NJ / 4;
    float2 sta[NS], stb[NS];
    float lmean[NS], lm2[NS];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        if constexpr (HAS_RESID) {
            if (i + RD - 1 < 8) load_resid(i + RD - 1, rbuf[(i + RD - 1) % RD]);
        }
        const int m = mbase + i * 16 + fr;
        if constexpr (CHECK_M && !OUT_BF16 && !STATS) {
            if (m >= p.M) continue;
        }
        const size_t obase = (size_t)map_row(m, p.grp, p.o_gs, p.o_go) * p.ldo + nbase + fq * 4;
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            if (j >= jmax) break;
            f32x4 v = acc[i][j];
            if constexpr (EPI == EPI_LN_FOLD) {
                // LN(x) W^T + b = rstd (x~ W'^T - mu c) + (b + W beta), W' = gamma o W (weight upload)
                const float mu = fst[i].x, rs = fst[i].y;
                v[0] = fmaf(rs, fmaf(-mu, foldc[j].x, v[0]), bias[j].x);
                v[1] = fmaf(rs, fmaf(-mu, foldc[j].y, v[1]), bias[j].y);
                v[2] = fmaf(rs, fmaf(-mu, foldc[j].z, v[2]), bias[j].z);
                v[3] = fmaf(rs, fmaf(-mu, foldc[j].w, v[3]), bias[j].w);
            } else {
                v[0] += bias[j].x; v[1] += bias[j].y; v[2] += bias[j].z; v[3] += bias[j].w;
            }
            if constexpr (ACT == ACT_GELU) {
                const f32x2 lo = gelu_pair(f32x2{v[0], v[1]}), hi = gelu_pair(f32x2{v[2], v[3]});
                v[0] = lo.x; v[1] = lo.y; v[2] = hi.x; v[3] = hi.y;
            } else {
                v[0] = apply_act<ACT>(v[0]); v[1] = apply_act<ACT>(v[1]);
                v[2] = apply_act<ACT>(v[2]); v[3] = apply_act<ACT>(v[3]);
            }
            if constexpr (HAS_RESID) {
                const float4 rr = rbuf[i % RD][j];
                v[0] += rr.x; v[1] += rr.y; v[2] += rr.z; v[3] += rr.w;
            }
            if constexpr (OUT_BF16) {
                uint2 o;
                o.x = pack_bf2(v[0], v[1]);
                o.y = pack_bf2(v[2], v[3]);
                if ((i & 1) == 0) {
                    pend[j] = o;
                } else {
                    // 16-B stores (guide T21): v_permlane16_swap trades the even row's columns
                    // 4q+4..4q+7 (held by the odd 16-lane group) for the odd row's columns 4q..4q+3,
                    // so an even-group lane ends with 8 consecutive columns of row i-1 and an
                    // odd-group lane with 8 of row i — half the store instructions of 8-B stores
                    const auto x = __builtin_amdgcn_permlane16_swap(pend[j].x, o.x, false, false);
                    const auto y = __builtin_amdgcn_permlane16_swap(pend[j].y, o.y, false, false);
                    const bool odd = (fq & 1) != 0;
                    const int mrow = odd ? m : m - 16;
                    bool ok = true;
                    if constexpr (CHECK_M) ok = mrow < p.M;
                    if (ok) {
                        const size_t ob = (size_t)map_row(mrow, p.grp, p.o_gs, p.o_go) * p.ldo + nbase +
                                          (fq & ~1) * 4 + j * 16;
                        *reinterpret_cast<uint4*>(static_cast<bf16_t*>(p.out) + ob) =
                            make_uint4(x[0], y[0], x[1], y[1]);
                    }
                }
            } else {
                // (the stats epilogue runs the past-the-end rows of the last M tile, with clamped
                // residual rows, so that each even row still meets its odd partner below)
                if (!HL_OUT && (!STATS || !CHECK_M || m < p.M))
                    *reinterpret_cast<float4*>(static_cast<float*>(p.out) + obase + j * 16) =
                        make_float4(v[0], v[1], v[2], v[3]);
                if constexpr (STATS) {
                    // Chan's pairwise update: the 4 values of block j join the lane's 4j earlier ones
                    const float m4 = ((v[0] + v[1]) + (v[2] + v[3])) * 0.25f;
                    const float d0 = v[0] - m4, d1 = v[1] - m4, d2 = v[2] - m4, d3 = v[3] - m4;
                    const float q4 = fmaf(d0, d0, fmaf(d1, d1, fmaf(d2, d2, d3 * d3)));
                    const int sl = j >> 2, jj = j & 3;
                    if (jj == 0) {
                        lmean[sl] = m4;
                        lm2[sl] = q4;
                    } else {
                        const float dl = m4 - lmean[sl];
                        lmean[sl] = fmaf(dl, 1.0f / (jj + 1), lmean[sl]);
                        lm2[sl] += fmaf(dl * dl, 4.0f * jj / (jj + 1), q4);
                    }
                    uint2 o, ol;
                    if constexpr (HL_OUT) {
                        split_hl(v[0], v[1], o.x, ol.x);
                        split_hl(v[2], v[3], o.y, ol.y);
                    } else {
                        o = make_uint2(pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3]));
                    }
                    if ((i & 1) == 0) {
                        pxb[j] = o;
                        if constexpr (HL_OUT) plo[j] = ol;
                    } else {
                        const auto x = __builtin_amdgcn_permlane16_swap(pxb[j].x, o.x, false, false);
                        const auto y = __builtin_amdgcn_permlane16_swap(pxb[j].y, o.y, false, false);
                        const int mrow = (fq & 1) ? m : m - 16;
                        const size_t ob = (size_t)mrow * p.ldo + nbase + (fq & ~1) * 4 + j * 16;
                        if (!CHECK_M || mrow < p.M)
                            *reinterpret_cast<uint4*>(p.xb + ob) = make_uint4(x[0], y[0], x[1], y[1]);
                        if constexpr (HL_OUT) {
                            const auto xl = __builtin_amdgcn_permlane16_swap(plo[j].x, ol.x, false, false);
                            const auto yl = __builtin_amdgcn_permlane16_swap(plo[j].y, ol.y, false, false);
                            if (!CHECK_M || mrow < p.M)
                                *reinterpret_cast<uint4*>(p.xb + p.hl_plane + ob) = make_uint4(xl[0], yl[0], xl[1], yl[1]);
                        }
                    }
                }
            }
        }
        if constexpr (STATS) {
            // (mean, M2) of this row's 64-column slab: 4 lanes (fq) of 4*NJ values each, combined
            // with Chan's formula for equal counts
#pragma unroll
            for (int sl = 0; sl < NS; ++sl) {
                float sm = lmean[sl];
                sm += __shfl_xor(sm, 16, 64);
                sm += __shfl_xor(sm, 32, 64);
                const float mean = sm * 0.25f;
                const float dl = lmean[sl] - mean;
                float q = fmaf(dl * dl, 16.0f, lm2[sl]);
                q += __shfl_xor(q, 16, 64);
                q += __shfl_xor(q, 32, 64);
                // every lane now holds the row's result: lane group fq keeps rows fq and fq + 4
                if (fq == (i & 3)) {
                    if (i < 4) sta[sl] = make_float2(mean, q);
                    else stb[sl] = make_float2(mean, q);
                }
            }
        }
    }
    if constexpr (STATS) {
        // stored after all other stores (no divergent store inside the loop to upset vmcnt counting)
        const int ma = mbase + fq * 16 + fr, mb = ma + 64;
        const size_t ns = p.N / 64;
#pragma unroll
        for (int sl = 0; sl < NS; ++sl) {
            if (!CHECK_M || ma < p.M) p.stats_part[(size_t)ma * ns + nbase / 64 + sl] = sta[sl];
            if (!CHECK_M || mb < p.M) p.stats_part[(size_t)mb * ns + nbase / 64 + sl] = stb[sl];
        }
    }
}

// Epilogue: lane holds C[m = mbase + 16i + (lane&15)][n = nbase + 16j + 4(lane>>4) .. +3].
// vmcnt counts stores as well as loads and retires in order, so a residual/bias load issued after
// earlier stores waits for those stores too: bias is loaded once up front and the residual rows of
// fragment row i+1 are issued before the stores of row i (two-deep register ring).  Column slabs
// are whole (N % 64 == 0), so the only bounds check is on rows, and only in the last M tile: the
// interior path has no divergent branch, which keeps hipcc's waitcnt counting exact.
template <int ACT, bool HAS_RESID, bool OUT_BF16, int NJ = 4, int RING = CE_RESID_RING, int EPI = EPI_PLAIN>
__device__ __forceinline__ void gemm_epilogue(const GemmParams& p, const f32x4 (&acc)[8][NJ], int mbase, int nbase,
                                              int lane, const FoldOps<NJ>* pre = nullptr) {
    if (nbase >= p.N) return;                                   // wave-uniform
    if (mbase + 128 <= p.M)
        gemm_epilogue_rows<ACT, HAS_RESID, OUT_BF16, false, NJ, RING, EPI>(p, acc, mbase, nbase, lane, pre);
    else
        gemm_epilogue_rows<ACT, HAS_RESID, OUT_BF16, true, NJ, RING, EPI>(p, acc, mbase, nbase, lane, pre);
}


// ------------------------------------------------------------------------------------------
// Four-wave (SCHED 11) epilogue for bf16 outputs without a residual (QKV / c_fc: bias or LN fold,
// optional activation).  Lane holds acc[i][j] = C[mbase + 16i + fr][nbase + 16j + 4fq .. +3].
// Written for one wave per SIMD, where nothing hides a stall:
//  * every load it needs (bias, fold columns, row statistics) is issued before its first store —
//    vmcnt retires loads and stores in issue order, so a load issued after stores would wait for
//    all of them;
//  * stores go through a buffer descriptor based at the quadrant's first row whose size ends at row
//    M: rows past M are dropped by the hardware range check, so there is no per-row branch, and the
//    addresses are one 32-bit VGPR (row-pair step added to it, 16-column step in the immediate);
//  * two fragment rows are paired with v_permlane16_swap so each lane stores 16 B (8 columns).
using u32x4 = __attribute__((ext_vector_type(4))) unsigned int;
using u32x2 = __attribute__((ext_vector_type(2))) unsigned int;

template <int ACT>
__device__ __forceinline__ float w4_act(float v) {
    if constexpr (ACT == ACT_GELU) return gelu_fast(v);
    else return apply_act<ACT>(v);
}

// Per-wave side area of the four-wave kernel's LDS (after the two 64-KB stage buffers): bias and
// LN-fold column sums of the wave's 128 columns, (mu, rstd) of its 128 rows.  Filled by LDS-DMA
// during the tile's last K-tile (retired by that K-tile's own vmcnt wait), read by ds_read in the
// epilogue, so the epilogue issues no global load at all.
constexpr int W4_SIDE_BYTES = 3 * 1024;     // [bias 512 B + pad][fold_c 512 B + pad][stats 1 KB]

template <int EPI>
__device__ __forceinline__ void w4_side_fill(const GemmParams& p, char* side, int mbase, int nbase, int lane) {
    const __amdgpu_buffer_rsrc_t bsrd = make_srd(p.bias ? (const void*)p.bias : (const void*)p.A, p.bias ? p.N * 4 : 0);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(bsrd, (CE_LDS void*)side, 16, (nbase + lane * 4) * 4, 0, 0, 0);
    if constexpr (EPI == EPI_LN_FOLD) {
        const __amdgpu_buffer_rsrc_t csrd = make_srd(p.fold_c, p.N * 4);
        const __amdgpu_buffer_rsrc_t ssrd = make_srd(p.fold_stats, p.M * 8);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(csrd, (CE_LDS void*)(side + 1024), 16, (nbase + lane * 4) * 4, 0, 0, 0);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(ssrd, (CE_LDS void*)(side + 2048), 16, (mbase + lane * 2) * 8, 0, 0, 0);
    }
}

template <int ACT, int EPI, int JN>
__device__ __forceinline__ void w4_epilogue_bf16_n(const GemmParams& p, const f32x4 (&acc)[8][8], int mbase, int nbase,
                                                   int lane, const char* side) {
    const int fr = lane & 15, fq = lane >> 4;
    const int rows = max(0, min(p.M - mbase, 128));
    const __amdgpu_buffer_rsrc_t osrd =
        make_srd(static_cast<bf16_t*>(p.out) + (size_t)mbase * p.ldo, rows * (int)p.ldo * 2);
    const int ldo2 = (int)p.ldo * 2;
    int voff = (fr + (fq & 1) * 16) * ldo2 + (fq >> 1) * 16 + nbase * 2;
    // column operands of all JN 16-column blocks up front (one LDS latency, not one per block)
    const float4* sb = reinterpret_cast<const float4*>(side) + fq;            // bias[16j + 4fq ..]
    const float4* sc = reinterpret_cast<const float4*>(side + 1024) + fq;     // fold_c
    const float2* ss = reinterpret_cast<const float2*>(side + 2048) + fr;     // (mu, rstd) of row 16i + fr
    float4 bv[JN], cv[JN];
#pragma unroll
    for (int j = 0; j < JN; ++j) {
        bv[j] = sb[4 * j];
        if constexpr (EPI == EPI_LN_FOLD) cv[j] = sc[4 * j];
    }
    float2 st[8];
    if constexpr (EPI == EPI_LN_FOLD) {
#pragma unroll
        for (int i = 0; i < 8; ++i) st[i] = ss[16 * i];
    }
    // pre-activation copy (training forward, EPI_PLAIN only: the inference epilogues keep their code)
    constexpr bool MAYPRE = EPI == EPI_PLAIN && ACT != ACT_NONE;
    const bool pre = MAYPRE && p.pre_out != nullptr;            // wave-uniform
    __amdgpu_buffer_rsrc_t psrd = osrd;
    if constexpr (MAYPRE)
        if (pre) psrd = make_srd(p.pre_out + (size_t)mbase * p.ldo, rows * (int)p.ldo * 2);
#pragma unroll
    for (int ip = 0; ip < 4; ++ip) {
#pragma unroll
        for (int j = 0; j < JN; ++j) {
            uint2 h[2], hp[2];
#pragma unroll
            for (int r = 0; r < 2; ++r) {
                f32x4 v = acc[2 * ip + r][j];
                const float4 b = bv[j];
                if constexpr (EPI == EPI_LN_FOLD) {
                    const float4 c = cv[j];
                    const float2 t = st[2 * ip + r];
                    v[0] = fmaf(t.y, fmaf(-t.x, c.x, v[0]), b.x);
                    v[1] = fmaf(t.y, fmaf(-t.x, c.y, v[1]), b.y);
                    v[2] = fmaf(t.y, fmaf(-t.x, c.z, v[2]), b.z);
                    v[3] = fmaf(t.y, fmaf(-t.x, c.w, v[3]), b.w);
                } else {
                    v[0] += b.x; v[1] += b.y; v[2] += b.z; v[3] += b.w;
                }
                if constexpr (MAYPRE)
                    if (pre) hp[r] = make_uint2(pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3]));
                if constexpr (ACT == ACT_GELU) {
                    v = gelu_fast4(v);
                } else {
#pragma unroll
                    for (int e = 0; e < 4; ++e) v[e] = apply_act<ACT>(v[e]);
                }
                h[r] = make_uint2(pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3]));
            }
            const auto x = __builtin_amdgcn_permlane16_swap(h[0].x, h[1].x, false, false);
            const auto y = __builtin_amdgcn_permlane16_swap(h[0].y, h[1].y, false, false);
            const u32x4 d = {x[0], y[0], x[1], y[1]};
            __builtin_amdgcn_raw_buffer_store_b128(d, osrd, voff + j * 32, 0, CE_STORE_AUX);
            if constexpr (MAYPRE) {
                if (pre) {
                    const auto px = __builtin_amdgcn_permlane16_swap(hp[0].x, hp[1].x, false, false);
                    const auto py = __builtin_amdgcn_permlane16_swap(hp[0].y, hp[1].y, false, false);
                    const u32x4 dp = {px[0], py[0], px[1], py[1]};
                    __builtin_amdgcn_raw_buffer_store_b128(dp, psrd, voff + j * 32, 0, CE_STORE_AUX);
                }
            }
        }
        voff += 32 * ldo2;
    }
}

// Activation-backward epilogue (ACT_GELU_BWD / ACT_QGELU_BWD, launch_gemm_act_bwd): the dX GEMM of
// the MLP's c_proj in the text-tower backward (transformer.py:235-239 under autograd).  out =
// bf16(bf16(acc) * act'(pre)) with pre the forward's pre-activation copy, and the column sums of
// those bf16 outputs over the wave's 128 rows into bwd_part[mbase / 128][n]: the values, roundings
// and bias-gradient inputs of launch_gemm + launch_act_bwd_colsum (train.hip), without writing and
// re-reading the [M][F] product.  pre is read 16 B per lane at the output's own addresses (the
// store layout below) and put back in fragment order by the inverse v_permlane16_swap; one 128-row
// block of reads is in flight ahead of the one being consumed.  Column sums: each lane adds its 8
// rows, then a reduce-scatter over the 16 lanes of a row group (DPP row_mirror, row_half_mirror,
// quad_perm ^2, ^1) leaves lane fr with the finished sums of its 2 columns.  Whole 128-column quadrants.
template <int CTRL>
__device__ __forceinline__ float dpp_mov_f(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
// one reduce-scatter step over N value pairs: lanes with `hi` keep c[N..2N) (moved to c[0..N)), the
// others c[0..N); each adds its partner's copy of the kept half
template <int N, int CTRL>
__device__ __forceinline__ void rs_step(float (&c)[32], bool hi) {
#pragma unroll
    for (int k = 0; k < N; ++k) {
        const float send = hi ? c[k] : c[k + N];
        const float keep = hi ? c[k + N] : c[k];
        c[k] = keep + dpp_mov_f<CTRL>(send);
    }
}
template <int ACT>
__device__ __forceinline__ void w4_epilogue_act_bwd(const GemmParams& p, const f32x4 (&acc)[8][8], int mbase,
                                                    int nbase, int lane) {
    if (mbase >= p.M) return;                                   // wave-uniform
    const int fr = lane & 15, fq = lane >> 4;
    const int rows = min(p.M - mbase, 128);
    const __amdgpu_buffer_rsrc_t osrd =
        make_srd(static_cast<bf16_t*>(p.out) + (size_t)mbase * p.ldo, rows * (int)p.ldo * 2);
    const __amdgpu_buffer_rsrc_t psrd = make_srd(p.bwd_pre + (size_t)mbase * p.ldo, rows * (int)p.ldo * 2);
    const int ldo2 = (int)p.ldo * 2;
    const int voff0 = (fr + (fq & 1) * 16) * ldo2 + (fq >> 1) * 16 + nbase * 2;
    float cs[32];
#pragma unroll
    for (int k = 0; k < 32; ++k) cs[k] = 0.f;
    u32x4 pv[2][8];
#pragma unroll
    for (int j = 0; j < 8; ++j) pv[0][j] = __builtin_amdgcn_raw_buffer_load_b128(psrd, voff0 + j * 32, 0, 0);
    auto grad = [](float x) { return ACT == ACT_QGELU_BWD ? qgelu_grad(x) : gelu_grad(x); };
#pragma unroll
    for (int ip = 0; ip < 4; ++ip) {
        if (ip + 1 < 4) {
#pragma unroll
            for (int j = 0; j < 8; ++j)
                pv[(ip + 1) & 1][j] = __builtin_amdgcn_raw_buffer_load_b128(psrd, voff0 + (ip + 1) * 32 * ldo2 + j * 32, 0, 0);
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const u32x4 d = pv[ip & 1][j];
            // (h0, h1) of the store below, inverted: pre of rows 16r + fr, columns 16j + 4fq + 0..3
            const auto px = __builtin_amdgcn_permlane16_swap(d[0], d[2], false, false);
            const auto py = __builtin_amdgcn_permlane16_swap(d[1], d[3], false, false);
            uint2 h[2];
#pragma unroll
            for (int r = 0; r < 2; ++r) {
                const f32x4 v = acc[2 * ip + r][j];
                const uint32_t d01 = pack_bf2(v[0], v[1]), d23 = pack_bf2(v[2], v[3]);   // dh as a bf16 GEMM output
                const uint32_t p01 = px[r], p23 = py[r];
                const float o0 = __uint_as_float(d01 << 16) * grad(__uint_as_float(p01 << 16));
                const float o1 = __uint_as_float(d01 & 0xffff0000u) * grad(__uint_as_float(p01 & 0xffff0000u));
                const float o2 = __uint_as_float(d23 << 16) * grad(__uint_as_float(p23 << 16));
                const float o3 = __uint_as_float(d23 & 0xffff0000u) * grad(__uint_as_float(p23 & 0xffff0000u));
                h[r] = make_uint2(pack_bf2(o0, o1), pack_bf2(o2, o3));
                cs[4 * j + 0] += __uint_as_float(h[r].x << 16);
                cs[4 * j + 1] += __uint_as_float(h[r].x & 0xffff0000u);
                cs[4 * j + 2] += __uint_as_float(h[r].y << 16);
                cs[4 * j + 3] += __uint_as_float(h[r].y & 0xffff0000u);
            }
            const auto x = __builtin_amdgcn_permlane16_swap(h[0].x, h[1].x, false, false);
            const auto y = __builtin_amdgcn_permlane16_swap(h[0].y, h[1].y, false, false);
            const u32x4 o = {x[0], y[0], x[1], y[1]};
            __builtin_amdgcn_raw_buffer_store_b128(o, osrd, voff0 + ip * 32 * ldo2 + j * 32, 0, CE_STORE_AUX);
        }
    }
    // column c = 16j + 4fq + e of value k = 4j + e; after the four steps lane fr holds k = 2fr, 2fr + 1
    rs_step<16, 0x140>(cs, (fr & 8) != 0);     // row_mirror: fr <-> 15 - fr
    rs_step<8, 0x141>(cs, (fr & 4) != 0);      // row_half_mirror: fr <-> 7 - fr (within each 8)
    rs_step<4, 0x4E>(cs, (fr & 2) != 0);       // quad_perm [2,3,0,1]
    rs_step<2, 0xB1>(cs, (fr & 1) != 0);       // quad_perm [1,0,3,2]
    const int col = nbase + 16 * (fr >> 1) + 4 * fq + 2 * (fr & 1);
    *reinterpret_cast<float2*>(p.bwd_part + (size_t)(mbase >> 7) * p.N + col) = make_float2(cs[0], cs[1]);
}

template <int ACT, int EPI>
__device__ __forceinline__ void w4_epilogue_bf16(const GemmParams& p, const f32x4 (&acc)[8][8], int mbase, int nbase,
                                                 int lane, const char* side) {
    if (nbase >= p.N) return;                                   // wave-uniform
    if constexpr (ACT == ACT_GELU_BWD || ACT == ACT_QGELU_BWD) {
        w4_epilogue_act_bwd<ACT>(p, acc, mbase, nbase, lane);        // (launch_gemm_act_bwd: N % 128 == 0)
    } else {
        if (p.N - nbase >= 128) w4_epilogue_bf16_n<ACT, EPI, 8>(p, acc, mbase, nbase, lane, side);
        else w4_epilogue_bf16_n<ACT, EPI, 4>(p, acc, mbase, nbase, lane, side);   // N % 128 == 64
    }
}

// Four-wave epilogue of the residual GEMMs with LN statistics (out-proj / c_proj of the folded image
// tower, EPI_LN_STATS): out f32 = acc + bias + resid, xb = bf16(out), per-64-column-slab (mean, M2)
// of every row.  The residual rows are prefetched RD - 1 fragment rows ahead through a buffer
// descriptor clipped at row M (rows past M read zeros; their outputs are dropped the same way), so
// each residual wait is for loads issued before the previous rows' stores.
template <int JN, int RD, int NJA>
__device__ __forceinline__ void epi_stats_rows(const GemmParams& p, const f32x4 (&acc)[8][NJA], int mbase, int nbase,
                                               int lane, const float4 (&bv)[JN]) {
    constexpr int NS = JN / 4;                                  // 64-column slabs of the quadrant
    const int fr = lane & 15, fq = lane >> 4;
    const int rows = max(0, min(p.M - mbase, 128));
    const int ldo = (int)p.ldo, ldr = (int)p.ldr;
    // one descriptor per buffer over the quadrant's rows [mbase, M); lane offsets advance by one
    // fragment row (16 rows) per step, the 16-column step is the immediate
    const __amdgpu_buffer_rsrc_t os = make_srd(static_cast<float*>(p.out) + (size_t)mbase * ldo, rows * ldo * 4);
    const __amdgpu_buffer_rsrc_t xs = make_srd(p.xb + (size_t)mbase * ldo, rows * ldo * 2);
    const __amdgpu_buffer_rsrc_t rs = make_srd(p.resid + (size_t)mbase * ldr, rows * ldr * 4);
    int ooff = (fr * ldo + nbase + fq * 4) * 4;                                    // + j*64
    int roff = (fr * ldr + nbase + fq * 4) * 4;
    int xoff = ((fr + (fq & 1) * 16) * ldo + nbase + (fq >> 1) * 8) * 2;           // row pair, + j*32
    const int ostep = 16 * ldo * 4, rstep = 16 * ldr * 4, xstep = 32 * ldo * 2;
    f32x4 rv[RD][JN];
    auto load_r = [&](f32x4 (&r)[JN]) {     // the next fragment row's residual
#pragma unroll
        for (int j = 0; j < JN; ++j)
            r[j] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, roff + j * 64, 0, 0));
        roff += rstep;
    };
#pragma unroll
    for (int i = 0; i < RD - 1; ++i) load_r(rv[i]);
    uint2 pxb[JN];
    float2 sta[NS], stb[NS];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        if (i + RD - 1 < 8) load_r(rv[(i + RD - 1) % RD]);
        float lmean[NS], lm2[NS];
#pragma unroll
        for (int j = 0; j < JN; ++j) {
            f32x4 v = acc[i][j];
            const f32x4 r = rv[i % RD][j];
            v[0] += bv[j].x + r[0]; v[1] += bv[j].y + r[1]; v[2] += bv[j].z + r[2]; v[3] += bv[j].w + r[3];
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), os, ooff + j * 64, 0, CE_STORE_AUX);
            // Chan's pairwise update: the 4 values of block j join the lane's 4jj earlier ones
            const float m4 = ((v[0] + v[1]) + (v[2] + v[3])) * 0.25f;
            const float d0 = v[0] - m4, d1 = v[1] - m4, d2 = v[2] - m4, d3 = v[3] - m4;
            const float q4 = fmaf(d0, d0, fmaf(d1, d1, fmaf(d2, d2, d3 * d3)));
            const int sl = j >> 2, jj = j & 3;
            if (jj == 0) {
                lmean[sl] = m4;
                lm2[sl] = q4;
            } else {
                const float dl = m4 - lmean[sl];
                lmean[sl] = fmaf(dl, 1.0f / (jj + 1), lmean[sl]);
                lm2[sl] += fmaf(dl * dl, 4.0f * jj / (jj + 1), q4);
            }
            const uint2 o = make_uint2(pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3]));
            if ((i & 1) == 0) {
                pxb[j] = o;
            } else {
                const auto x = __builtin_amdgcn_permlane16_swap(pxb[j].x, o.x, false, false);
                const auto y = __builtin_amdgcn_permlane16_swap(pxb[j].y, o.y, false, false);
                const u32x4 d = {x[0], y[0], x[1], y[1]};
                __builtin_amdgcn_raw_buffer_store_b128(d, xs, xoff + j * 32, 0, CE_STORE_AUX);
            }
        }
        ooff += ostep;
        if (i & 1) xoff += xstep;
        // (mean, M2) of this row's 64-column slabs: 4 lanes (fq) of 16 values each, Chan's formula
        // for equal counts; lane group fq keeps fragment rows fq and fq + 4
#pragma unroll
        for (int sl = 0; sl < NS; ++sl) {
            float sm = lmean[sl];
            sm += __shfl_xor(sm, 16, 64);
            sm += __shfl_xor(sm, 32, 64);
            const float mean = sm * 0.25f;
            const float dl = lmean[sl] - mean;
            float q = fmaf(dl * dl, 16.0f, lm2[sl]);
            q += __shfl_xor(q, 16, 64);
            q += __shfl_xor(q, 32, 64);
            if (fq == (i & 3)) {
                if (i < 4) sta[sl] = make_float2(mean, q);
                else stb[sl] = make_float2(mean, q);
            }
        }
    }
    const int ma = mbase + fq * 16 + fr, mb = ma + 64;
    const size_t ns = p.N / 64;
#pragma unroll
    for (int sl = 0; sl < NS; ++sl) {
        if (ma < p.M) p.stats_part[(size_t)ma * ns + nbase / 64 + sl] = sta[sl];
        if (mb < p.M) p.stats_part[(size_t)mb * ns + nbase / 64 + sl] = stb[sl];
    }
}

template <int JN, int RD>
__device__ __forceinline__ void w4_epilogue_stats_n(const GemmParams& p, const f32x4 (&acc)[8][8], int mbase, int nbase,
                                                    int lane, const char* side) {
    const float4* sb = reinterpret_cast<const float4*>(side) + (lane >> 4);
    float4 bv[JN];
#pragma unroll
    for (int j = 0; j < JN; ++j) bv[j] = sb[4 * j];
    epi_stats_rows<JN, RD>(p, acc, mbase, nbase, lane, bv);
}

__device__ __forceinline__ void w4_epilogue_stats(const GemmParams& p, const f32x4 (&acc)[8][8], int mbase, int nbase,
                                                  int lane, const char* side) {
    if (nbase >= p.N) return;                                   // wave-uniform
    if (p.N - nbase >= 128) w4_epilogue_stats_n<8, 2>(p, acc, mbase, nbase, lane, side);
    else w4_epilogue_stats_n<4, 2>(p, acc, mbase, nbase, lane, side);   // N % 128 == 64
}

// Diagnostic timeline (ce_set_gemm_trace): wave 0 of each workgroup records s_memrealtime (100 MHz,
// chip-wide) at start, after the K-loop and after its epilogue, plus the hardware id word, into
// its own buffer (nothing else reads it).  Null in normal runs.
__device__ __forceinline__ void trace_stamp(const GemmParams& p, int slot_idx, int rec = -1) {
    if (rec < 0) rec = blockIdx.x;
    if (p.trace && threadIdx.x == 0 && rec < p.trace_n) {
        unsigned long long* r = p.trace + (size_t)rec * 4;
        r[slot_idx] = __builtin_amdgcn_s_memrealtime();
        if (slot_idx == 0) {
            unsigned hw;
            asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
            unsigned xcc;
            asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
            r[3] = ((unsigned long long)xcc << 32) | hw;
        }
    }
}

__device__ __forceinline__ void stagger_sleep(const GemmParams& p) {
    const int b = blockIdx.x;
    if (p.stagger > 0 && b >= p.stagger_lo && b < p.stagger_hi && (p.stagger_bit < 0 || ((b >> p.stagger_bit) & 1)))
        for (int i = 0; i < p.stagger; ++i) __builtin_amdgcn_s_sleep(127);
}

// Bijective XCD-aware remap: blocks b and b+8 share an XCD; give each XCD a contiguous range
// of tile ids so the tiles that share A / W panels run on one L2.
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
    const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

// Tile id -> (tm, tn).  gm <= 1: row-major (all N tiles of one M panel, then the next panel).
// gm > 1: groups of gm M panels walked column-major, so the ~32 workgroups an XCD runs at once
// share gm A panels and 32/gm W panels in its L2 instead of 2 A panels and every W panel.
__device__ __forceinline__ void tile_of(int wgid, int tiles_m, int tiles_n, int gm, int& tm, int& tn) {
    if (gm <= 1) {
        tm = wgid / tiles_n;
        tn = wgid - tm * tiles_n;
        return;
    }
    const int per = gm * tiles_n;
    const int g = wgid / per;
    const int first = g * gm;
    const int gsz = min(tiles_m - first, gm);
    const int l = wgid - g * per;
    tn = l / gsz;
    tm = first + (l - tn * gsz);
}

// SCHED 1: 4 phases per K-tile; the K-tile is split in half-tiles {A rows of quadrant-row mh,
//          W rows of quadrant-col nh}, each double-buffered; phase p computes one 64x32
//          quadrant of every wave's 128x64 output (16 MFMAs) and issues the LDS-DMA of one
//          half-tile of K-tile t+1, so every load has ~3 phases to land; one barrier per phase.
template <int ACT, bool HAS_RESID, bool OUT_BF16, int RING = CE_RESID_RING, int EPI = EPI_PLAIN>
__global__ __launch_bounds__(NTHREADS, 2) void gemm_bf16_nt(GemmParams p) {
    __shared__ __attribute__((aligned(16))) char smem[2 * STAGE_BYTES];
    trace_stamp(p, 0);
    stagger_sleep(p);

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave >> 2;   // 0..1 : 128-row slab
    const int wn = wave & 3;    // 0..3 : 64-col slab

    // ---- XCD-aware bijective tile remap -------------------------------------------------
    const int tiles_m = (p.M + BM - 1) / BM;
    const int tiles_n = (p.N + BN - 1) / BN;
    const int nwg = tiles_m * tiles_n;
    int bid = blockIdx.x;
    const int nk = p.K / BK;
    // split-K tail: blocks past t_main (dispatched last, so they fill the final, otherwise
    // mostly idle round of the grid) each take one K-chunk of one of the last `tail` tiles
    const int t_main = nwg - p.tail;
    int wgid, kt0 = 0, kt1 = nk, slab = -1;
    if (p.tail_only) bid += t_main;      // only the split-K chunks (SCHED 11's tail)
    if (bid < t_main) {
        // (packed rows: the live tiles are the first tile indices; blockIdx order spreads them over
        // the XCDs round-robin instead of the first XCDs' contiguous ranges)
        wgid = p.m_dev ? bid : xcd_remap(bid, t_main);
    } else {
        slab = bid - t_main;
        const int c = slab % p.split;
        wgid = t_main + slab / p.split;
        kt0 = c * nk / p.split;
        kt1 = (c + 1) * nk / p.split;
    }
    int tm, tn;
    tile_of(wgid, tiles_m, tiles_n, p.gm, tm, tn);
    const int m0 = tm * BM, n0 = tn * BN;
    // packed rows: clip at the live count, a tile wholly past it exits (no split-K with m_dev)
    if (p.m_dev) {
        p.M = min(p.M, __builtin_amdgcn_readfirstlane(*p.m_dev));
        if (m0 >= p.M) return;
    }

    const int fr = lane & 15;
    const int fq = lane >> 4;
    const int frag_off0 = fr * 128 + ((((0 * 4) + fq) ^ (fr >> 1)) << 4);
    const int frag_off1 = fr * 128 + ((((1 * 4) + fq) ^ (fr >> 1)) << 4);

    FoldOps<4> fold;
    constexpr bool PRE = EPI == EPI_LN_FOLD && CE_FOLD_PREFETCH;
    if constexpr (PRE) {
        if (slab < 0 && n0 + wn * 64 < p.N) fold.load(p, m0 + wm * 128, n0 + wn * 64, lane);
    }

    f32x4 acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    {
        // ---- half-tile staging ---------------------------------------------------------------
        // LDS per buffer: A image rows 0..255 (32 KB) then W image rows 0..255 (32 KB), 128-B rows,
        // chunk c of row r at c ^ ((r>>1)&7).  Half-tile HA[mh] = A rows {mh*64 + j*128 + 0..63},
        // HB[nh] = W rows {g*64 + nh*32 + 0..31 : g = 0..3}; each is 128 rows = 2 glds per thread.
        const int rr = tid >> 3;                       // 0..63 row within a 64-row pass
        const int ca = (tid & 7) ^ ((rr >> 1) & 7);    // source chunk (rows here are ==rr mod 16)
        // A rows for (mh, j): mh*64 + j*128 + rr ; W rows for (nh, j): (j*2 + (rr>>5))*64 + nh*32 + (rr&31)
        const bf16_t* a_src[2][2];
        const bf16_t* w_src[2][2];
        int a_lds[2][2], w_lds[2][2];
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int arow = h * 64 + j * 128 + rr;
                const int wrow = (j * 2 + (rr >> 5)) * 64 + h * 32 + (rr & 31);
                a_src[h][j] = p.A + (size_t)min(m0 + arow, p.M - 1) * p.lda + ca * 8;
                w_src[h][j] = p.W + (size_t)min(n0 + wrow, p.N - 1) * p.ldw + ((tid & 7) ^ ((wrow >> 1) & 7)) * 8;
                // wave-uniform LDS destination of this wave's 8 rows
                const int arow_w = h * 64 + j * 128 + wave * 8;
                const int wrow_w = (j * 2 + ((wave * 8) >> 5)) * 64 + h * 32 + ((wave * 8) & 31);
                a_lds[h][j] = arow_w * 128;
                w_lds[h][j] = TILE_BYTES + wrow_w * 128;
            }
        auto stageA = [&](int kt, int buf, int h) {
            char* base = smem + buf * STAGE_BYTES;
            const int koff = kt * BK;
            glds16(a_src[h][0] + koff, base + a_lds[h][0]);
            glds16(a_src[h][1] + koff, base + a_lds[h][1]);
        };
        auto stageB = [&](int kt, int buf, int h) {
            char* base = smem + buf * STAGE_BYTES;
            const int koff = kt * BK;
            glds16(w_src[h][0] + koff, base + w_lds[h][0]);
            glds16(w_src[h][1] + koff, base + w_lds[h][1]);
        };
        const int a_off = wm * 128 * 128;
        const int w_off = TILE_BYTES + wn * 64 * 128;

        // prologue: K-tile kt0, issue order A0, B0, B1, A1 (same as the steady-state phases)
        stageA(kt0, 0, 0);
        stageB(kt0, 0, 0);
        stageB(kt0, 0, 1);
        stageA(kt0, 0, 1);
        if (kt1 - kt0 > 1) wait_vm(4); else wait_vm(0);
        barrier();

        bf16x8 af[4][2], bfr[2][2];
        auto readA = [&](const char* sb, int mh) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                af[i][0] = *reinterpret_cast<const bf16x8*>(sb + a_off + (mh * 4 + i) * 16 * 128 + frag_off0);
                af[i][1] = *reinterpret_cast<const bf16x8*>(sb + a_off + (mh * 4 + i) * 16 * 128 + frag_off1);
            }
        };
        auto readB = [&](const char* sb, int nh) {
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                bfr[j][0] = *reinterpret_cast<const bf16x8*>(sb + w_off + (nh * 2 + j) * 16 * 128 + frag_off0);
                bfr[j][1] = *reinterpret_cast<const bf16x8*>(sb + w_off + (nh * 2 + j) * 16 * 128 + frag_off1);
            }
        };

        // MFMAs of one quadrant, optionally split in two halves with `mid` issued in between
        auto mfma_half = [&](int mh, int nh, int ks) {
            __builtin_amdgcn_s_setprio(1);
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j)
                    acc[mh * 4 + i][nh * 2 + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                        bfr[j][ks], af[i][ks], acc[mh * 4 + i][nh * 2 + j], 0, 0, 0);
            __builtin_amdgcn_s_setprio(0);
        };
        auto phase = [&](int mh, int nh, auto&& loads) {
            loads();
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            mfma_half(mh, nh, 0);
            mfma_half(mh, nh, 1);
        };
        for (int kt = kt0; kt < kt1; ++kt) {
            const int cur = (kt - kt0) & 1, nxt = cur ^ 1;
            const bool more = kt + 1 < kt1;
            const char* sb = smem + cur * STAGE_BYTES;
            // phase 1: quadrant (0,0); prefetch HA0(t+1)
            readA(sb, 0);
            readB(sb, 0);
            phase(0, 0, [&] { if (more) stageA(kt + 1, nxt, 0); });
            wait_vm(more ? 4 : 0);        // HB1(t) landed
            barrier();
            // phase 2: quadrant (0,1); prefetch HB0(t+1)
            readB(sb, 1);
            phase(0, 1, [&] { if (more) stageB(kt + 1, nxt, 0); });
            wait_vm(more ? 4 : 0);        // HA1(t) landed
            barrier();
            // phase 3: quadrant (1,1); prefetch HB1(t+1)
            readA(sb, 1);
            phase(1, 1, [&] { if (more) stageB(kt + 1, nxt, 1); });
            barrier();
            // phase 4: quadrant (1,0); prefetch HA1(t+1)
            readB(sb, 0);
            phase(1, 0, [&] { if (more) stageA(kt + 1, nxt, 1); });
            wait_vm(more ? 4 : 0);        // HA0(t+1), HB0(t+1) landed
            barrier();
        }
    }

    if (slab >= 0) {
        // split-K tail chunk: raw f32 partial tile, row-major [256][256], slab `slab` of p.part
        float* dst = p.part + (size_t)slab * (BM * BN) + (size_t)(wm * 128 + fr) * BN + wn * 64 + fq * 4;
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j)
                *reinterpret_cast<f32x4*>(dst + (size_t)i * 16 * BN + j * 16) = acc[i][j];
        return;
    }
    trace_stamp(p, 1);
    gemm_epilogue<ACT, HAS_RESID, OUT_BF16, 4, RING, EPI>(p, acc, m0 + wm * 128, n0 + wn * 64, lane,
                                                           PRE ? &fold : nullptr);
    trace_stamp(p, 2);
}

// Split-K tail fixup: sums the `split` partial slabs of each tail tile in fixed order (deterministic)
// and applies the epilogue (bias, activation, residual, f32/bf16 store).  One thread per 4 columns
// of one row; 64 blocks of 256 threads per tile.
template <int ACT, bool HAS_RESID, bool OUT_BF16, int EPI = EPI_PLAIN>
__global__ __launch_bounds__(256) void gemm_splitk_fixup(GemmParams p) {
    const int tiles_m = (p.M + BM - 1) / BM, tiles_n = (p.N + BN - 1) / BN;
    const int t_main = tiles_m * tiles_n - p.tail;
    const int r = blockIdx.x >> 6;
    const int e = ((blockIdx.x & 63) << 8) + threadIdx.x;     // float4 index inside the 256x256 tile
    const int row = e >> 6, c4 = (e & 63) * 4;
    int tm, tn;
    tile_of(t_main + r, tiles_m, tiles_n, p.gm, tm, tn);
    const int m = tm * BM + row, n = tn * BN + c4;
    if (m >= p.M || n >= p.N) return;
    const float* src = p.part + (size_t)r * p.split * (BM * BN) + (size_t)row * BN + c4;
    f32x4 v = *reinterpret_cast<const f32x4*>(src);
    for (int c = 1; c < p.split; ++c) v += *reinterpret_cast<const f32x4*>(src + (size_t)c * (BM * BN));
    const float4 b = p.bias ? *reinterpret_cast<const float4*>(p.bias + n) : make_float4(0.f, 0.f, 0.f, 0.f);
    if constexpr (EPI == EPI_LN_FOLD) {
        const float4 c = *reinterpret_cast<const float4*>(p.fold_c + n);
        const float2 st = p.fold_stats[m];
        v[0] = fmaf(st.y, fmaf(-st.x, c.x, v[0]), b.x);
        v[1] = fmaf(st.y, fmaf(-st.x, c.y, v[1]), b.y);
        v[2] = fmaf(st.y, fmaf(-st.x, c.z, v[2]), b.z);
        v[3] = fmaf(st.y, fmaf(-st.x, c.w, v[3]), b.w);
    } else {
        v[0] += b.x; v[1] += b.y; v[2] += b.z; v[3] += b.w;
    }
    if constexpr (ACT == ACT_GELU) {
        const f32x2 lo = gelu_pair(f32x2{v[0], v[1]}), hi = gelu_pair(f32x2{v[2], v[3]});
        v[0] = lo.x; v[1] = lo.y; v[2] = hi.x; v[3] = hi.y;
    } else {
        v[0] = apply_act<ACT>(v[0]); v[1] = apply_act<ACT>(v[1]);
        v[2] = apply_act<ACT>(v[2]); v[3] = apply_act<ACT>(v[3]);
    }
    constexpr bool STATS = EPI == EPI_LN_STATS || EPI == EPI_LN_STATS_HL;
    constexpr bool HL_IN = EPI == EPI_LN_STATS_HL || EPI == EPI_HL_F32;
    if constexpr (HAS_RESID) {
        const size_t ro = (size_t)map_row(m, p.grp, p.r_gs, p.r_go) * p.ldr + n;
        float4 rr;
        if constexpr (HL_IN) {
            const uint2 hi = *reinterpret_cast<const uint2*>(p.rhl + ro);
            const uint2 lo = *reinterpret_cast<const uint2*>(p.rhl + p.hl_plane + ro);
            const float2 a = join_hl(hi.x, lo.x), c = join_hl(hi.y, lo.y);
            rr = make_float4(a.x, a.y, c.x, c.y);
        } else {
            rr = *reinterpret_cast<const float4*>(p.resid + ro);
        }
        v[0] += rr.x; v[1] += rr.y; v[2] += rr.z; v[3] += rr.w;
    }
    const size_t o = (size_t)map_row(m, p.grp, p.o_gs, p.o_go) * p.ldo + n;
    if constexpr (EPI == EPI_LN_STATS_HL) {
        uint2 hi, lo;
        split_hl(v[0], v[1], hi.x, lo.x);
        split_hl(v[2], v[3], hi.y, lo.y);
        *reinterpret_cast<uint2*>(p.xb + o) = hi;
        *reinterpret_cast<uint2*>(p.xb + p.hl_plane + o) = lo;
    } else if constexpr (OUT_BF16) {
        *reinterpret_cast<uint2*>(static_cast<bf16_t*>(p.out) + o) = make_uint2(pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3]));
    } else {
        *reinterpret_cast<float4*>(static_cast<float*>(p.out) + o) = make_float4(v[0], v[1], v[2], v[3]);
    }
    if constexpr (STATS) {
        // a row's 256 columns are one wave (64 threads x 4); a 64-column slab = 16 consecutive lanes
        if constexpr (EPI == EPI_LN_STATS)
            *reinterpret_cast<uint2*>(p.xb + o) = make_uint2(pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3]));
        float sm = (v[0] + v[1]) + (v[2] + v[3]);
#pragma unroll
        for (int o2 = 1; o2 < 16; o2 <<= 1) sm += __shfl_xor(sm, o2, 64);
        const float mean = sm * (1.0f / 64);
        float q = (v[0] - mean) * (v[0] - mean) + (v[1] - mean) * (v[1] - mean) + (v[2] - mean) * (v[2] - mean) +
                  (v[3] - mean) * (v[3] - mean);
#pragma unroll
        for (int o2 = 1; o2 < 16; o2 <<= 1) q += __shfl_xor(q, o2, 64);
        if ((c4 & 63) == 0) p.stats_part[(size_t)m * (p.N / 64) + n / 64] = make_float2(mean, q);
    }
}

// ------------------------------------------------------------------------------------------
// SCHED 11 (four-wave persistent): 4 waves (one per SIMD), 128x128 per wave (acc[8][8] pinned in
// AGPRs), BK = 64, two 64-KB stage buffers (LDS image as SCHED 1: 128-B rows, chunk c of row r at
// c ^ ((r>>1)&7)), run as one continuous K-tile stream over the tiles a workgroup owns (grid = one
// workgroup per CU; tile r*grid + xcd_remap(b) in round r).  The DMA two K-tiles ahead runs into
// the next tile's first K-tiles, so the next tile's operands are in flight while this tile's
// epilogue runs and there is no per-tile prologue.  Epilogue for one wave per SIMD with its
// operands in an LDS side area (w4_epilogue_bf16 / _stats / _act_bwd); a K-tile's 16 operand DMAs
// spread over B2 (10, one per 6 MFMAs) and B3 (6).  (Measured and removed in round 6: whole-tile
// and BK = 32 rings, non-persistent and early-DMA schedules, the 12+4 / 8+8 / even-gap DMA splits,
// the register epilogue)
template <int ACT, bool HAS_RESID, bool OUT_BF16, int EPI = EPI_PLAIN>
__global__ __launch_bounds__(256, 1) void gemm_bf16_w4pp(GemmParams p) {
    // the epilogues of w4_ok (host side): bf16 without residual, the f32 LN-statistics residual, plain f32
    constexpr bool EPI_F32 = !OUT_BF16 && !HAS_RESID && EPI == EPI_PLAIN && ACT == ACT_NONE;
    static_assert((OUT_BF16 && !HAS_RESID && EPI != EPI_LN_STATS) || (EPI == EPI_LN_STATS && HAS_RESID && !OUT_BF16) ||
                  EPI_F32, "four-wave epilogues: bf16 without residual, the f32 LN-statistics residual, plain f32");
    // DMAs of a K-tile issued in B2 (the rest in B3); the B2 wait leaves exactly these in flight
    constexpr int DMA_B2 = 10;
    constexpr int P2 = 64 / DMA_B2;                          // MFMAs per DMA in B2
    constexpr int P3 = 32 / (16 - DMA_B2);                   // and in B3
    __shared__ __attribute__((aligned(16))) char smem[2 * STAGE_BYTES + 4 * W4_SIDE_BYTES];
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    char* const side = smem + 2 * STAGE_BYTES + wave * W4_SIDE_BYTES;
    const int wm = wave >> 1, wn = wave & 1;
    const int tiles_m = (p.M + BM - 1) / BM;
    const int tiles_n = (p.N + BN - 1) / BN;
    const int nwg = tiles_m * tiles_n;
    const int grid = gridDim.x;
    // (packed rows: blockIdx order, so the live tiles, the first indices, spread over all XCDs)
    const int slot = p.m_dev ? (int)blockIdx.x : xcd_remap(blockIdx.x, grid);
    const int nk = p.K / BK;
    // whole rounds only when the host planned a split-K tail (its p.tail tiles run as K-chunks on
    // the 4-phase kernel in tail-only mode, then gemm_splitk_fixup)
    const int t_main = nwg - p.tail;
    int my_tiles = slot < t_main ? (t_main - 1 - slot) / grid + 1 : 0;
    // packed rows (one tile per workgroup, forced by the host): clip at the live count; a tile
    // wholly past it does nothing
    if (p.m_dev) {
        p.M = min(p.M, __builtin_amdgcn_readfirstlane(*p.m_dev));
        int tm, tn;
        tile_of(min(slot, nwg - 1), tiles_m, tiles_n, p.gm, tm, tn);
        if (tm * BM >= p.M) return;
    }
    const int nsteps = my_tiles * nk;
    const bool nowait = (p.variant & GEMM_VAR_W4PP_NOWAIT) != 0;
    // De-synchronised start (p.stagger, units of s_sleep 16 ~ 1k cycles): equal tiles keep every
    // CU in lock-step, so all epilogues would store at once and share the HBM write bandwidth
    // (a 128-KB bf16 tile stores at ~100 GB/s from one CU alone, ~27 GB/s when all 256 store).
    // Phase k in 1..7 of the CUs that own one tile fewer than the others starts k x stagger late,
    // which spreads the epilogues over the tile period without lengthening the launch.
    if (p.stagger > 0 && p.tail == 0 && nwg % grid != 0 && slot >= nwg % grid) {
        const int ph = 1 + slot % 7;
        for (int i = 0; i < ph * p.stagger; ++i) __builtin_amdgcn_s_sleep(16);
    }

    const int srow = wave * 8 + (lane >> 3);
    const int schunk = (lane & 7) ^ ((srow >> 1) & 7);
    const int voffA = srow * (int)p.lda * 2 + schunk * 16;
    const int voffW = srow * (int)p.ldw * 2 + schunk * 16;
    const int jstrA = 32 * (int)p.lda * 2, jstrW = 32 * (int)p.ldw * 2;
    // DMA stream state: K-tile `dk` of this workgroup's tile number `dt` (0-based), descriptors
    // for that tile; advanced once per K-tile
    int dt = 0, dk = 0;
    __amdgpu_buffer_rsrc_t srdA, srdW;
    auto set_srd = [&](int t) {
        int tm, tn;
        tile_of(min(slot + t * grid, nwg - 1), tiles_m, tiles_n, p.gm, tm, tn);
        const int mm = tm * BM, nn = tn * BN;
        srdA = make_srd(p.A + (size_t)mm * p.lda, max(0, min(p.M - mm, BM)) * (int)p.lda * 2);
        srdW = make_srd(p.W + (size_t)nn * p.ldw, max(0, min(p.N - nn, BN)) * (int)p.ldw * 2);
    };
    set_srd(0);
    auto dma = [&](int buf, int j, bool live) {
        const int kb = live ? dk * BK * 2 : 0x7ffff000;
        char* base = smem + buf * STAGE_BYTES;
        // the row-group offset is made opaque so hipcc forms each DMA's VGPR offset in place
        // (one v_add) instead of keeping 16 loop-invariant offsets live across the epilogue
        int jo = (j < 8 ? j : j - 8) * (j < 8 ? jstrA : jstrW);
        asm volatile("" : "+s"(jo));
        if (j < 8)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(srdA, (CE_LDS void*)(base + (j * 32 + wave * 8) * 128), 16,
                                                     voffA + jo, kb, 0, 0);
        else
            __builtin_amdgcn_raw_ptr_buffer_load_lds(srdW, (CE_LDS void*)(base + TILE_BYTES + ((j - 8) * 32 + wave * 8) * 128),
                                                     16, voffW + jo, kb, 0, 0);
    };
    auto advance = [&] {
        if (++dk == nk) {
            dk = 0;
            ++dt;
            set_srd(dt);
        }
    };

    const int fr = lane & 15, fq = lane >> 4;
    const int fo0 = fr * 128 + (((0 + fq) ^ (fr >> 1)) << 4);
    const int fo1 = fr * 128 + (((4 + fq) ^ (fr >> 1)) << 4);
    const int a_off = wm * 128 * 128;
    const int w_off = TILE_BYTES + wn * 128 * 128;

    f32x4 acc[8][8];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    bf16x8 a0[8], b0[8], a1[8], b1[8];

    // prologue: steps 0 and 1 in flight, set0 of step 0
#pragma unroll
    for (int j = 0; j < 16; ++j) dma(0, j, 0 < nsteps);
    advance();
#pragma unroll
    for (int j = 0; j < 16; ++j) dma(1, j, 1 < nsteps);
    advance();
    asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    barrier();
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        a0[q] = *reinterpret_cast<const bf16x8*>(smem + a_off + q * 16 * 128 + fo0);
        b0[q] = *reinterpret_cast<const bf16x8*>(smem + w_off + q * 16 * 128 + fo0);
    }

    // MFMAs as inline asm with the accumulator pinned in AGPRs ("+a"): with the builtin, hipcc
    // shuffles accumulators between AGPRs and VGPRs in this loop.  A volatile asm is also a
    // barrier for memory instructions in the machine scheduler, so the ds_reads and DMAs below
    // stay exactly where the source interleaves them; hipcc still inserts the lgkmcnt waits for
    // the fragments each MFMA reads.
#define CE_MFMA_AGPR(ACC, BV, AV) \
    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(ACC) : "v"(BV), "v"(AV))
    // (C = 0 form of the MFMA: a first K-tile that skips zeroing the accumulators; unused)
#define CE_MFMA_AGPR0(ACC, BV, AV) \
    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=a"(ACC) : "v"(BV), "v"(AV))
    // K-tile phases.  ZERO: first K-tile of a tile (C = 0 on each accumulator's first MFMA).
    // B3's PRE: read set0 of the next K-tile under its MFMAs; the last K-tile of a tile
    // does not (the next tile's set0 is read after the epilogue, so the epilogue has those 64
    // VGPRs), reading it after the epilogue instead (read_set0).
    auto B1 = [&](const char* sb, auto zero) __attribute__((always_inline)) {
#pragma unroll
        for (int s2 = 0; s2 < 32; ++s2) {
            const int i = s2 >> 3, j = s2 & 7;
            if constexpr (decltype(zero)::value) CE_MFMA_AGPR0(acc[i][j], b0[j], a0[i]);
            else CE_MFMA_AGPR(acc[i][j], b0[j], a0[i]);
            if (s2 & 1) {
                const int q = s2 >> 1;      // 0..15: b1[0..7], a1[0..7]
                if (q < 8) b1[q] = *reinterpret_cast<const bf16x8*>(sb + w_off + q * 16 * 128 + fo1);
                else a1[q - 8] = *reinterpret_cast<const bf16x8*>(sb + a_off + (q - 8) * 16 * 128 + fo1);
            }
        }
    };
    auto B2 = [&](int buf, bool live, auto zero) __attribute__((always_inline)) {
#pragma unroll
        for (int s2 = 0; s2 < 64; ++s2) {
            const int i = (s2 >> 3) & 3, j = s2 & 7;
            if (s2 < 32) {
                if constexpr (decltype(zero)::value) CE_MFMA_AGPR0(acc[4 + i][j], b0[j], a0[4 + i]);
                else CE_MFMA_AGPR(acc[4 + i][j], b0[j], a0[4 + i]);
            } else {
                CE_MFMA_AGPR(acc[i][j], b1[j], a1[i]);
            }
            if (s2 % P2 == P2 - 1 && s2 / P2 < DMA_B2) dma(buf, s2 / P2, live);
        }
    };
    auto B3 = [&](const char* so, auto pre, int buf, bool live) __attribute__((always_inline)) {
#pragma unroll
        for (int s2 = 0; s2 < 32; ++s2) {
            const int i = s2 >> 3, j = s2 & 7;
            CE_MFMA_AGPR(acc[4 + i][j], b1[j], a1[4 + i]);
            if (s2 % P3 == P3 - 1 && DMA_B2 + s2 / P3 < 16) dma(buf, DMA_B2 + s2 / P3, live);
            if constexpr (decltype(pre)::value) {
                if (s2 & 1) {
                    const int q = s2 >> 1;      // a0[0], b0[0..7], a0[1..7]
                    if (q == 0) a0[0] = *reinterpret_cast<const bf16x8*>(so + a_off + fo0);
                    else if (q < 9) b0[q - 1] = *reinterpret_cast<const bf16x8*>(so + w_off + (q - 1) * 16 * 128 + fo0);
                    else a0[q - 8] = *reinterpret_cast<const bf16x8*>(so + a_off + (q - 8) * 16 * 128 + fo0);
                }
            }
        }
    };
    auto read_set0 = [&](const char* so) __attribute__((always_inline)) {
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            b0[q] = *reinterpret_cast<const bf16x8*>(so + w_off + q * 16 * 128 + fo0);
            a0[q] = *reinterpret_cast<const bf16x8*>(so + a_off + q * 16 * 128 + fo0);
        }
    };
    using T_ = std::integral_constant<bool, true>;
    using F_ = std::integral_constant<bool, false>;
    int g = 0;
    for (int t = 0; t < my_tiles; ++t) {
        int tm, tn;
        tile_of(slot + t * grid, tiles_m, tiles_n, p.gm, tm, tn);
        trace_stamp(p, 0, t * grid + blockIdx.x);     // diagnostics: one record per tile
        // one K-tile: B1 | barrier | B2 + DMA(step g+2) | wait + barrier | B3
        auto ktile = [&](int kt, auto pre) __attribute__((always_inline)) {
            // epilogue operands of this tile into the side area; retired by this K-tile's B2 wait
            if (kt == nk - 1) w4_side_fill<EPI>(p, side, tm * BM + wm * 128, tn * BN + wn * 128, lane);
            const int buf = g & 1;
            const char* sb = smem + buf * STAGE_BYTES;
            const char* so = smem + (buf ^ 1) * STAGE_BYTES;
            // ---- B1: MFMA(set0, rows 0-3), set1 of this K-tile read under it (one per 2 MFMAs) ----
            B1(sb, F_{});
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            barrier();
            // ---- B2: MFMA(set0, rows 4-7), MFMA(set1, rows 0-3); 10 DMAs of step g+2 (one per 6) ----
            const bool live = g + 2 < nsteps;
            B2(buf, live, F_{});
            // K-tile g+1 landed.  Right after an epilogue (kt == 0 of a later tile) it already has:
            // the epilogue began with vmcnt(0) and B1 ended with a barrier.  Waiting here would also
            // drain every store of that epilogue (vmcnt retires loads, DMAs and stores in issue
            // order), exposing their write latency; skipped, they drain under this tile's MFMAs.
            if (!nowait || kt != 0 || t == 0) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(DMA_B2) : "memory");
            barrier();
            // ---- B3: MFMA(set1, rows 4-7); set0 of the next step read under it, and the rest of
            // step g+2's DMAs (buf's last reader was B1, before the first barrier) ----
            B3(so, pre, buf, live);
            advance();
            ++g;
        };
        // the last K-tile does not read the next tile's set0 (read after the epilogue, which then
        // has those 64 VGPRs)
        for (int kt = 0; kt < nk - 1; ++kt) ktile(kt, T_{});
        ktile(nk - 1, F_{});
        trace_stamp(p, 1, t * grid + blockIdx.x);
        // the next tile's K-tile 1 (DMA issued in this tile's last B2) retires before any epilogue
        // load or store is issued (see the B2 wait above)
        if (nowait) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if constexpr (EPI == EPI_LN_STATS) {
            w4_epilogue_stats(p, acc, tm * BM + wm * 128, tn * BN + wn * 128, lane, side);
        } else if constexpr (OUT_BF16) {
            w4_epilogue_bf16<ACT, EPI>(p, acc, tm * BM + wm * 128, tn * BN + wn * 128, lane, side);
        } else {
            // plain f32 output: the register epilogue as two 64-column halves (NJ = 4 path)
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                f32x4 q[8][4];
#pragma unroll
                for (int i = 0; i < 8; ++i)
#pragma unroll
                    for (int j = 0; j < 4; ++j) q[i][j] = acc[i][h * 4 + j];
                gemm_epilogue<ACT, HAS_RESID, OUT_BF16, 4, CE_RESID_RING, EPI>(p, q, tm * BM + wm * 128,
                                                                            tn * BN + wn * 128 + h * 64, lane);
            }
        }
        trace_stamp(p, 2, t * grid + blockIdx.x);
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        // set0 of the next tile's first K-tile (step g; its DMA was retired before the epilogue
        // and published by the last B2 barrier; its buffer is not refilled before that K-tile's B2)
        read_set0(smem + (g & 1) * STAGE_BYTES);
    }
#undef CE_MFMA_AGPR0
#undef CE_MFMA_AGPR
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
}

// The lane id recomputed where it is used (volatile: never hoisted out of a loop or merged with
// another copy, so lane-derived offsets are rematerialised instead of held in spilled VGPRs)
__device__ __forceinline__ int fresh_lane_id() {
    int l;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
    return l;
}

// Sum over the four 16-lane groups of a wave (lanes l, l^16, l^32, l^48) with two lane-swap pairs
// (no LDS permute, no lane-id arithmetic)
__device__ __forceinline__ float sum_lane_groups(float v) {
    const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    const float s = __uint_as_float(a[0]) + __uint_as_float(a[1]);
    const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(s), __float_as_uint(s), false, false);
    return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}

// ------------------------------------------------------------------------------------------
// SCHED 11 for the residual GEMMs of the folded image tower (out-proj / c_proj with
// EPI_LN_STATS_HL: x += A W^T + b on the hi/lo bf16 planes, LN slab statistics).  SCHED 11's
// epilogue pays vmcnt's issue order twice: a residual load waits for every store issued before it,
// and the next tile's DMAs (issued before the epilogue) sit behind nothing, but the ones after it sit
// behind all its stores.  This variant orders the traffic so that no wait covers a store that has not
// had half an epilogue or a K-tile to drain:
//  * the last two K-tiles of a tile DMA the residual of fragment rows 0-3 of every wave (hi plane at
//    K-tile nk-2, lo plane at nk-1, each into the stage buffer that K-tile frees, 64 KB per plane,
//    16-B chunks XOR-swizzled by row) in place of the next tile's first K-tiles;
//  * the epilogue (a) loads the residual of fragment rows 4-5 into registers (before any store),
//    (b) finishes rows 0-3 from LDS and stores them, (a2) loads rows 6-7, (c) releases the LDS,
//    (d) issues the next tile's bias and K-tiles 0 and 1, (e) finishes rows 4-7 from registers and
//    stores them plus the slab statistics;
//  * the next tile waits for its K-tile 0 with vmcnt(52): the 36 stores of (e) and the 16 DMAs of
//    K-tile 1 may stay in flight.
// Requires N % 256 == 0 (the host falls back to SCHED 1 otherwise) and K >= 128.  A K-tile's
// operand DMAs are spread over B2 (10) and B3 (6) as in SCHED 11.  (Timing ablations without residual
// loads / stores, a store drain per tile and early rows 6-7: DESIGN.md §6.4, §6.12; removed in round 6.)
__global__ __launch_bounds__(256, 1) void gemm_w4_resid_hl(GemmParams p) {
    constexpr bool RSPREAD = true;
    __shared__ __attribute__((aligned(16))) char smem[2 * STAGE_BYTES + 4 * W4_SIDE_BYTES];
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    char* const side = smem + 2 * STAGE_BYTES + wave * W4_SIDE_BYTES;
    const int wm = wave >> 1, wn = wave & 1;
    const int tiles_m = (p.M + BM - 1) / BM;
    const int tiles_n = p.N / BN;
    const int nwg = tiles_m * tiles_n;
    const int grid = gridDim.x;
    // (packed rows: blockIdx order, so the live tiles, the first indices, spread over all XCDs)
    const int slot = p.m_dev ? (int)blockIdx.x : xcd_remap(blockIdx.x, grid);
    const int nk = p.K / BK;
    // tiles t_main..nwg-1 (a last round of <= grid/8 tiles) run as split-K chunks on the 4-phase
    // kernel + gemm_splitk_fixup (plan_tail_rhl)
    const int t_main = nwg - p.tail;
    int my_tiles = slot < t_main ? (t_main - 1 - slot) / grid + 1 : 0;
    // packed rows (one tile per workgroup, forced by the host): clip at the live count
    if (p.m_dev) {
        p.M = min(p.M, __builtin_amdgcn_readfirstlane(*p.m_dev));
        int tm, tn;
        tile_of(min(slot, nwg - 1), tiles_m, tiles_n, p.gm, tm, tn);
        if (tm * BM >= p.M) my_tiles = 0;
    }
    // de-synchronised start (p.stagger x s_sleep 127 for the odd slots): equal tiles keep the CUs in
    // lock-step, K-loops (MFMA-bound) and epilogues (HBM-bound) each chip-wide at once
    if (p.stagger > 0 && (slot & 1))
        for (int i = 0; i < p.stagger; ++i) __builtin_amdgcn_s_sleep(127);

    // per-lane DMA source offsets of a K-tile (A rows, W rows; 16-B chunks swizzled by row pair)
    auto k_offsets = [&](int ln, int& vA, int& vW) {
        const int srow = wave * 8 + (ln >> 3);
        const int schunk = (ln & 7) ^ ((srow >> 1) & 7);
        vA = srow * (int)p.lda * 2 + schunk * 16;
        vW = srow * (int)p.ldw * 2 + schunk * 16;
    };
    int voffA, voffW;
    k_offsets(lane, voffA, voffW);
    const int jstrA = 32 * (int)p.lda * 2, jstrW = 32 * (int)p.ldw * 2;
    __amdgpu_buffer_rsrc_t srdA, srdW, srdH, srdL;
    int m0 = 0, n0 = 0;
    auto set_tile = [&](int t) {
        int tm, tn;
        tile_of(slot + t * grid, tiles_m, tiles_n, p.gm, tm, tn);
        m0 = tm * BM;
        n0 = tn * BN;
        const int rows = max(0, min(p.M - m0, BM));
        srdA = make_srd(p.A + (size_t)m0 * p.lda, rows * (int)p.lda * 2);
        srdW = make_srd(p.W + (size_t)n0 * p.ldw, BN * (int)p.ldw * 2);
        srdH = make_srd(p.rhl + (size_t)m0 * p.ldr, rows * (int)p.ldr * 2);
        srdL = make_srd(p.rhl + p.hl_plane + (size_t)m0 * p.ldr, rows * (int)p.ldr * 2);
    };
    // K-tile kt of the current tile into stage buffer `buf` (16 DMAs per thread)
    // (scalar operands are derived from opaque copies so that the 16 per-instruction offsets and LDS
    // addresses are recomputed at each issue instead of being hoisted into spilled SGPRs)
    auto dma_k = [&](int buf, int kt, int j, int voffA, int voffW) {
        int lb = buf * STAGE_BYTES + wave * 8 * 128;
        int st = j < 8 ? jstrA : jstrW;
        asm volatile("" : "+s"(lb), "+s"(st));
        char* base = smem + lb;
        const int jo = (j < 8 ? j : j - 8) * st;
        if (j < 8)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(srdA, (CE_LDS void*)(base + j * 32 * 128), 16, voffA + jo, kt * BK * 2, 0, 0);
        else
            __builtin_amdgcn_raw_ptr_buffer_load_lds(srdW, (CE_LDS void*)(base + TILE_BYTES + (j - 8) * 32 * 128), 16,
                                                     voffW + jo, kt * BK * 2, 0, 0);
    };
    // residual plane (0 hi, 1 lo) of the staged rows into stage buffer `plane`: staged row
    // r = 0..127 is tile row (r >> 6) * 128 + (r & 63) (fragment rows 0-3 of the two wave rows),
    // 512 B (256 columns), 16-B chunk c of row r at c ^ (r & 15)
    // (the row offset stays in voffset, where the descriptor clips it at row M; the column offset
    // n0 goes to soffset; per-instruction row offsets are opaque so they are not hoisted to VGPRs)
    // (vr0 / vr1: lane offsets of the even / odd instructions, from r_offsets at each use)
    auto r_offsets = [&](int& vr0, int& vr1) {
        const int ln = fresh_lane_id();
        const int rpair = wave * 2 + (ln >> 5);                 // r & 7 of the staged row
        vr0 = (ln >> 5) * (int)p.ldr * 2 + ((ln & 31) ^ rpair) * 16;
        vr1 = (ln >> 5) * (int)p.ldr * 2 + ((ln & 31) ^ (rpair | 8)) * 16;
    };
    auto dma_r = [&](int buf, int plane, int j, int vr0, int vr1) {
        int lb = buf * STAGE_BYTES + wave * 2 * 512;
        int l2 = (int)p.ldr * 2;
        asm volatile("" : "+s"(lb), "+s"(l2));
        const int ro = (j * 8 + wave * 2 + (j >= 8 ? 64 : 0)) * l2;
        char* base = smem + lb + j * 8 * 512;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(plane ? srdL : srdH, (CE_LDS void*)base, 16, ((j & 1) ? vr1 : vr0) + ro,
                                                 n0 * 2, 0, 0);
    };

    const int fr = lane & 15, fq = lane >> 4;
    const int fo0 = fr * 128 + (((0 + fq) ^ (fr >> 1)) << 4);
    const int fo1 = fr * 128 + (((4 + fq) ^ (fr >> 1)) << 4);
    const int a_off = wm * 128 * 128;
    const int w_off = TILE_BYTES + wn * 128 * 128;

    f32x4 acc[8][8];
    bf16x8 a0[8], b0[8], a1[8], b1[8];
    u32x4 rah[8], ral[8];                       // residual of fragment rows 4-5 (hi, lo planes)
    u32x4 rbh[8], rbl[8];                       // rows 6-7
#define CE_MFMA_AGPR(ACC, BV, AV) \
    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(ACC) : "v"(BV), "v"(AV))
    auto read_set0 = [&](const char* sb0) __attribute__((always_inline)) {
        int bo = 0;
        asm volatile("" : "+s"(bo));
        const char* sb = sb0 + bo;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            b0[q] = *reinterpret_cast<const bf16x8*>(sb + w_off + q * 16 * 128 + fo0);
            a0[q] = *reinterpret_cast<const bf16x8*>(sb + a_off + q * 16 * 128 + fo0);
        }
    };
    // one K-tile: B1 | barrier | B2 + 16 DMAs | wait + barrier | B3 (as SCHED 11).  MODE 0: the
    // DMAs fetch K-tile kt + 2 and B3 prefetches set 0 of K-tile kt + 1; MODE 1 (kt = nk - 2): they
    // fetch the hi residual plane; MODE 2 (kt = nk - 1): the lo plane, no prefetch
    auto ktile = [&](int kt, int wait_n, auto mode) __attribute__((always_inline)) {
        constexpr int MODE = decltype(mode)::value;
        const int buf = kt & 1;
        // stage-buffer bases from an opaque scalar: the fragment addresses are formed per K-tile
        // instead of being kept (and spilled) for both buffers
        int bo = buf * STAGE_BYTES;
        asm volatile("" : "+s"(bo));
        const char* sb = smem + bo;
        const char* so = smem + (STAGE_BYTES - bo);
#pragma unroll
        for (int s2 = 0; s2 < 32; ++s2) {
            const int i = s2 >> 3, j = s2 & 7;
            CE_MFMA_AGPR(acc[i][j], b0[j], a0[i]);
            if (s2 & 1) {
                const int q = s2 >> 1;
                if (q < 8) b1[q] = *reinterpret_cast<const bf16x8*>(sb + w_off + q * 16 * 128 + fo1);
                else a1[q - 8] = *reinterpret_cast<const bf16x8*>(sb + a_off + (q - 8) * 16 * 128 + fo1);
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        barrier();
        // K-tile kt + 2, or for the last two K-tiles the residual planes, into this buffer; MODE 1
        // also loads the residual of fragment rows 4-5 into registers (16-B store layout, see
        // load_pair), retired by the last K-tile's wait instead of inside the epilogue
        int rpk = 0, vr0 = 0, vr1 = 0;
        if constexpr (MODE >= 1) r_offsets(vr0, vr1);
        if constexpr (MODE == 1) {
            const int lnr = fresh_lane_id();
            rpk = ((wm * 128 + 64 + (lnr & 15) + ((lnr >> 4) & 1) * 16) * (int)p.ldr + wn * 128 + (lnr >> 5) * 8) * 2;
        }
#pragma unroll
        for (int s2 = 0; s2 < 64; ++s2) {
            const int i = (s2 >> 3) & 3, j = s2 & 7;
            if (s2 < 32) CE_MFMA_AGPR(acc[4 + i][j], b0[j], a0[4 + i]);
            else CE_MFMA_AGPR(acc[i][j], b1[j], a1[i]);
            if constexpr (MODE == 0 && RSPREAD) {
                // 10 of K-tile kt + 2's DMAs here (one per 6 MFMAs), the other 6 in B3
                if (s2 % 6 == 5 && s2 / 6 < 10) dma_k(buf, kt + 2, s2 / 6, voffA, voffW);
            } else if ((s2 & 3) == 3) {
                if constexpr (MODE == 0) dma_k(buf, kt + 2, s2 >> 2, voffA, voffW);
                else dma_r(buf, MODE - 1, s2 >> 2, vr0, vr1);
            }
            if constexpr (MODE == 1) {
                if ((s2 & 3) == 1) {
                    const int q = s2 >> 2;
                    if (q < 8) rah[q] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(srdH, rpk + q * 32, n0 * 2, 0));
                    else ral[q - 8] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(srdL, rpk + (q - 8) * 32, n0 * 2, 0));
                }
            }
        }
        if constexpr (MODE == 1) {
            // 16 residual DMAs + 16 register loads younger than K-tile nk - 1 (+ the previous
            // epilogue's 36 stores when nk == 2: 68 > 63, so the wait over-covers by 5)
            if (wait_n == 16) asm volatile("s_waitcnt vmcnt(32)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(63)" ::: "memory");
        } else if constexpr (MODE == 0 && RSPREAD) {
            // only this B2's 10 DMAs (+ after an epilogue its 36 stores) are younger than K-tile kt + 1
            if (wait_n == 16) asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
            else if (wait_n == 52) asm volatile("s_waitcnt vmcnt(46)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        } else {
            if (wait_n == 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
            else if (wait_n == 52) asm volatile("s_waitcnt vmcnt(52)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        barrier();
#pragma unroll
        for (int s2 = 0; s2 < 32; ++s2) {
            const int i = s2 >> 3, j = s2 & 7;
            CE_MFMA_AGPR(acc[4 + i][j], b1[j], a1[4 + i]);
            if constexpr (MODE == 0 && RSPREAD) {
                // the other 6 DMAs of K-tile kt + 2 (buf's last reader was B1, before the first barrier)
                if (s2 % 5 == 4) dma_k(buf, kt + 2, 10 + s2 / 5, voffA, voffW);
            }
            if constexpr (MODE < 2) {
                if (s2 & 1) {
                    const int q = s2 >> 1;
                    if (q == 0) a0[0] = *reinterpret_cast<const bf16x8*>(so + a_off + fo0);
                    else if (q < 9) b0[q - 1] = *reinterpret_cast<const bf16x8*>(so + w_off + (q - 1) * 16 * 128 + fo0);
                    else a0[q - 8] = *reinterpret_cast<const bf16x8*>(so + a_off + (q - 8) * 16 * 128 + fo0);
                }
            }
        }
    };
    using K_ = std::integral_constant<int, 0>;
    using R0_ = std::integral_constant<int, 1>;
    using R1_ = std::integral_constant<int, 2>;

    const int ldo = (int)p.ldo, ldr = (int)p.ldr;
    constexpr int NS = 2;                                       // 64-column slabs per wave quadrant
    if (my_tiles > 0) {
        set_tile(0);
        w4_side_fill<EPI_PLAIN>(p, side, m0 + wm * 128, n0 + wn * 128, lane);
#pragma unroll
        for (int j = 0; j < 16; ++j) dma_k(0, 0, j, voffA, voffW);
#pragma unroll
        for (int j = 0; j < 16; ++j) dma_k(1, 1, j, voffA, voffW);
    }
    for (int t = 0; t < my_tiles; ++t) {
        // K-tile 0 landed: the younger ops are K-tile 1's 16 DMAs and (t > 0) the 32 stores of the
        // previous epilogue's rows 4-7 + its 4 slab-statistics stores, which keep draining
        if (t == 0) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(52)" ::: "memory");
        barrier();
        {
            // the accumulators start at the bias (DMA'd to the side area ahead of K-tile 0)
            // (read with asm ds_reads: the bias DMA is older than K-tile 0, which the wait above
            // retired, but the compiler would wait for every LDS-DMA in flight, K-tile 1's included)
            const int lnb = fresh_lane_id();
            const unsigned ba = (unsigned)(uintptr_t)(CE_LDS void*)side + (lnb >> 4) * 16;
            f32x4 bv[8];
#define CE_RD(J) asm volatile("ds_read_b128 %0, %1 offset:" #J "" : "=v"(bv[J / 64]) : "v"(ba))
            CE_RD(0); CE_RD(64); CE_RD(128); CE_RD(192); CE_RD(256); CE_RD(320); CE_RD(384); CE_RD(448);
#undef CE_RD
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
            for (int i = 0; i < 8; ++i)
#pragma unroll
                for (int j = 0; j < 8; ++j) acc[i][j] = bv[j];
        }
        read_set0(smem);
        trace_stamp(p, 0, t * grid + blockIdx.x);
        // K-tile kt + 1 landed (kt = 0 of a later tile: the previous epilogue's 36 stores are younger
        // than K-tile 1 too)
        for (int kt = 0; kt < nk - 2; ++kt) ktile(kt, (kt == 0 && t > 0) ? 52 : 16, K_{});
        ktile(nk - 2, (nk == 2 && t > 0) ? 52 : 16, R0_{});
        ktile(nk - 1, 0, R1_{});                // residual planes landed for every wave
        trace_stamp(p, 1, t * grid + blockIdx.x);

        const int mbase = m0 + wm * 128, nbase = n0 + wn * 128;
        // lane-derived offsets from an opaque copy of the lane id: recomputed per tile rather than
        // hoisted out of the tile loop into (spilled) registers
        const int lne = fresh_lane_id();
        const int fre = lne & 15, fqe = lne >> 4;
        const int rows = max(0, min(p.M - mbase, 128));
        // residual rows in registers (per-row offsets are opaque: hoisted, they would be spilled, and
        // a scratch reload waits for every store)
        const __amdgpu_buffer_rsrc_t hs = make_srd(p.rhl + (size_t)mbase * ldr, rows * ldr * 2);
        const __amdgpu_buffer_rsrc_t ls = make_srd(p.rhl + p.hl_plane + (size_t)mbase * ldr, rows * ldr * 2);
        // a fragment-row pair (i0, i0 + 1) is loaded in the store layout (16 B = 8 columns of one
        // row per lane, half the instructions of the 8-B fragment layout) and turned into fragments
        // by the same v_permlane16_swap pairing that the stores use (an involution)
        const int rp = ((fre + (fqe & 1) * 16) * ldr + nbase + (fqe >> 1) * 8) * 2;
        auto load_pair = [&](u32x4 (&h)[8], u32x4 (&l)[8], int i0) __attribute__((always_inline)) {
            int io = i0 * 16 * ldr * 2;
            asm volatile("" : "+s"(io));
            const int vo = rp + io;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                h[j] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(hs, vo + j * 32, 0, 0));
                l[j] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(ls, vo + j * 32, 0, 0));
            }
        };
        // (a) rows 6-7 (rows 4-5 arrived with the last K-tiles)
        load_pair(rbh, rbl, 6);
        const __amdgpu_buffer_rsrc_t xs = make_srd(p.xb + (size_t)mbase * ldo, rows * ldo * 2);
        const __amdgpu_buffer_rsrc_t xl = make_srd(p.xb + p.hl_plane + (size_t)mbase * ldo, rows * ldo * 2);
        int xo = ((fre + (fqe & 1) * 16) * ldo + nbase + (fqe >> 1) * 8) * 2;
        float2 sta[NS], stb[NS];                 // initialised: not carried across tiles
#pragma unroll
        for (int sl = 0; sl < NS; ++sl) sta[sl] = stb[sl] = make_float2(0.f, 0.f);
        // fragment rows i0 and i0 + 1: v = acc (+ bias) + residual; (mean, M2) per 64-column slab;
        // hi/lo planes of the two rows paired by v_permlane16_swap into 16-B stores
        auto row_pair = [&](int i0, auto get_r) __attribute__((always_inline)) {
            float lmean[2][NS], lm2[2][NS];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                uint2 h[2], l[2];
                float4 rr[2];
                get_r(i0, j, rr);
#pragma unroll
                for (int r2 = 0; r2 < 2; ++r2) {
                    f32x4 v = acc[i0 + r2][j];
                    const float4 r = rr[r2];
                    v[0] += r.x; v[1] += r.y; v[2] += r.z; v[3] += r.w;
                    const float m4 = ((v[0] + v[1]) + (v[2] + v[3])) * 0.25f;
                    const float d0 = v[0] - m4, d1 = v[1] - m4, d2 = v[2] - m4, d3 = v[3] - m4;
                    const float q4 = fmaf(d0, d0, fmaf(d1, d1, fmaf(d2, d2, d3 * d3)));
                    const int sl = j >> 2, jj = j & 3;
                    if (jj == 0) {
                        lmean[r2][sl] = m4;
                        lm2[r2][sl] = q4;
                    } else {
                        const float dl = m4 - lmean[r2][sl];
                        lmean[r2][sl] = fmaf(dl, 1.0f / (jj + 1), lmean[r2][sl]);
                        lm2[r2][sl] += fmaf(dl * dl, 4.0f * jj / (jj + 1), q4);
                    }
                    split_hl(v[0], v[1], h[r2].x, l[r2].x);
                    split_hl(v[2], v[3], h[r2].y, l[r2].y);
                }
                const auto x = __builtin_amdgcn_permlane16_swap(h[0].x, h[1].x, false, false);
                const auto y = __builtin_amdgcn_permlane16_swap(h[0].y, h[1].y, false, false);
                const auto xx = __builtin_amdgcn_permlane16_swap(l[0].x, l[1].x, false, false);
                const auto yy = __builtin_amdgcn_permlane16_swap(l[0].y, l[1].y, false, false);
                const u32x4 dh = {x[0], y[0], x[1], y[1]};
                const u32x4 dl = {xx[0], yy[0], xx[1], yy[1]};
                __builtin_amdgcn_raw_buffer_store_b128(dh, xs, xo + j * 32, 0, CE_STORE_AUX);
                __builtin_amdgcn_raw_buffer_store_b128(dl, xl, xo + j * 32, 0, CE_STORE_AUX);
            }
            xo += 32 * ldo * 2;
#pragma unroll
            for (int r2 = 0; r2 < 2; ++r2) {
                const int i = i0 + r2;
#pragma unroll
                for (int sl = 0; sl < NS; ++sl) {
                    const float mean = sum_lane_groups(lmean[r2][sl]) * 0.25f;
                    const float dl = lmean[r2][sl] - mean;
                    const float q = sum_lane_groups(fmaf(dl * dl, 16.0f, lm2[r2][sl]));
                    if (fqe == (i & 3)) {
                        if (i < 4) sta[sl] = make_float2(mean, q);
                        else stb[sl] = make_float2(mean, q);
                    }
                }
            }
        };
        // (b) fragment rows 0-3: residual from the staged planes
        const int lr0 = ((nk - 2) & 1) * STAGE_BYTES + (wm * 64 + fre) * 512;
        const int llo = (((nk - 1) & 1) - ((nk - 2) & 1)) * STAGE_BYTES;
        auto lds_r = [&](int i0, int j, float4 (&rr)[2]) {
            const int c = (wn * 16 + 2 * j + (fqe >> 1)) ^ fre;        // staged row r has r & 15 == fre
#pragma unroll
            for (int r2 = 0; r2 < 2; ++r2) {
                const int off = lr0 + (i0 + r2) * 16 * 512 + (c << 4) + (fqe & 1) * 8;
                int offl = llo + off;
                const uint2 h = *reinterpret_cast<const uint2*>(smem + off);
                const uint2 l = *reinterpret_cast<const uint2*>(smem + offl);
                const float2 a = join_hl(h.x, l.x), b = join_hl(h.y, l.y);
                rr[r2] = make_float4(a.x, a.y, b.x, b.y);
            }
        };
        row_pair(0, lds_r);
        asm volatile("" ::: "memory");          // rows 2-3's LDS reads stay behind rows 0-1 (VGPRs)
        row_pair(2, lds_r);
        // (c) every wave's LDS residual reads done -> (d) the next tile's bias and K-tiles 0 and 1
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        barrier();
        if (t + 1 < my_tiles) {
            set_tile(t + 1);
            w4_side_fill<EPI_PLAIN>(p, side, m0 + wm * 128, n0 + wn * 128, lne);
            int vA, vW;
            k_offsets(lne, vA, vW);
#pragma unroll
            for (int j = 0; j < 16; ++j) dma_k(0, 0, j, vA, vW);
#pragma unroll
            for (int j = 0; j < 16; ++j) dma_k(1, 1, j, vA, vW);
        }
        // (e) fragment rows 4-7 from the registers of (a) and (a2)
        auto reg_r = [&](int i0, int j, float4 (&rr)[2]) {
            const u32x4 dh = i0 == 4 ? rah[j] : rbh[j], dl = i0 == 4 ? ral[j] : rbl[j];
            const auto hx = __builtin_amdgcn_permlane16_swap(dh[0], dh[2], false, false);
            const auto hy = __builtin_amdgcn_permlane16_swap(dh[1], dh[3], false, false);
            const auto lx = __builtin_amdgcn_permlane16_swap(dl[0], dl[2], false, false);
            const auto ly = __builtin_amdgcn_permlane16_swap(dl[1], dl[3], false, false);
#pragma unroll
            for (int r2 = 0; r2 < 2; ++r2) {
                const float2 a = join_hl(hx[r2], lx[r2]), b = join_hl(hy[r2], ly[r2]);
                rr[r2] = make_float4(a.x, a.y, b.x, b.y);
            }
        };
        row_pair(4, reg_r);
        row_pair(6, reg_r);
        // slab statistics: rows fqe and fqe + 4 of this lane's 16-row groups (clipped at M)
        {
            const int ns = p.N / 64;
            const __amdgpu_buffer_rsrc_t ss = make_srd(p.stats_part + (size_t)mbase * ns, rows * ns * 8);
            const int so = ((fqe * 16 + fre) * ns + nbase / 64) * 8;
#pragma unroll
            for (int sl = 0; sl < NS; ++sl) {
                __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, sta[sl]), ss, so + sl * 8, 0, 0);
                __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, stb[sl]), ss, so + 64 * ns * 8 + sl * 8, 0, 0);
            }
        }
        trace_stamp(p, 2, t * grid + blockIdx.x);
    }
#undef CE_MFMA_AGPR
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
}

// Process-wide A/B knobs (knobs.h: atomics, env value published by the first reader)
std::atomic<int> g_variant{kKnobUnset};
int variant_env() { const int v = env_int("CE_GEMM_VARIANT", CE_GEMM_VAR_DEFAULT); return v < 0 ? 0 : v; }
int gemm_variant() { return knob_get(g_variant, variant_env); }

// Main-loop schedule: 1 = the default shape policy (SCHED 1 / the four-wave kernels by shape), 11 = the
// four-wave persistent kernel wherever its epilogues apply.
bool sched_ok(int sc) { return sc == 1 || sc == 11; }
// The schedule knobs in ONE atomic word, so a launch never sees a half-applied ce_set_gemm_schedule:
// bits 0-7 schedule, 8-15 tile-order M-group, 16-30 first-round stagger (units of s_sleep 127).
constexpr int pack_sched(int sc, int gm, int st) { return sc | (gm << 8) | (st << 16); }
std::atomic<int> g_sched{kKnobUnset};
int sched_env() {
    const int sc = env_int("CE_GEMM_SCHED", 1), g = env_int("CE_GEMM_GROUPM", 4);
    const int st = std::max(0, std::min(env_int("CE_GEMM_STAGGER", 0), 0x7fff));
    return pack_sched(sched_ok(sc) ? sc : 1, (g < 1 || g > 64) ? 1 : g, st);
}
int gemm_sched_word() { return knob_get(g_sched, sched_env); }
// diagnostic timeline buffer (ce_set_gemm_trace): process-wide by contract (clipembed.h); pointer and
// size change together under the lock and a launch reads them together
struct TraceBuf { unsigned long long* buf = nullptr; long n = 0; };
TraceBuf g_trace;
std::mutex g_trace_mu;

int num_cus() { return device_cus(); }

// Split-K tail plan: with one 512-thread workgroup per CU, a grid of T tiles runs in ceil(T / CUs)
// rounds; when the last round holds only R = T % CUs tiles the chip idles for most of a tile time.
// Those R tiles are split into S K-chunks (R * S <= CUs) so the last round is ~1/S of a tile, plus a
// tiny fixup launch.
std::atomic<int> g_splitk{kKnobUnset};
int splitk_env() { return env_int("CE_GEMM_SPLITK", 1) != 0; }
bool splitk_enabled() { return knob_get(g_splitk, splitk_env) != 0; }

void plan_tail(GemmParams& p, int nwg) {
    p.tail = 0;
    p.split = 1;
    const int C = num_cus(), nk = p.K / BK;
    if (!p.kn.splitk || !p.part) return;
    int R, cap;
    if ((nwg <= C / 2 && nk >= 32) || (nwg <= C / 16 && nk >= 8)) {
        // small grid, long K (weight gradients: M = out features, K = tokens), or a grid of a few
        // tiles (the pooled rows' GEMMs, M = batch): split every tile
        R = nwg;
        cap = 64;
    } else {
        if (nwg <= C) return;
        R = nwg % C;
        if (R == 0 || R > C / 32) return;     // measured: R = 4 (out/c_proj) gains 3-5 %, R = 12 (QKV) loses
        cap = 16;
    }
    int S = std::min(std::min(nk, cap), C / R);
    while (S >= 2 && (long)R * S * BM * BN > p.part_elems) --S;
    if (S < 2) return;
    p.tail = R;
    p.split = S;
}

// Per-device partial-tile workspace for the kernel-level entry point (engine handles pass their own).
// Allocated once per device under a lock (kernel-level callers on several threads); the slabs are
// used by one launch at a time per device stream order — concurrent kernel-level GEMMs with a
// split-K tail on two streams of one device would share them, so the engine passes its own.
float* g_part[kMaxDevices] = {};
std::mutex g_part_mu;
constexpr long kPartElems = 256L * BM * BN;     // 64 MB: R * S <= 256 slabs
float* kernel_api_part() {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevices) return nullptr;
    std::lock_guard<std::mutex> lk(g_part_mu);
    if (!g_part[dev] && hipMalloc(&g_part[dev], kPartElems * sizeof(float)) != hipSuccess) {
        (void)hipGetLastError();
        g_part[dev] = nullptr;
    }
    return g_part[dev];
}

// The epilogues the four-wave persistent kernel has: bf16 without residual (plain / LN fold; the
// one-wave-per-SIMD epilogue, GEMM_VAR_W4_EPI2), the f32 LN-statistics residual (EPI2, identity row
// map), and a plain f32 output without residual or activation (the generic register epilogue: the
// PACL head's linear branch)
template <int ACT, bool HAS_RESID, bool OUT_BF16, int EPI>
constexpr bool w4_has() {
    return (OUT_BF16 && !HAS_RESID && (EPI == EPI_PLAIN || EPI == EPI_LN_FOLD)) ||
           (EPI == EPI_LN_STATS && HAS_RESID && !OUT_BF16) || (!OUT_BF16 && !HAS_RESID && EPI == EPI_PLAIN && ACT == ACT_NONE);
}
template <int ACT, bool HAS_RESID, bool OUT_BF16, int EPI>
bool w4_ok(const GemmParams& p) {
    if constexpr (OUT_BF16 && !HAS_RESID && (EPI == EPI_PLAIN || EPI == EPI_LN_FOLD))
        return (p.variant & GEMM_VAR_W4_EPI2) != 0;
    else if constexpr (EPI == EPI_LN_STATS && HAS_RESID && !OUT_BF16) return (p.variant & GEMM_VAR_W4_EPI2) != 0 && p.grp == 0;
    else if constexpr (!OUT_BF16 && !HAS_RESID && EPI == EPI_PLAIN && ACT == ACT_NONE) return true;
    else return false;
}

// SCHED 11 split-K tail: a grid of nwg tiles over `grid` persistent workgroups whose last round
// holds r <= grid / 8 tiles idles most of the chip for a whole tile; the persistent kernel runs the
// whole rounds only, and those r tiles follow as S K-chunks (about 4 K-tiles each, r * S <= grid) on
// the 4-phase kernel in tail-only mode, summed and finished by gemm_splitk_fixup (vision QKV
// 6924 = 27 * 256 + 12 tiles, c_fc 9232 = 36 * 256 + 16).  Off by default (GEMM_VAR_W4_TAIL).
void plan_tail_w4(GemmParams& p, int nwg, int grid) {
    p.tail = 0;
    p.split = 1;
    if (!p.kn.splitk || !p.part || !(p.variant & GEMM_VAR_W4_TAIL)) return;
    const int r = nwg % grid, nk = p.K / BK;
    if (nwg < grid || r == 0 || r > grid / 8) return;
    int S = std::min(std::min(std::max(nk / 4, 2), 16), std::min(grid / r, nk));
    while (S >= 2 && (long)r * S * BM * BN > p.part_elems) --S;
    if (S < 2) return;
    p.tail = r;
    p.split = S;
}

// Split-K tail of the staged-residual kernel (default on with split-K): a last round of r <= grid/8
// tiles (B = 256: 2308 tiles = 9 x 256 + 4) would hold one tile period (c_proj ~135 us) for r CUs;
// those tiles run as S K-chunks on the 4-phase kernel instead (tail_only) + the hi/lo fixup
void plan_tail_rhl(GemmParams& p, int nwg, int grid) {
    p.tail = 0;
    p.split = 1;
    if (!p.kn.splitk || !p.part) return;
    const int r = nwg % grid, nk = p.K / BK;
    if (nwg < grid || r == 0 || r > grid / 8) return;
    int S = std::min(std::min(std::max(nk / 4, 2), 16), std::min(grid / r, nk));
    while (S >= 2 && (long)r * S * BM * BN > p.part_elems) --S;
    if (S < 2) return;
    p.tail = r;
    p.split = S;
}

// SCHED 11 grid: one workgroup per CU, a multiple of 8 so every XCD group is complete
// (GEMM_VAR_W4_ONETILE: one workgroup per tile)
int w4pp_grid(const GemmParams& p, int nwg, bool onetile = false) {
    const int need = ((nwg + 7) / 8) * 8;
    if (onetile || (p.variant & GEMM_VAR_W4_ONETILE)) return need;
    const int grid = (num_cus() / 8) * 8;
    return grid < need ? grid : need;
}

// Shape policy of the default schedule (CE_GEMM_AUTO, default 1): SCHED 11 for large grids
// (>= 4 tiles per CU) without a residual — the vision QKV and c_fc GEMMs, plain or LN-folded, with
// or without GELU — when its one-wave-per-SIMD epilogue (GEMM_VAR_W4_EPI2) is on; otherwise only
// the no-activation ones (the round-1 policy).  The hi/lo residual GEMMs (out-proj / c_proj) run on
// their own staged-residual four-wave kernel (launch_epi); the f32-stream residual epilogues stay on
// SCHED 1: on the persistent grid vmcnt retires the epilogue's stores and the next tile's DMAs in
// issue order, so their 384 KB per tile must drain within two K-tiles (r02 A/B: out-proj 572 vs
// 593 TF/s, c_proj 1037 vs 1025; with the stores ablated 855 / 1204, profiles/r02).
// CE_GEMM_AUTO=0 pins SCHED 1, =2 sends every large grid to SCHED 11, =3 every residual-free one.
std::atomic<int> g_auto{kKnobUnset};
int auto_env() { const int a = env_int("CE_GEMM_AUTO", 1); return (a < 0 || a > 3) ? 1 : a; }
int gemm_auto() { return knob_get(g_auto, auto_env); }
bool auto_w4pp(const GemmParams& p, int act, bool resid) {
    const int on = p.kn.autom;
    if (!on || p.kn.sched != 1) return false;
    if (p.onetile) return !resid && (act == ACT_NONE || (p.variant & GEMM_VAR_W4_EPI2) != 0);
    // enough tiles that the persistent grid's last-round imbalance stays small (small grids keep
    // SCHED 1 and its split-K tail)
    const int nwg = ((p.M + BM - 1) / BM) * ((p.N + BN - 1) / BN);
    if (nwg < 4 * num_cus()) return false;
    if (on == 2) return true;
    if (on == 3) return !resid;
    if (resid) return false;
    return act == ACT_NONE || (p.variant & GEMM_VAR_W4_EPI2) != 0;
}

// Launch counters per kernel path (ce_gemm_path_counts): lets the parity tests assert that the
// instantiations a configuration selects by default (e.g. SCHED 11 + LN fold, split-K + LN stats at
// B = 256) are the ones they just checked.
std::atomic<long long> g_path[GEMM_PATH_COUNT];
inline void count_path(int path) { g_path[path].fetch_add(1, std::memory_order_relaxed); }

// SCHED 1 (one workgroup per CU): half the CUs of every XCD (bit 3 of the block id: blocks b and
// b + 8 share an XCD) start their first tile late
void set_stagger_1(GemmParams& p, int nwg) {
    if (nwg <= 2 * num_cus()) return;
    p.stagger = p.kn.stagger;
    p.stagger_lo = 0;
    p.stagger_hi = num_cus();
    p.stagger_bit = 3;
}

// The four-wave persistent kernel (+ its optional split-K tail on the 4-phase kernel)
template <int ACT, bool HAS_RESID, bool OUT_BF16, int EPI>
hipError_t launch_w4pp(GemmParams& p, hipStream_t s) {
    p.gm = p.kn.groupm;
    p.stagger = p.kn.stagger;
    const int nwg = ((p.M + BM - 1) / BM) * ((p.N + BN - 1) / BN);
    const int grid = w4pp_grid(p, nwg, p.onetile);
    plan_tail_w4(p, nwg, grid);
    if (p.pre_out && p.tail > 0) return hipErrorInvalidValue;     // the tail kernel has no pre_out store
    hipLaunchKernelGGL((gemm_bf16_w4pp<ACT, HAS_RESID, OUT_BF16, EPI>), dim3(grid), dim3(256), 0, s, p);
    count_path(GEMM_PATH_W4PP + EPI);
    if (p.tail > 0) {
        GemmParams q = p;
        q.tail_only = 1;
        hipLaunchKernelGGL((gemm_bf16_nt<ACT, HAS_RESID, OUT_BF16, EPI == EPI_LN_STATS ? 3 : CE_RESID_RING, EPI>),
                           dim3(p.tail * p.split), dim3(NTHREADS), 0, s, q);
        hipLaunchKernelGGL((gemm_splitk_fixup<ACT, HAS_RESID, OUT_BF16, EPI>), dim3(p.tail * 64), dim3(256), 0, s, p);
        count_path(GEMM_PATH_FIXUP + EPI);
    }
    return hipGetLastError();
}

template <int ACT, bool HAS_RESID, bool OUT_BF16, int EPI>
hipError_t launch_epi(const GemmParams& p0, hipStream_t s) {
    GemmParams p = p0;
    constexpr bool HL = EPI == EPI_LN_STATS_HL || EPI == EPI_HL_F32;
    if constexpr (EPI == EPI_LN_STATS_HL) {
        // staged-residual four-wave kernel (default policy): whole 256-column tiles, >= 2 K-tiles,
        // a grid of >= 2 tiles per CU (no split-K tail); CE_GEMM_AUTO=0 or a pinned schedule keeps
        // SCHED 1 (r02 A/B at B = 256: out-proj 682 vs 589 TF/s, c_proj 1,092 vs 995)
        const int nwg = ((p.M + BM - 1) / BM) * (p.N / BN);
        if ((p.variant & GEMM_VAR_W4_RHL) && p.kn.autom != 0 && p.kn.sched == 1 && p.N % BN == 0 &&
            p.K >= 2 * BK && (nwg >= 2 * num_cus() || p.onetile)) {
            p.gm = p.kn.groupm;
            p.stagger = p.kn.stagger;
            const int grid = w4pp_grid(p, nwg, p.onetile);
            plan_tail_rhl(p, nwg, grid);
            hipLaunchKernelGGL(gemm_w4_resid_hl, dim3(grid), dim3(256), 0, s, p);
            count_path(GEMM_PATH_W4PP + EPI_LN_STATS);
            if (p.tail > 0) {
                GemmParams q = p;
                q.tail_only = 1;
                hipLaunchKernelGGL((gemm_bf16_nt<ACT_NONE, true, false, 3, EPI_LN_STATS_HL>), dim3(p.tail * p.split),
                                   dim3(NTHREADS), 0, s, q);
                hipLaunchKernelGGL((gemm_splitk_fixup<ACT_NONE, true, false, EPI_LN_STATS_HL>), dim3(p.tail * 64),
                                   dim3(256), 0, s, p);
                count_path(GEMM_PATH_FIXUP + EPI_LN_STATS);
            }
            return hipGetLastError();
        }
    }
    if constexpr (!HL && w4_has<ACT, HAS_RESID, OUT_BF16, EPI>())
        if ((p.kn.sched == 11 || auto_w4pp(p, ACT, HAS_RESID)) && w4_ok<ACT, HAS_RESID, OUT_BF16, EPI>(p))
            return launch_w4pp<ACT, HAS_RESID, OUT_BF16, EPI>(p, s);
    p.gm = p.kn.groupm;
    const int nwg = ((p.M + BM - 1) / BM) * ((p.N + BN - 1) / BN);
    p.tail = 0;
    p.split = 1;
    plan_tail(p, nwg);
    set_stagger_1(p, nwg);
    constexpr int RG = (EPI == EPI_LN_STATS || EPI == EPI_LN_STATS_HL) ? 3 : CE_RESID_RING;
    // path counters: the hi/lo epilogues count as their f32-stream counterparts
    constexpr int CNT = EPI == EPI_LN_STATS_HL ? EPI_LN_STATS : EPI == EPI_HL_F32 ? EPI_PLAIN : EPI;
    hipLaunchKernelGGL((gemm_bf16_nt<ACT, HAS_RESID, OUT_BF16, RG, EPI>), dim3(nwg - p.tail + p.tail * p.split),
                       dim3(NTHREADS), 0, s, p);
    count_path(GEMM_PATH_NT + CNT);
    if (p.tail > 0) {
        hipLaunchKernelGGL((gemm_splitk_fixup<ACT, HAS_RESID, OUT_BF16, EPI>), dim3(p.tail * 64), dim3(256), 0, s, p);
        count_path(GEMM_PATH_FIXUP + CNT);
    }
    return hipGetLastError();
}

// The pre-activation copy (GemmParams::pre_out) is written only by the four-wave persistent kernel's
// one-wave-per-SIMD bf16 epilogue (w4_epilogue_bf16_n, EPI_PLAIN with an activation) over every tile:
// no split-K tail (its tiles run on SCHED 1, which has no pre_out store), no one-tile grid.
// launch_gemm routes pre_out launches through here only when this holds, and launch_w4pp rejects
// a launch whose plan would leave pre_out unwritten (the backward would read stale values).
bool pre_out_fused(const GemmParams& p, int act) {
    return act != ACT_NONE && !p.onetile && auto_w4pp(p, act, false) && (p.variant & GEMM_VAR_W4_EPI2) &&
           !(p.variant & GEMM_VAR_W4_TAIL);
}

// knobs of one launch (launch_gemm's snapshot, GemmParams::kn)
void snapshot_knobs(GemmParams& p) {
    {
        std::lock_guard<std::mutex> lk(g_trace_mu);
        p.trace = g_trace.buf;
        p.trace_n = (int)std::min<long>(g_trace.n, 1 << 30);
    }
    p.variant = gemm_variant();
    const int sw = gemm_sched_word();
    p.kn.sched = sw & 0xff;
    p.kn.groupm = (sw >> 8) & 0xff;
    p.kn.stagger = (sw >> 16) & 0x7fff;
    p.kn.autom = gemm_auto();
    p.kn.splitk = splitk_enabled() ? 1 : 0;
    p.kn.snap = 1;
    p.onetile = (p.onetile && (p.variant & GEMM_VAR_SMALL_ONETILE)) ? 1 : 0;
}

// The activation-backward epilogue exists on the four-wave persistent kernel only, without a split-K
// tail, for whole 128-column quadrants.
bool act_bwd_fused_k(const GemmParams& p, int act) {
    return (act == ACT_GELU || act == ACT_QGELU) && p.bwd_pre && p.bwd_part && p.out && !p.bias && !p.resid &&
           !p.rhl && !p.pre_out && !p.m_dev && !p.grp && !p.onetile && p.M > 0 && p.ldo == p.N && p.N % 128 == 0 &&
           p.K > 0 && p.K % BK == 0 && auto_w4pp(p, act, false) && (p.variant & GEMM_VAR_W4_EPI2) &&
           !(p.variant & GEMM_VAR_W4_TAIL);
}

template <int ACT, bool HAS_RESID, bool OUT_BF16>
hipError_t launch_t(const GemmParams& p0, hipStream_t s) {
    GemmParams p = p0;
    if (p.pre_out && !(OUT_BF16 && !HAS_RESID && pre_out_fused(p, ACT))) return hipErrorInvalidValue;
    if constexpr (w4_has<ACT, HAS_RESID, OUT_BF16, EPI_PLAIN>())
        if ((p.kn.sched == 11 || auto_w4pp(p, ACT, HAS_RESID)) && w4_ok<ACT, HAS_RESID, OUT_BF16, EPI_PLAIN>(p))
            return launch_w4pp<ACT, HAS_RESID, OUT_BF16, EPI_PLAIN>(p, s);
    if (p.pre_out) return hipErrorInvalidValue;
    p.gm = p.kn.groupm;
    const int nwg = ((p.M + BM - 1) / BM) * ((p.N + BN - 1) / BN);
    p.tail = 0;
    p.split = 1;
    set_stagger_1(p, nwg);
    plan_tail(p, nwg);
    hipLaunchKernelGGL((gemm_bf16_nt<ACT, HAS_RESID, OUT_BF16>), dim3(nwg - p.tail + p.tail * p.split),
                       dim3(NTHREADS), 0, s, p);
    count_path(GEMM_PATH_NT);
    if (p.tail > 0) {
        hipLaunchKernelGGL((gemm_splitk_fixup<ACT, HAS_RESID, OUT_BF16>), dim3(p.tail * 64), dim3(256), 0, s, p);
        count_path(GEMM_PATH_FIXUP);
    }
    return hipGetLastError();
}

}  // namespace

int set_gemm_variant(int bits) {
    const int prev = gemm_variant();
    g_variant = bits >= 0 ? bits : CE_GEMM_VAR_DEFAULT;
    return prev;
}

int set_gemm_auto(int mode) {
    const int prev = gemm_auto();
    g_auto = (mode >= 0 && mode <= 3) ? mode : 1;
    return prev;
}

void gemm_path_counts(long long* out, int n, bool reset) {
    for (int i = 0; i < GEMM_PATH_COUNT; ++i) {
        const long long v = reset ? g_path[i].exchange(0) : g_path[i].load();
        if (i < n) out[i] = v;
    }
}

int set_gemm_splitk(int on) {
    const int prev = splitk_enabled() ? 1 : 0;
    g_splitk = on != 0;
    return prev;
}

float* gemm_kernel_api_workspace(long* elems) {
    *elems = kPartElems;
    return kernel_api_part();
}

int set_gemm_schedule(int v) {
    // one read-modify-write of the packed word: schedule (bits 0-7; other values select 1), M-group
    // (8-15, 0 keeps it), stagger + 1 (24-30, 0 keeps it)
    int cur = gemm_sched_word();
    for (;;) {
        const int sc = v & 0xff, gm = (v >> 8) & 0xff, st = (v >> 24) & 0x7f;
        const int nsc = sched_ok(sc) ? sc : 1;
        const int ngm = gm ? (gm <= 64 ? gm : 1) : (cur >> 8) & 0xff;
        const int nst = st ? st - 1 : (cur >> 16) & 0x7fff;
        if (g_sched.compare_exchange_weak(cur, pack_sched(nsc, ngm, nst), std::memory_order_acq_rel))
            return cur & 0xffff;
    }
}

int current_gemm_sched() { return gemm_sched_word() & 0xff; }

void set_gemm_trace(unsigned long long* buf, long n) {
    std::lock_guard<std::mutex> lk(g_trace_mu);
    g_trace.buf = buf;
    g_trace.n = buf ? n : 0;
}

bool gemm_act_bwd_fused(GemmParams& p, int act) {
    snapshot_knobs(p);
    return act_bwd_fused_k(p, act);
}

hipError_t launch_gemm_act_bwd(const GemmParams& p0, int act, hipStream_t s) {
    GemmParams p = p0;
    if (!p.kn.snap) snapshot_knobs(p);      // (gemm_act_bwd_fused's snapshot otherwise: one decision)
    if (!act_bwd_fused_k(p, act)) return hipErrorNotSupported;
    p.gm = p.kn.groupm;
    p.stagger = p.kn.stagger;
    const int nwg = ((p.M + BM - 1) / BM) * (p.N / BN);
    const int grid = w4pp_grid(p, nwg);
    plan_tail_w4(p, nwg, grid);
    if (p.tail) return hipErrorNotSupported;      // (W4_TAIL excluded by act_bwd_fused_k: unreachable)
    if (act == ACT_GELU)
        hipLaunchKernelGGL((gemm_bf16_w4pp<ACT_GELU_BWD, false, true, EPI_PLAIN>), dim3(grid), dim3(256), 0, s, p);
    else
        hipLaunchKernelGGL((gemm_bf16_w4pp<ACT_QGELU_BWD, false, true, EPI_PLAIN>), dim3(grid), dim3(256), 0, s, p);
    count_path(GEMM_PATH_W4PP + EPI_PLAIN);
    return hipGetLastError();
}

hipError_t launch_gemm(const GemmParams& p0, int act, bool out_bf16, hipStream_t s, int epi) {
    GemmParams p = p0;
    snapshot_knobs(p);
    if (p.bwd_pre || p.bwd_part) return hipErrorInvalidValue;   // launch_gemm_act_bwd only
    if (p.M <= 0 || p.N <= 0) return hipSuccess;
    if (p.m_dev) {
        // packed rows: the folded-tower epilogues on one tile per workgroup, no split-K; only the default
        // schedule's kernels clip at the device row count (run_text turns the packing off otherwise)
        if ((epi != EPI_LN_FOLD && epi != EPI_LN_STATS_HL) || p.kn.sched != 1) return hipErrorInvalidValue;
        p.onetile = 1;
        p.part = nullptr;
        p.part_elems = 0;
    }
    const bool res = p.resid != nullptr;
    if (p.K % BK != 0 || p.N % 64 != 0 || p.K <= 0) return hipErrorInvalidValue;
    if (p.pre_out) {
        // pre-activation copy: written by the four-wave kernel's one-wave-per-SIMD epilogue (the
        // default policy's path for this GEMM); on any other path the GEMM writes pre and the
        // activation kernel forms out = act(pre)
        if (act == ACT_NONE || !out_bf16 || res || epi != EPI_PLAIN || p.grp || p.m_dev || p.ldo != p.N)
            return hipErrorInvalidValue;
        if (!pre_out_fused(p, act)) {
            GemmParams q = p0;
            q.out = p.pre_out;
            q.pre_out = nullptr;
            const hipError_t e = launch_gemm(q, ACT_NONE, true, s, epi);
            if (e != hipSuccess) return e;
            return launch_act(static_cast<bf16_t*>(p.out), p.pre_out, nullptr, (long)p.M * p.N, act, s);
        }
    }
    if (p.rhl && epi != EPI_LN_STATS_HL && epi != EPI_HL_F32) return hipErrorInvalidValue;
    if (epi == EPI_LN_STATS) {
        if (act != ACT_NONE || !res || out_bf16 || !p.xb || !p.stats_part) return hipErrorInvalidValue;
        return launch_epi<ACT_NONE, true, false, EPI_LN_STATS>(p, s);
    }
    if (epi == EPI_LN_STATS_HL) {
        if (act != ACT_NONE || !p.rhl || p.hl_plane <= 0 || !p.xb || !p.stats_part || p.grp) return hipErrorInvalidValue;
        return launch_epi<ACT_NONE, true, false, EPI_LN_STATS_HL>(p, s);
    }
    if (epi == EPI_HL_F32) {
        if (act != ACT_NONE || !p.rhl || p.hl_plane <= 0 || out_bf16 || p.grp) return hipErrorInvalidValue;
        return launch_epi<ACT_NONE, true, false, EPI_HL_F32>(p, s);
    }
    if (epi == EPI_LN_FOLD) {
        if (res || !out_bf16 || !p.fold_c || !p.fold_stats || !p.bias) return hipErrorInvalidValue;
        if (act == ACT_NONE) return launch_epi<ACT_NONE, false, true, EPI_LN_FOLD>(p, s);
        if (act == ACT_GELU) return launch_epi<ACT_GELU, false, true, EPI_LN_FOLD>(p, s);
        if (act == ACT_QGELU) return launch_epi<ACT_QGELU, false, true, EPI_LN_FOLD>(p, s);
        return hipErrorInvalidValue;
    }
#define CE_GEMM_CASE(A_, R_, O_) \
    if (act == A_ && res == R_ && out_bf16 == O_) return launch_t<A_, R_, O_>(p, s);
    CE_GEMM_CASE(ACT_NONE, false, true)
    CE_GEMM_CASE(ACT_NONE, false, false)
    CE_GEMM_CASE(ACT_NONE, true, true)
    CE_GEMM_CASE(ACT_NONE, true, false)
    CE_GEMM_CASE(ACT_GELU, false, true)
    CE_GEMM_CASE(ACT_QGELU, false, true)
    CE_GEMM_CASE(ACT_GELU, false, false)
    CE_GEMM_CASE(ACT_QGELU, false, false)
#undef CE_GEMM_CASE
    return hipErrorInvalidValue;
}

}  // namespace ce
