// SCHED 13 ("db"): persistent four-wave bf16 GEMM whose tile-t epilogue runs inside tile t+1's K-loop.
//
// One wave per SIMD (the four-wave persistent layout of gemm.hip's SCHED 11) cannot hide an epilogue
// behind another wave's MFMAs, and a 128 x 128 wave tile needs all 256 AGPRs, so SCHED 11 and the
// staged-residual kernel serialise every epilogue with the matrix pipe idle (c_fc: ~8 of ~32 us per
// tile; out-proj: ~19 of ~50 us).  Here a workgroup owns 256 x 128 tiles (waves 2 x 2 of
// 128 x 64: acc[8][4], 128 AGPRs) and keeps TWO accumulator sets: tile t accumulates into set t & 1
// while the set of tile t-1 is drained in 16 sub-chunks (fragment rows 2 (c >> 2) and 2 (c >> 2) + 1,
// column fragment c & 3), one per K-tile 0..15 of tile t, as micro-steps of a few VALU ops placed
// one per MFMA gap (sched_barrier-pinned) and ONE 16-B store per K-tile (v_permlane16_swap pairs the
// two rows) instead of a burst: beside the DMA pieces a store costs its issue, not its bytes (two
// 8-B stores per K-tile: 878 TF/s on c_fc-plain; the same without stores 1,284).
//  * LDS: a 3-stage ring of 48-KB stages (A 256 x 64, W 128 x 64 bf16; 128-B rows, 16-B chunk c of
//    row r at c ^ ((r >> 1) & 7)) + per wave two 1.5-KB side sets (bias, LN-fold column sums,
//    (mu, rstd) of the tile's rows: LDS-DMA'd during the tile's K-tile 0, read by the next tile).
//  * K-tile g: [set-0 MFMAs | set-1 reads | 6 DMA pieces of step g+2 | row 2 EP] -> wait for step
//    g+1 -> barrier -> [set-1 MFMAs | set-0 reads of step g+1 | 6 DMA pieces | row 2 EP + 1, store]: one
//    barrier per K-tile; step g+2 goes into the stage step g-1 used (free since the last barrier)
//    and every wait's vmcnt is exact, stores included (the first tile's sub-chunks store through a
//    0-row descriptor: dropped, still counted).
// bf16 output without residual (EPI_PLAIN / EPI_LN_FOLD, any activation); N % 128 == 0, K >= 1024.
// Built with -fno-slp-vectorize (Makefile): packed f32 VALU beside MFMAs costs more issue cycles
// than two scalar ops (MI355X_MICROARCH constants table).
#include "ce_device.h"
#include "ce_kernels.h"

#include <type_traits>
#include <utility>

namespace ce {
namespace {

constexpr int BM = 256, BK = 64;
using u32x2 = __attribute__((ext_vector_type(2))) unsigned int;
using u32x4 = __attribute__((ext_vector_type(4))) unsigned int;

__device__ __forceinline__ void barrier() {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

// buffer descriptor from wave-uniform inputs (readfirstlane: no waterfall loops)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_srd(const void* base, int nbytes) {
    const uint64_t b = reinterpret_cast<uint64_t>(base);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)b);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32));
    const int n = __builtin_amdgcn_readfirstlane(nbytes);
    return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(((uint64_t)hi << 32) | lo), (short)0, n,
                                             0x00020000);
}

// bijective XCD-aware remap (blocks b and b + 8 share an XCD) and the grouped tile order, as gemm.hip
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
    const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}
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

// compile-time loop: f(integral_constant<int, 0>) .. f(integral_constant<int, N - 1>)
template <typename F, int... I>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, I...>) {
    (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
    static_for_impl(f, std::make_integer_sequence<int, N>{});
}
constexpr int DB_BN = 128;
constexpr int DB_A_BYTES = BM * BK * 2;                 // 32 KB
constexpr int DB_STAGE = DB_A_BYTES + DB_BN * BK * 2;   // 48 KB
constexpr int DB_SIDE = 1536;                           // bias 256 B | fold_c 256 B | (mu, rstd) 1 KB

// V: timing variants (GEMM variant bits 14..17): bit 0 = no sched_barrier pinning of the
// micro-steps (the compiler schedules them; measured equal to the pinned form, no longer
// instantiated); bit 1 = no sub-chunks at all (ablation: no output); bit 2 = sub-chunks without
// their stores (ablation); bit 3 = stores through a 0-record descriptor (issued, dropped); bit 4 =
// non-temporal stores
template <int ACT, int EPI, int V = 0>
__global__ __launch_bounds__(256, 1) void gemm_db(GemmParams p) {
    constexpr bool FOLD = EPI == EPI_LN_FOLD;
    constexpr int NSIDE = FOLD ? 3 : 1;                 // side-fill DMAs per wave (K-tile 0)
    __shared__ __attribute__((aligned(16))) char smem[3 * DB_STAGE + 8 * DB_SIDE];
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave >> 1, wn = wave & 1;
    char* const side0 = smem + 3 * DB_STAGE + wave * 2 * DB_SIDE;
    const int tiles_m = (p.M + BM - 1) / BM, tiles_n = p.N / DB_BN;
    const int nwg = tiles_m * tiles_n, grid = gridDim.x;
    const int slot = xcd_remap(blockIdx.x, grid);
    const int nk = p.K / BK;
    const int my_tiles = slot < nwg ? (nwg - 1 - slot) / grid + 1 : 0;
    if (my_tiles == 0) return;                          // the whole workgroup
    const int nsteps = my_tiles * nk;

    const int srow = wave * 8 + (lane >> 3);
    const int schunk = (lane & 7) ^ ((srow >> 1) & 7);
    const int voffA = srow * (int)p.lda * 2 + schunk * 16;
    const int voffW = srow * (int)p.ldw * 2 + schunk * 16;
    const int jstrA = 32 * (int)p.lda * 2, jstrW = 32 * (int)p.ldw * 2;
    auto tile_mn = [&](int t, int& mm, int& nn) {
        int tm, tn;
        tile_of(min(slot + t * grid, nwg - 1), tiles_m, tiles_n, p.gm, tm, tn);
        mm = tm * BM;
        nn = tn * DB_BN;
    };
    // DMA stream state: K-tile dk of this workgroup's tile dt
    int dt = 0, dk = 0;
    __amdgpu_buffer_rsrc_t srdA, srdW;
    auto set_srd = [&](int t) {
        int mm, nn;
        tile_mn(t, mm, nn);
        srdA = make_srd(p.A + (size_t)mm * p.lda, max(0, min(p.M - mm, BM)) * (int)p.lda * 2);
        srdW = make_srd(p.W + (size_t)nn * p.ldw, DB_BN * (int)p.ldw * 2);
    };
    set_srd(0);
    // DMA j of the current step into stage stg (j < 8: A rows 32j + srow; else W rows 32(j-8) + srow);
    // past the last step the offset lies beyond the descriptor (zeros, still counted by vmcnt)
    auto dma = [&](int stg, int j, bool live) {
        const int kb = live ? dk * BK * 2 : 0x7ffff000;
        int sbase = stg * DB_STAGE;
        int jo = (j < 8 ? j : j - 8) * (j < 8 ? jstrA : jstrW);
        asm volatile("" : "+s"(jo), "+s"(sbase));
        char* base = smem + sbase;
        if (j < 8)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(srdA, (CE_LDS void*)(base + (j * 32 + wave * 8) * 128), 16,
                                                     voffA + jo, kb, 0, 0);
        else
            __builtin_amdgcn_raw_ptr_buffer_load_lds(srdW, (CE_LDS void*)(base + DB_A_BYTES + ((j - 8) * 32 + wave * 8) * 128),
                                                     16, voffW + jo, kb, 0, 0);
    };
    auto advance = [&] {
        if (++dk == nk) {
            dk = 0;
            ++dt;
            set_srd(dt);
        }
    };
    // side set s <- tile t's bias (64 columns), fold_c, (mu, rstd) of its 128 rows (this wave's)
    auto side_fill = [&](int t, int s) {
        int mm, nn;
        tile_mn(t, mm, nn);
        int so = s * DB_SIDE;
        asm volatile("" : "+s"(so));
        char* sd = side0 + so;
        const __amdgpu_buffer_rsrc_t bsrd = make_srd(p.bias ? (const void*)p.bias : (const void*)p.A, p.bias ? p.N * 4 : 0);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(bsrd, (CE_LDS void*)sd, 4, (nn + wn * 64 + lane) * 4, 0, 0, 0);
        if constexpr (FOLD) {
            const __amdgpu_buffer_rsrc_t csrd = make_srd(p.fold_c, p.N * 4);
            const __amdgpu_buffer_rsrc_t ssrd = make_srd(p.fold_stats, p.M * 8);
            __builtin_amdgcn_raw_ptr_buffer_load_lds(csrd, (CE_LDS void*)(sd + 256), 4, (nn + wn * 64 + lane) * 4, 0, 0, 0);
            __builtin_amdgcn_raw_ptr_buffer_load_lds(ssrd, (CE_LDS void*)(sd + 512), 16, (mm + wm * 128 + lane * 2) * 8, 0,
                                                     0, 0);
        }
    };

    const int fr = lane & 15, fq = lane >> 4;
    const int fo0 = fr * 128 + (((0 + fq) ^ (fr >> 1)) << 4);
    const int fo1 = fr * 128 + (((4 + fq) ^ (fr >> 1)) << 4);
    const int a_off = wm * 128 * 128;
    const int w_off = DB_A_BYTES + wn * 64 * 128;

    f32x4 accA[8][4], accB[8][4];
    bf16x8 a0[8], b0[4], a1[8], b1[4];
    // prologue: steps 0 and 1 in flight, set 0 of step 0
#pragma unroll
    for (int s = 0; s < 2; ++s) {
#pragma unroll
        for (int j = 0; j < 12; ++j) dma(s, j, s < nsteps);
        advance();
    }
    asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
    barrier();
#pragma unroll
    for (int q = 0; q < 8; ++q) a0[q] = *reinterpret_cast<const bf16x8*>(smem + a_off + q * 16 * 128 + fo0);
#pragma unroll
    for (int q = 0; q < 4; ++q) b0[q] = *reinterpret_cast<const bf16x8*>(smem + w_off + q * 16 * 128 + fo0);

#define CE_MFMA_AGPR(ACC, BV, AV) \
    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(ACC) : "v"(BV), "v"(AV))
#define CE_MFMA_AGPR0(ACC, BV, AV) \
    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=a"(ACC) : "v"(BV), "v"(AV))

    int g = 0, st = 0;                                  // global K-step, its stage (g % 3)
    // epilogue of one fragment (i, jj) of a drained set: value, store
    auto epi_value = [&](f32x4 v, const float4& b, const float4& c, const float2& s) __attribute__((always_inline)) {
        if constexpr (FOLD) {
            v[0] = fmaf(s.y, fmaf(-s.x, c.x, v[0]), b.x);
            v[1] = fmaf(s.y, fmaf(-s.x, c.y, v[1]), b.y);
            v[2] = fmaf(s.y, fmaf(-s.x, c.z, v[2]), b.z);
            v[3] = fmaf(s.y, fmaf(-s.x, c.w, v[3]), b.w);
        } else {
            v[0] += b.x; v[1] += b.y; v[2] += b.z; v[3] += b.w;
        }
        if constexpr (ACT == ACT_GELU) {
            v = gelu_fast4(v);
        } else {
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = apply_act<ACT>(v[e]);
        }
        return v;
    };

    // one tile: accumulate into set PAR, drain set PAR ^ 1 (the previous tile, t > 0)
    auto run_tile = [&](auto parc, int t) __attribute__((always_inline)) {
        constexpr int PAR = decltype(parc)::value;
        f32x4 (&accC)[8][4] = PAR ? accB : accA;
        f32x4 (&accP)[8][4] = PAR ? accA : accB;
        int pm = 0, pn = 0;
        if (t > 0) tile_mn(t - 1, pm, pn);
        const int pmb = pm + wm * 128, pnb = pn + wn * 64;
        const int prow = t > 0 ? max(0, min(p.M - pmb, 128)) : 0;
        const __amdgpu_buffer_rsrc_t osrd = make_srd(static_cast<bf16_t*>(p.out) + (size_t)pmb * p.ldo, prow * (int)p.ldo * 2);
        int pso = (PAR ^ 1) * DB_SIDE;
        asm volatile("" : "+s"(pso));
        const char* psd = side0 + pso;
        // this lane's store offset: row fr + 16 (fq & 1) of a fragment-row pair, columns 8 (fq >> 1) ..
        const int ovo = ((fr + (fq & 1) * 16) * (int)p.ldo + pnb + (fq >> 1) * 8) * 2;

        auto ktile = [&](auto kc) __attribute__((always_inline)) {
            // KT 0..15: K-tile KT of the tile, carrying sub-chunk KT of the previous tile; -1: K-tile 16
            // (no sub-chunk; stores of K-tiles 14, 15 still younger than the awaited step); -2: later
            constexpr int KT = decltype(kc)::value;
            constexpr bool SUB = KT >= 0 && (V & 2) == 0;
            constexpr bool PIN = SUB && (V & 1) == 0;
            int bo = st * DB_STAGE;
            asm volatile("" : "+s"(bo));
            const char* sb = smem + bo;
            const int st1 = st == 2 ? 0 : st + 1;
            int bn = st1 * DB_STAGE;
            asm volatile("" : "+s"(bn));
            const char* sn = smem + bn;
            const int st2 = st == 0 ? 2 : st - 1;               // (g + 2) % 3
            const bool live = g + 2 < nsteps;
            // sub-chunk KT: fragment rows 2 EP (first half) and 2 EP + 1 (second half), column EJ,
            // each as 18 micro-steps of <= 4 VALU ops placed one per MFMA (sched_barrier-pinned):
            // one wave per SIMD issues them in the shadow of its own MFMAs
            constexpr int EP = SUB ? (KT >> 2) : 0;          // fragment rows 2 EP (first half), 2 EP + 1
            constexpr int EJ = SUB ? (KT & 3) : 0;           // column fragment
            float4 ebv[1], ecv[1];
            float2 esv[2];
            f32x4 ex[2], eu[2], ew[2], ez[2], ed[2];
            float eq0[2], eq1[2];
            u32x2 eo[2];
            auto estep = [&](auto kk, auto hh) __attribute__((always_inline)) {
                constexpr int K = decltype(kk)::value, H = decltype(hh)::value;
                constexpr bool GL = ACT == ACT_GELU;
                f32x4& x = ex[H];
                if constexpr (K == 0) {
                    x = accP[2 * EP + H][EJ];
                } else if constexpr (K == 1) {
                    if constexpr (FOLD) {
                        const float c[4] = {ecv[0].x, ecv[0].y, ecv[0].z, ecv[0].w};
#pragma unroll
                        for (int e = 0; e < 4; ++e) x[e] = fmaf(-esv[H].x, c[e], x[e]);
                    } else {
                        const float b[4] = {ebv[0].x, ebv[0].y, ebv[0].z, ebv[0].w};
#pragma unroll
                        for (int e = 0; e < 4; ++e) x[e] += b[e];
                    }
                } else if constexpr (K == 2) {
                    if constexpr (FOLD) {
                        const float b[4] = {ebv[0].x, ebv[0].y, ebv[0].z, ebv[0].w};
#pragma unroll
                        for (int e = 0; e < 4; ++e) x[e] = fmaf(esv[H].y, x[e], b[e]);
                    }
                    if constexpr (!GL && ACT != ACT_NONE) {
#pragma unroll
                        for (int e = 0; e < 4; ++e) x[e] = apply_act<ACT>(x[e]);
                    }
                } else if constexpr (GL && K == 3) {
                    eu[H][0] = __builtin_amdgcn_fmed3f(x[0], -CE_GELU_CLAMP, CE_GELU_CLAMP);
                    eu[H][1] = __builtin_amdgcn_fmed3f(x[1], -CE_GELU_CLAMP, CE_GELU_CLAMP);
                } else if constexpr (GL && K == 4) {
                    eu[H][2] = __builtin_amdgcn_fmed3f(x[2], -CE_GELU_CLAMP, CE_GELU_CLAMP);
                    eu[H][3] = __builtin_amdgcn_fmed3f(x[3], -CE_GELU_CLAMP, CE_GELU_CLAMP);
                } else if constexpr (GL && K == 5) {
#pragma unroll
                    for (int e = 0; e < 4; ++e) ew[H][e] = eu[H][e] * eu[H][e];
                } else if constexpr (GL && K == 6) {
#pragma unroll
                    for (int e = 0; e < 4; ++e) ez[H][e] = fmaf(ew[H][e], CE_GELU_C2, CE_GELU_C1);
                } else if constexpr (GL && K == 7) {
#pragma unroll
                    for (int e = 0; e < 4; ++e) ez[H][e] = fmaf(ez[H][e], ew[H][e], CE_GELU_C0);
                } else if constexpr (GL && K == 8) {
#pragma unroll
                    for (int e = 0; e < 4; ++e) ez[H][e] = eu[H][e] * ez[H][e];
                } else if constexpr (GL && K == 9) {
                    ed[H][0] = __builtin_amdgcn_exp2f(ez[H][0]);
                    ed[H][1] = __builtin_amdgcn_exp2f(ez[H][1]);
                } else if constexpr (GL && K == 10) {
                    ed[H][2] = __builtin_amdgcn_exp2f(ez[H][2]);
                    ed[H][3] = __builtin_amdgcn_exp2f(ez[H][3]);
                } else if constexpr (GL && K == 11) {
#pragma unroll
                    for (int e = 0; e < 4; ++e) ed[H][e] += 1.0f;
                } else if constexpr (GL && K == 12) {
                    eq0[H] = ed[H][0] * ed[H][1];
                    eq1[H] = ed[H][2] * ed[H][3];
                } else if constexpr (GL && K == 13) {
                    eq0[H] = __builtin_amdgcn_rcpf(eq0[H]);
                    eq1[H] = __builtin_amdgcn_rcpf(eq1[H]);
                } else if constexpr (GL && K == 14) {
                    const f32x4 inv = {ed[H][1] * eq0[H], ed[H][0] * eq0[H], ed[H][3] * eq1[H], ed[H][2] * eq1[H]};
                    ew[H] = inv;
                } else if constexpr (GL && K == 15) {
#pragma unroll
                    for (int e = 0; e < 4; ++e) x[e] *= ew[H][e];
                } else if constexpr (K == 16) {
                    eo[H] = u32x2{pack_bf2(x[0], x[1]), pack_bf2(x[2], x[3])};
                } else if constexpr (K == 17 && H == 1) {
                    // rows 2 EP and 2 EP + 1 paired by v_permlane16_swap: each lane stores 8 columns of
                    // one row (16 B), one store instruction per sub-chunk (a wave's store issue is
                    // the cost beside the DMAs, not its bytes); row / column step in soffset
                    const auto px = __builtin_amdgcn_permlane16_swap(eo[0][0], eo[1][0], false, false);
                    const auto py = __builtin_amdgcn_permlane16_swap(eo[0][1], eo[1][1], false, false);
                    const u32x4 d = {px[0], py[0], px[1], py[1]};
                    int so = 32 * EP * (int)p.ldo * 2 + 32 * EJ;
                    asm volatile("" : "+s"(so));
                    // (timing variants: V bit 3 stores through a 0-record descriptor, dropped after issue;
                    // V bit 4 stores with the non-temporal policy)
                    if constexpr ((V & 4) == 0 && (V & 8) == 0 && (V & 16) == 0)
                        __builtin_amdgcn_raw_buffer_store_b128(d, osrd, ovo, so, 0);
                    else if constexpr ((V & 8) != 0)
                        __builtin_amdgcn_raw_buffer_store_b128(d, make_srd(p.out, 0), ovo, so, 0);
                    else if constexpr ((V & 16) != 0)
                        __builtin_amdgcn_raw_buffer_store_b128(d, osrd, ovo, so, 2);
                }
            };
            // ---- first half: set-0 MFMAs, set-1 reads, column fragment EJ of the sub-chunk ----
            static_for<32>([&](auto sc) __attribute__((always_inline)) {
                constexpr int s2 = decltype(sc)::value;
                constexpr int i = s2 >> 2, j = s2 & 3;
                if constexpr (PIN) __builtin_amdgcn_sched_barrier(0);
                if constexpr (KT == 0) CE_MFMA_AGPR0(accC[i][j], b0[j], a0[i]);
                else CE_MFMA_AGPR(accC[i][j], b0[j], a0[i]);
                if constexpr (s2 & 1) {
                    constexpr int q = s2 >> 1;
                    if constexpr (q < 4) b1[q] = *reinterpret_cast<const bf16x8*>(sb + w_off + q * 16 * 128 + fo1);
                    else if constexpr (q < 12) a1[q - 4] = *reinterpret_cast<const bf16x8*>(sb + a_off + (q - 4) * 16 * 128 + fo1);
                }
                // DMA pieces 0..5 of step g+2 (into the stage step g-1 used: free since the last barrier)
                if constexpr (s2 % 5 == 2 && s2 / 5 < 6) dma(st2, s2 / 5, live);
                if constexpr (KT == 0 && s2 == 30) side_fill(t, PAR);
                if constexpr (SUB) {
                    if (s2 == 0) {
                        // side reads by inline asm: a plain LDS read here gets an s_waitcnt vmcnt(0)
                        // (hipcc cannot tell the side set from the stages the DMAs in flight write),
                        // which would drain every store and DMA; retired by the lgkmcnt(2) at slot 3
                        const unsigned cb = (unsigned)(uintptr_t)(CE_LDS const void*)psd + (4 * fq) * 4;
                        asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(ebv[0]) : "v"(cb), "n"(64 * EJ));
                        if constexpr (FOLD) {
                            const unsigned sa = (unsigned)(uintptr_t)(CE_LDS const void*)psd + fr * 8;
                            asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(ecv[0]) : "v"(cb), "n"(256 + 64 * EJ));
                            asm volatile("ds_read_b64 %0, %1 offset:%2" : "=v"(esv[0]) : "v"(sa), "n"(512 + 256 * EP));
                            asm volatile("ds_read_b64 %0, %1 offset:%2" : "=v"(esv[1]) : "v"(sa), "n"(512 + 256 * EP + 128));
                        }
                    }
                    // the side reads are older than the set-1 reads of slots 1 and 3
                    if (s2 == 3) asm volatile("s_waitcnt lgkmcnt(2)" ::: "memory");
                    if constexpr (s2 >= 2 && s2 <= 18)
                        estep(std::integral_constant<int, s2 - 2>{}, std::integral_constant<int, 0>{});
                }
            });
            if constexpr (PIN) __builtin_amdgcn_sched_barrier(0);
            // step g+1 landed (its last pieces were issued in K-tile g-1's second half).  Younger: the
            // second-half store of K-tile g-1, step g+2's first 6 pieces, the side fill of K-tile 0 and
            // the first-half store of K-tile g (the fewest possible assumed where the tile boundary
            // leaves it open: a longer wait, never a short one)
            {
                // C1 / C2: stores of a sub-chunk in its first / second half
                constexpr int C1 = 0, C2 = (V & 6) ? 0 : 1;
                constexpr int CNT = 6 + (KT == 0 ? NSIDE : 0) + (KT >= 1 || KT == -1 ? C2 : 0) + (KT >= 0 ? C1 : 0);
                asm volatile("s_waitcnt vmcnt(%0)" :: "n"(CNT) : "memory");
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            barrier();
            // ---- second half: set-1 MFMAs, set-0 reads of step g+1, DMA pieces 6..11 of step g+2,
            // column fragment EJ + 1 of the sub-chunk (stored after the DMAs) ----
            static_for<32>([&](auto sc) __attribute__((always_inline)) {
                constexpr int s2 = decltype(sc)::value;
                constexpr int i = s2 >> 2, j = s2 & 3;
                if constexpr (PIN) __builtin_amdgcn_sched_barrier(0);
                CE_MFMA_AGPR(accC[i][j], b1[j], a1[i]);
                if constexpr (s2 % 5 == 2 && s2 / 5 < 6) dma(st2, 6 + s2 / 5, live);
                if constexpr (s2 & 1) {
                    constexpr int q = s2 >> 1;
                    if constexpr (q < 4) b0[q] = *reinterpret_cast<const bf16x8*>(sn + w_off + q * 16 * 128 + fo0);
                    else if constexpr (q < 12) a0[q - 4] = *reinterpret_cast<const bf16x8*>(sn + a_off + (q - 4) * 16 * 128 + fo0);
                }
                if constexpr (SUB) {
                    if constexpr (s2 <= 16) estep(std::integral_constant<int, s2>{}, std::integral_constant<int, 1>{});
                    if constexpr (s2 == 31) estep(std::integral_constant<int, 17>{}, std::integral_constant<int, 1>{});
                }
            });
            if constexpr (PIN) __builtin_amdgcn_sched_barrier(0);
            advance();
            ++g;
            st = st1;
        };
        ktile(std::integral_constant<int, 0>{});
        ktile(std::integral_constant<int, 1>{});
        ktile(std::integral_constant<int, 2>{});
        ktile(std::integral_constant<int, 3>{});
        ktile(std::integral_constant<int, 4>{});
        ktile(std::integral_constant<int, 5>{});
        ktile(std::integral_constant<int, 6>{});
        ktile(std::integral_constant<int, 7>{});
        ktile(std::integral_constant<int, 8>{});
        ktile(std::integral_constant<int, 9>{});
        ktile(std::integral_constant<int, 10>{});
        ktile(std::integral_constant<int, 11>{});
        ktile(std::integral_constant<int, 12>{});
        ktile(std::integral_constant<int, 13>{});
        ktile(std::integral_constant<int, 14>{});
        ktile(std::integral_constant<int, 15>{});
        if (nk > 16) ktile(std::integral_constant<int, -1>{});
        for (int kt = 17; kt < nk; ++kt) ktile(std::integral_constant<int, -2>{});
    };
    // the last tile's set, drained after the loop (all 16 sub-chunks, no MFMAs beside them)
    auto drain = [&](auto parc, int t) __attribute__((always_inline)) {
        constexpr int PAR = decltype(parc)::value;
        f32x4 (&acc)[8][4] = PAR ? accB : accA;
        int pm, pn;
        tile_mn(t, pm, pn);
        const int pmb = pm + wm * 128, pnb = pn + wn * 64;
        const int prow = max(0, min(p.M - pmb, 128));
        const __amdgpu_buffer_rsrc_t osrd = make_srd(static_cast<bf16_t*>(p.out) + (size_t)pmb * p.ldo, prow * (int)p.ldo * 2);
        const char* psd = side0 + PAR * DB_SIDE;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");      // the side fill landed
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) {
                const float4 b = *reinterpret_cast<const float4*>(psd + (16 * jj + 4 * fq) * 4);
                float4 c = make_float4(0.f, 0.f, 0.f, 0.f);
                float2 s = make_float2(0.f, 0.f);
                if constexpr (FOLD) {
                    c = *reinterpret_cast<const float4*>(psd + 256 + (16 * jj + 4 * fq) * 4);
                    s = *reinterpret_cast<const float2*>(psd + 512 + (16 * i + fr) * 8);
                }
                const f32x4 v = epi_value(acc[i][jj], b, c, s);
                const u32x2 o = {pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3])};
                __builtin_amdgcn_raw_buffer_store_b64(o, osrd, (16 * i + fr) * (int)p.ldo * 2 + (pnb + 16 * jj + 4 * fq) * 2, 0, 0);
            }
    };
    for (int t = 0; t < my_tiles; t += 2) {
        run_tile(std::integral_constant<int, 0>{}, t);
        if (t + 1 < my_tiles) run_tile(std::integral_constant<int, 1>{}, t + 1);
    }
    if ((my_tiles - 1) & 1) drain(std::integral_constant<int, 1>{}, my_tiles - 1);
    else drain(std::integral_constant<int, 0>{}, my_tiles - 1);
#undef CE_MFMA_AGPR0
#undef CE_MFMA_AGPR
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
}


}  // namespace

hipError_t launch_gemm_db(const GemmParams& p, int act, int epi, int grid, hipStream_t s) {
    const dim3 g((unsigned)grid), b(256);
    const int v = ((p.variant >> 14) & 31);
#define CE_DB(A_, E_) \
    if (act == A_ && epi == E_) { \
        if (v == 2) hipLaunchKernelGGL((gemm_db<A_, E_, 2>), g, b, 0, s, p); \
        else if (v == 4) hipLaunchKernelGGL((gemm_db<A_, E_, 4>), g, b, 0, s, p); \
        else if (v == 8) hipLaunchKernelGGL((gemm_db<A_, E_, 8>), g, b, 0, s, p); \
        else if (v == 16) hipLaunchKernelGGL((gemm_db<A_, E_, 16>), g, b, 0, s, p); \
        else hipLaunchKernelGGL((gemm_db<A_, E_>), g, b, 0, s, p); \
        return hipGetLastError(); }
    CE_DB(ACT_NONE, EPI_PLAIN) CE_DB(ACT_GELU, EPI_PLAIN) CE_DB(ACT_QGELU, EPI_PLAIN)
    CE_DB(ACT_NONE, EPI_LN_FOLD) CE_DB(ACT_GELU, EPI_LN_FOLD) CE_DB(ACT_QGELU, EPI_LN_FOLD)
#undef CE_DB
    return hipErrorInvalidValue;
}

}  // namespace ce
