// SCHED 14 ("w2b"): bf16 GEMM with TWO independent 256-thread workgroups per CU, so one workgroup's
// epilogue, barrier waits and LDS-DMA issue stalls run beside the other workgroup's MFMAs.
//
// Why: the four-wave persistent kernels (SCHED 11, the staged-residual kernel) hold
// all 512 registers of a SIMD in one wave (128 x 128 accumulators), so every epilogue runs with the
// matrix pipe idle (c_fc ~8 of ~32 us per tile, out-proj ~19 of ~50) and every LDS-DMA issue stall
// (~60 cycles per 1-KB piece beside MFMAs, 16 pieces per 64-deep K-tile) is paid by the only wave the
// SIMD has.  Here each wave owns 128 x 64 outputs (acc[8][4] of v_mfma_f32_16x16x32_bf16, 128 AGPRs,
// <= 256 registers), a workgroup a 256 x 128 tile, and two workgroups share each CU's SIMDs with
// independent barriers and vmcnt counters: the hardware interleaves them, nothing in the code pairs
// their phases.  The price is the smaller tile: 1.5x the operand bytes per MFMA of a 256 x 256 tile
// (48 B/clk per CU at the full MFMA rate, inside the L2's ~56-64).
//
//  * LDS per workgroup: a 3-slot ring of K-steps of 32 (A 256 x 64 B + W 128 x 64 B = 24 KB), 72 KB;
//    two workgroups fit a CU.  64-B rows, 16-B chunk c of row r at c ^ 2((r >> 3) & 1): conflict-free
//    for the four 16-lane groups of ds_read_b128 (tools/lds_bank_sim.py); the DMA source carries the
//    inverse permutation.
//  * K-step t: vmcnt(6) (step t+1's 6 pieces stay in flight) -> barrier -> the 6 pieces of step t+2
//    (into the slot step t-1 used, free once every wave passed the barrier) spread over the first
//    MFMA rows -> 12 fragment reads by inline asm with counted lgkmcnt (W fragments double-buffered
//    by step parity, A fragments in a 3-deep ring two rows ahead) -> 32 asm MFMAs into AGPRs.  One
//    barrier per step; no store or load in the loop besides the DMA pieces, so every wait is exact.
//  * One tile per workgroup (grid = tiles, XCD-aware remap + grouped tile order as gemm.hip): an
//    exiting workgroup's stores drain while the CU's other workgroup computes, and a new one's
//    prologue overlaps it too.
//  * Epilogue operands (bias, LN-fold column sums, row (mu, rstd)) are loaded into registers after
//    the K-loop (loading them during the last K-step spilled); bf16 output rows paired by v_permlane16_swap into 16-B stores through a buffer
//    descriptor clipped at row M (rows past M dropped).
// Supported: bf16 output without residual, EPI_PLAIN / EPI_LN_FOLD, any activation; or EPI_LN_STATS_HL
// (hi/lo residual planes in and out + 64-column slab statistics: out-proj / c_proj); N % 128 == 0,
// K % 32 == 0, K >= 64; grp == 0; no pre-activation copy.  (launch_gemm_w2b checks.)
#include "ce_device.h"
#include "ce_kernels.h"

#include <type_traits>
#include <utility>

namespace ce {
namespace {

constexpr int TM = 256, TN = 128, KS = 32;
constexpr int A_BYTES = TM * KS * 2;                 // 16 KB
constexpr int SLOT = (TM + TN) * KS * 2;             // 24 KB
constexpr int NSLOT = 3;

using u32x4 = __attribute__((ext_vector_type(4))) unsigned int;

__device__ __forceinline__ void barrier() {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_srd(const void* base, int nbytes) {
    const uint64_t b = reinterpret_cast<uint64_t>(base);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)b);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32));
    const int n = __builtin_amdgcn_readfirstlane(nbytes);
    return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(((uint64_t)hi << 32) | lo), (short)0, n,
                                             0x00020000);
}

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

template <typename F, int... I>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, I...>) {
    (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
    static_for_impl(f, std::make_integer_sequence<int, N>{});
}

// Sum over the four 16-lane groups of a wave (lanes l, l ^ 16, l ^ 32, l ^ 48) by two lane-swap pairs
__device__ __forceinline__ float sum_lane_groups(float v) {
    const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    const float s = __uint_as_float(a[0]) + __uint_as_float(a[1]);
    const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(s), __float_as_uint(s), false, false);
    return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}

// EPI_LN_STATS_HL (out-proj / c_proj of the folded towers): v = acc + bias + (hi + lo) of the residual
// planes; hi' = bf16(v), lo' = bf16(v - hi') into the xb planes; per row the (mean, M2) of its 64
// columns = one slab (a wave's 64 columns are exactly slab nbase / 64).  The residual of a row pair
// (2ip, 2ip + 1) is loaded in the store layout (16 B = 8 columns of one row per lane) one pair ahead,
// and turned into fragments by the stores' own v_permlane16_swap pairing (an involution).
using u32x2 = __attribute__((ext_vector_type(2))) unsigned int;
__device__ __forceinline__ void hl_epilogue(const GemmParams& p, const f32x4 (&acc)[8][4], const float4 (&bv)[4],
                                            int mbase, int nbase, int rows, int fr, int fq) {
    const int ldr = (int)p.ldr, ldo = (int)p.ldo;
    const __amdgpu_buffer_rsrc_t hs = make_srd(p.rhl + (size_t)mbase * ldr, rows * ldr * 2);
    const __amdgpu_buffer_rsrc_t ls = make_srd(p.rhl + p.hl_plane + (size_t)mbase * ldr, rows * ldr * 2);
    const __amdgpu_buffer_rsrc_t xs = make_srd(p.xb + (size_t)mbase * ldo, rows * ldo * 2);
    const __amdgpu_buffer_rsrc_t xl = make_srd(p.xb + p.hl_plane + (size_t)mbase * ldo, rows * ldo * 2);
    const int rp = ((fr + (fq & 1) * 16) * ldr + nbase + (fq >> 1) * 8) * 2;
    const int xp = ((fr + (fq & 1) * 16) * ldo + nbase + (fq >> 1) * 8) * 2;
    u32x4 rh[2][4], rl[2][4];
    auto load = [&](int ip, u32x4 (&h)[4], u32x4 (&l)[4]) __attribute__((always_inline)) {
        int io = ip * 32 * ldr * 2;
        asm volatile("" : "+s"(io));
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            h[j] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(hs, rp + io + j * 32, 0, 0));
            l[j] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(ls, rp + io + j * 32, 0, 0));
        }
    };
    float2 sta = make_float2(0.f, 0.f), stb = make_float2(0.f, 0.f);
    load(0, rh[0], rl[0]);
#pragma unroll
    for (int ip = 0; ip < 4; ++ip) {
        if (ip + 1 < 4) load(ip + 1, rh[(ip + 1) & 1], rl[(ip + 1) & 1]);
        float lmean[2], lm2[2];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const u32x4 dh = rh[ip & 1][j], dl = rl[ip & 1][j];
            const auto hx = __builtin_amdgcn_permlane16_swap(dh[0], dh[2], false, false);
            const auto hy = __builtin_amdgcn_permlane16_swap(dh[1], dh[3], false, false);
            const auto lx = __builtin_amdgcn_permlane16_swap(dl[0], dl[2], false, false);
            const auto ly = __builtin_amdgcn_permlane16_swap(dl[1], dl[3], false, false);
            uint2 h[2], l[2];
#pragma unroll
            for (int r2 = 0; r2 < 2; ++r2) {
                const float2 a = join_hl(hx[r2], lx[r2]), b = join_hl(hy[r2], ly[r2]);
                f32x4 v = acc[2 * ip + r2][j];
                const float4 bb = bv[j];
                v[0] += bb.x + a.x; v[1] += bb.y + a.y; v[2] += bb.z + b.x; v[3] += bb.w + b.y;
                // (mean, M2) of the lane's 4 values, merged over the slab's 4 fragments (Chan)
                const float m4 = ((v[0] + v[1]) + (v[2] + v[3])) * 0.25f;
                const float d0 = v[0] - m4, d1 = v[1] - m4, d2 = v[2] - m4, d3 = v[3] - m4;
                const float q4 = fmaf(d0, d0, fmaf(d1, d1, fmaf(d2, d2, d3 * d3)));
                if (j == 0) {
                    lmean[r2] = m4;
                    lm2[r2] = q4;
                } else {
                    const float dm = m4 - lmean[r2];
                    lmean[r2] = fmaf(dm, 1.0f / (j + 1), lmean[r2]);
                    lm2[r2] += fmaf(dm * dm, 4.0f * j / (j + 1), q4);
                }
                split_hl(v[0], v[1], h[r2].x, l[r2].x);
                split_hl(v[2], v[3], h[r2].y, l[r2].y);
            }
            const auto x = __builtin_amdgcn_permlane16_swap(h[0].x, h[1].x, false, false);
            const auto y = __builtin_amdgcn_permlane16_swap(h[0].y, h[1].y, false, false);
            const auto xx = __builtin_amdgcn_permlane16_swap(l[0].x, l[1].x, false, false);
            const auto yy = __builtin_amdgcn_permlane16_swap(l[0].y, l[1].y, false, false);
            const u32x4 oh = {x[0], y[0], x[1], y[1]};
            const u32x4 ol = {xx[0], yy[0], xx[1], yy[1]};
            __builtin_amdgcn_raw_buffer_store_b128(oh, xs, xp + ip * 32 * ldo * 2 + j * 32, 0, 0);
            __builtin_amdgcn_raw_buffer_store_b128(ol, xl, xp + ip * 32 * ldo * 2 + j * 32, 0, 0);
        }
        // the row's 64-column (mean, M2): the 4 lane groups' 16-value summaries combined
#pragma unroll
        for (int r2 = 0; r2 < 2; ++r2) {
            const int i = 2 * ip + r2;
            const float mean = sum_lane_groups(lmean[r2]) * 0.25f;
            const float dm = lmean[r2] - mean;
            const float q = sum_lane_groups(fmaf(dm * dm, 16.0f, lm2[r2]));
            if (fq == (i & 3)) {
                if (i < 4) sta = make_float2(mean, q);
                else stb = make_float2(mean, q);
            }
        }
    }
    // lane (fr, fq) holds rows 16 fq + fr (sta) and 16 fq + fr + 64 (stb); clipped at row M
    const int ns = p.N / 64;
    const __amdgpu_buffer_rsrc_t ss = make_srd(p.stats_part + (size_t)mbase * ns, rows * ns * 8);
    const int so = ((fq * 16 + fr) * ns + nbase / 64) * 8;
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, sta), ss, so, 0, 0);
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, stb), ss, so + 64 * ns * 8, 0, 0);
}

template <int ACT>
__device__ __forceinline__ f32x4 act4(f32x4 v) {
    if constexpr (ACT == ACT_GELU) return gelu_fast4(v);
    else {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = apply_act<ACT>(v[e]);
        return v;
    }
}

// VAR (A/B, GemmParams::variant bits 22-23): 1 = "block" steps: all 12 fragment reads and the 6 DMA
// pieces right after the barrier, one lgkmcnt(0), then 32 back-to-back MFMAs (a load segment and a
// compute segment per step, for the CU's other workgroup to interleave with); 2 = s_setprio 1 over the
// MFMA segment.
template <int ACT, int EPI, int VAR = 0>
__global__ __launch_bounds__(256, 2) void gemm_w2b(GemmParams p) {
    constexpr bool BLOCK = (VAR & 1) != 0;
    constexpr bool PRIO = (VAR & 2) != 0;
    __shared__ __attribute__((aligned(16))) char smem[NSLOT * SLOT];
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave >> 1, wn = wave & 1;
    const int tiles_m = (p.M + TM - 1) / TM;
    const int tiles_n = p.N / TN;
    const int nwg = tiles_m * tiles_n;
    int tm, tn;
    tile_of(xcd_remap(blockIdx.x, nwg), tiles_m, tiles_n, p.gm, tm, tn);
    const int m0 = tm * TM, n0 = tn * TN;
    const int nk = p.K / KS;

    // ---- staging: piece j (0..5) of wave w moves 16 rows x 64 B: j < 4 A rows 16(4j + w) + (lane >> 2),
    // else W rows 16(4(j - 4) + w) + (lane >> 2); LDS chunk lane & 3 holds source chunk (lane & 3) ^ f(row)
    const int srow = lane >> 2;
    const int schunk = (lane & 3) ^ (((lane >> 5) & 1) << 1);
    const __amdgpu_buffer_rsrc_t srdA = make_srd(p.A + (size_t)m0 * p.lda, max(0, min(p.M - m0, TM)) * (int)p.lda * 2);
    const __amdgpu_buffer_rsrc_t srdW = make_srd(p.W + (size_t)n0 * p.ldw, TN * (int)p.ldw * 2);
    const int voffA = srow * (int)p.lda * 2 + schunk * 16;
    const int voffW = srow * (int)p.ldw * 2 + schunk * 16;
    const int gstrA = 64 * (int)p.lda * 2, gstrW = 64 * (int)p.ldw * 2;     // 4 groups of 16 rows
    auto piece = [&](int kt, int j) __attribute__((always_inline)) {
        char* base = smem + (kt % NSLOT) * SLOT;
        const int kb = kt * KS * 2;
        if (j < 4) {
            int go = j * gstrA;
            asm volatile("" : "+s"(go));
            __builtin_amdgcn_raw_ptr_buffer_load_lds(srdA, (CE_LDS void*)(base + (16 * j + 4 * wave) * 256), 16,
                                                     voffA + wave * 16 * (int)p.lda * 2 + go, kb, 0, 0);
        } else {
            int go = (j - 4) * gstrW;
            asm volatile("" : "+s"(go));
            __builtin_amdgcn_raw_ptr_buffer_load_lds(srdW, (CE_LDS void*)(base + A_BYTES + (16 * (j - 4) + 4 * wave) * 256),
                                                     16, voffW + wave * 16 * (int)p.ldw * 2 + go, kb, 0, 0);
        }
    };

    // ---- fragment reads: lane reads row fr of a 16-row fragment, k = 8 fq .. 8 fq + 7 (source chunk fq)
    const int fr = lane & 15, fq = lane >> 4;
    const int fo = fr * 64 + ((fq ^ (((fr >> 3) & 1) << 1)) << 4);
    const unsigned abase = (unsigned)(uintptr_t)(CE_LDS void*)(smem + wm * 128 * 64 + fo);
    const unsigned wbase = (unsigned)(uintptr_t)(CE_LDS void*)(smem + A_BYTES + wn * 64 * 64 + fo);

    f32x4 acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    bf16x8 bw[2][4], ar[BLOCK ? 8 : 3];

    // epilogue operands, loaded during the last K-step
    float4 bv[4], cv[4];
    float2 st[8];
    const int mbase = m0 + wm * 128, nbase = n0 + wn * 64;
    // through buffer descriptors (a null bias = a 0-record descriptor: reads return 0), no branches
    auto load_epi_ops = [&]() __attribute__((always_inline)) {
        const __amdgpu_buffer_rsrc_t bsrd =
            make_srd(p.bias ? (const void*)p.bias : (const void*)p.A, p.bias ? p.N * 4 : 0);
#pragma unroll
        for (int j = 0; j < 4; ++j)
            bv[j] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(bsrd, (nbase + 16 * j + 4 * fq) * 4, 0, 0));
        if constexpr (EPI == EPI_LN_FOLD) {
            const __amdgpu_buffer_rsrc_t csrd = make_srd(p.fold_c, p.N * 4);
            const __amdgpu_buffer_rsrc_t ssrd = make_srd(p.fold_stats, p.M * 8);
#pragma unroll
            for (int j = 0; j < 4; ++j)
                cv[j] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(csrd, (nbase + 16 * j + 4 * fq) * 4, 0, 0));
#pragma unroll
            for (int i = 0; i < 8; ++i)
                st[i] = __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(ssrd, (mbase + 16 * i + fr) * 8, 0, 0));
        }
    };

#define W2B_RD(DST, BASE, IMM) asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(DST) : "v"(BASE), "n"(IMM))
#define W2B_MFMA(ACC, BV, AV) \
    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(ACC) : "v"(BV), "v"(AV))

    // one K-step from ring slot S (compile time) with W-fragment set P (step parity)
    auto step = [&](int t, auto sc, auto pc) __attribute__((always_inline)) {
        constexpr int S = decltype(sc)::value;
        constexpr int P = decltype(pc)::value;
        constexpr int SO = S * SLOT;
        if (t + 1 < nk) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        barrier();
        const bool pf = t + 2 < nk;
        if constexpr (BLOCK) {
            W2B_RD(bw[P][0], wbase, SO + 0 * 1024);
            W2B_RD(bw[P][1], wbase, SO + 1 * 1024);
            W2B_RD(bw[P][2], wbase, SO + 2 * 1024);
            W2B_RD(bw[P][3], wbase, SO + 3 * 1024);
            W2B_RD(ar[0], abase, SO + 0 * 1024);
            W2B_RD(ar[1], abase, SO + 1 * 1024);
            W2B_RD(ar[2 % (BLOCK ? 8 : 3)], abase, SO + 2 * 1024);
            W2B_RD(ar[3 % (BLOCK ? 8 : 3)], abase, SO + 3 * 1024);
            W2B_RD(ar[4 % (BLOCK ? 8 : 3)], abase, SO + 4 * 1024);
            W2B_RD(ar[5 % (BLOCK ? 8 : 3)], abase, SO + 5 * 1024);
            W2B_RD(ar[6 % (BLOCK ? 8 : 3)], abase, SO + 6 * 1024);
            W2B_RD(ar[7 % (BLOCK ? 8 : 3)], abase, SO + 7 * 1024);
            if (pf) {
#pragma unroll
                for (int j = 0; j < 6; ++j) piece(t + 2, j);
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            if constexpr (PRIO) asm volatile("s_setprio 1" ::: "memory");
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                W2B_MFMA(acc[i][0], bw[P][0], ar[i % (BLOCK ? 8 : 3)]);
                W2B_MFMA(acc[i][1], bw[P][1], ar[i % (BLOCK ? 8 : 3)]);
                W2B_MFMA(acc[i][2], bw[P][2], ar[i % (BLOCK ? 8 : 3)]);
                W2B_MFMA(acc[i][3], bw[P][3], ar[i % (BLOCK ? 8 : 3)]);
            }
            if constexpr (PRIO) asm volatile("s_setprio 0" ::: "memory");
            return;
        }
        // W fragments 0..3, A fragments 0..1
        W2B_RD(bw[P][0], wbase, SO + 0 * 1024);
        W2B_RD(bw[P][1], wbase, SO + 1 * 1024);
        W2B_RD(bw[P][2], wbase, SO + 2 * 1024);
        W2B_RD(bw[P][3], wbase, SO + 3 * 1024);
        W2B_RD(ar[0], abase, SO + 0 * 1024);
        W2B_RD(ar[1], abase, SO + 1 * 1024);
        if constexpr (PRIO) asm volatile("s_setprio 1" ::: "memory");
        static_for<8>([&](auto ic) {
            constexpr int i = decltype(ic)::value;
            // fragments of row i landed (row i + 1's read may stay in flight)
            if constexpr (i < 7) asm volatile("s_waitcnt lgkmcnt(1)" ::: "memory");
            else asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            W2B_MFMA(acc[i][0], bw[P][0], ar[i % 3]);
            W2B_MFMA(acc[i][1], bw[P][1], ar[i % 3]);
            // row i + 2's A fragment into the ring register row i - 1 used (its MFMAs issued >= 2 ago)
            if constexpr (i + 2 < 8) W2B_RD(ar[(i + 2) % 3], abase, SO + (i + 2) * 1024);
            W2B_MFMA(acc[i][2], bw[P][2], ar[i % 3]);
            if (i < 6 && pf) piece(t + 2, i);
            W2B_MFMA(acc[i][3], bw[P][3], ar[i % 3]);
        });
        if constexpr (PRIO) asm volatile("s_setprio 0" ::: "memory");
    };

    piece(0, 0); piece(0, 1); piece(0, 2); piece(0, 3); piece(0, 4); piece(0, 5);
    if (nk > 1) { piece(1, 0); piece(1, 1); piece(1, 2); piece(1, 3); piece(1, 4); piece(1, 5); }
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    using I2 = std::integral_constant<int, 2>;
    // unrolled by 6 so the ring slot (t % 3) and the W-fragment set (t % 2) are compile-time
    int t = 0;
    for (; t + 6 <= nk; t += 6) {
        step(t, I0{}, I0{});
        step(t + 1, I1{}, I1{});
        step(t + 2, I2{}, I0{});
        step(t + 3, I0{}, I1{});
        step(t + 4, I1{}, I0{});
        step(t + 5, I2{}, I1{});
    }
    if (t < nk) step(t, I0{}, I0{});
    if (t + 1 < nk) step(t + 1, I1{}, I1{});
    if (t + 2 < nk) step(t + 2, I2{}, I0{});
    if (t + 3 < nk) step(t + 3, I0{}, I1{});
    if (t + 4 < nk) step(t + 4, I1{}, I0{});
#undef W2B_MFMA
#undef W2B_RD
    // epilogue operands (L2-resident; the CU's other workgroup covers the latency)
    load_epi_ops();
    // the last MFMAs' results are read by VALU below (asm MFMAs: no hazard tracking by hipcc)
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");

    // ---- epilogue: lane holds C[mbase + 16 i + fr][nbase + 16 j + 4 fq .. +3]; rows 2ip, 2ip + 1 of a
    // lane pair (l, l ^ 16) traded by v_permlane16_swap so each lane stores 8 consecutive columns
    const int rows = max(0, min(p.M - mbase, 128));
    if constexpr (EPI == EPI_LN_STATS_HL) {
        hl_epilogue(p, acc, bv, mbase, nbase, rows, fr, fq);
        return;
    }
    const __amdgpu_buffer_rsrc_t osrd = make_srd(static_cast<bf16_t*>(p.out) + (size_t)mbase * p.ldo, rows * (int)p.ldo * 2);
    const int ldo2 = (int)p.ldo * 2;
    int voff = (fr + (fq & 1) * 16) * ldo2 + (fq >> 1) * 16 + nbase * 2;
#pragma unroll
    for (int ip = 0; ip < 4; ++ip) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            uint2 h[2];
#pragma unroll
            for (int r = 0; r < 2; ++r) {
                f32x4 v = acc[2 * ip + r][j];
                const float4 b = bv[j];
                if constexpr (EPI == EPI_LN_FOLD) {
                    const float4 c = cv[j];
                    const float2 s2 = st[2 * ip + r];
                    v[0] = fmaf(s2.y, fmaf(-s2.x, c.x, v[0]), b.x);
                    v[1] = fmaf(s2.y, fmaf(-s2.x, c.y, v[1]), b.y);
                    v[2] = fmaf(s2.y, fmaf(-s2.x, c.z, v[2]), b.z);
                    v[3] = fmaf(s2.y, fmaf(-s2.x, c.w, v[3]), b.w);
                } else {
                    v[0] += b.x; v[1] += b.y; v[2] += b.z; v[3] += b.w;
                }
                v = act4<ACT>(v);
                h[r] = make_uint2(pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3]));
            }
            const auto x = __builtin_amdgcn_permlane16_swap(h[0].x, h[1].x, false, false);
            const auto y = __builtin_amdgcn_permlane16_swap(h[0].y, h[1].y, false, false);
            const u32x4 d = {x[0], y[0], x[1], y[1]};
            __builtin_amdgcn_raw_buffer_store_b128(d, osrd, voff + j * 32, 0, 0);
        }
        voff += 32 * ldo2;
    }
}

}  // namespace

bool gemm_w2b_supported(const GemmParams& p, int epi, bool out_bf16, bool resid) {
    const bool base = p.N % TN == 0 && p.K % KS == 0 && p.K >= 2 * KS && p.grp == 0 && !p.m_dev && !p.pre_out &&
                      p.M > 0;
    if (epi == EPI_LN_STATS_HL)     // hi/lo planes in and out (the resid pointer is unused: p.rhl)
        return base && !out_bf16 && p.rhl && p.hl_plane > 0 && p.xb && p.stats_part;
    return base && out_bf16 && !resid && (epi == EPI_PLAIN || epi == EPI_LN_FOLD) &&
           (epi != EPI_LN_FOLD || (p.fold_c && p.fold_stats && p.bias));
}

hipError_t launch_gemm_w2b(const GemmParams& p, int act, int epi, hipStream_t s) {
    if (!gemm_w2b_supported(p, epi, epi != EPI_LN_STATS_HL, false)) return hipErrorInvalidValue;
    const int nwg = ((p.M + TM - 1) / TM) * (p.N / TN);
    const int var = (p.variant >> 22) & 3;
#define W2B_LAUNCH(A_, E_)                                                                                   \
    do {                                                                                                  \
        if (var == 1) hipLaunchKernelGGL((gemm_w2b<A_, E_, 1>), dim3(nwg), dim3(256), 0, s, p);            \
        else if (var == 2) hipLaunchKernelGGL((gemm_w2b<A_, E_, 2>), dim3(nwg), dim3(256), 0, s, p);       \
        else if (var == 3) hipLaunchKernelGGL((gemm_w2b<A_, E_, 3>), dim3(nwg), dim3(256), 0, s, p);       \
        else hipLaunchKernelGGL((gemm_w2b<A_, E_, 0>), dim3(nwg), dim3(256), 0, s, p);                     \
    } while (0)
    if (epi == EPI_LN_STATS_HL) {
        if (act != ACT_NONE) return hipErrorInvalidValue;
        W2B_LAUNCH(ACT_NONE, EPI_LN_STATS_HL);
    } else if (epi == EPI_LN_FOLD) {
        if (act == ACT_GELU) W2B_LAUNCH(ACT_GELU, EPI_LN_FOLD);
        else if (act == ACT_QGELU) W2B_LAUNCH(ACT_QGELU, EPI_LN_FOLD);
        else W2B_LAUNCH(ACT_NONE, EPI_LN_FOLD);
    } else {
        if (act == ACT_GELU) W2B_LAUNCH(ACT_GELU, EPI_PLAIN);
        else if (act == ACT_QGELU) W2B_LAUNCH(ACT_QGELU, EPI_PLAIN);
        else W2B_LAUNCH(ACT_NONE, EPI_PLAIN);
    }
#undef W2B_LAUNCH
    return hipGetLastError();
}

}  // namespace ce
