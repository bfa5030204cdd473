// Weight-gradient GEMM with MN-major operands for gfx950 (CDNA4).
//
// The text tower's backward (open_clip transformer.py:228-239 run in reverse; autograd of
// train_negclip.py in the reference) needs, per block, dW[o][i] = sum over tokens t of
// dY[t][o] X[t][i] for in_proj, out_proj, c_fc and c_proj.  Both operands are the row-major
// [tokens][features] activations the forward kept and the backward produced, and the reduction
// runs down their rows: neither is K-contiguous.  Through round 4 each was transposed first (eight
// transposes per block, 14 ms of a 481-ms NegCLIP step); this kernel reads them in place:
//
//   C[m][n] = scale_m * sum_k A[k][m] B[k][n]      A [K][lda], B [K][ldb] bf16;  C [M][ldc] f32
//   scale_m = scale for m < scale_rows, else 1 (in_proj's q rows carry kAttnQScale in the engine)
//
// Design:
//  * the four-wave main loop of gemm.hip's SCHED 10/11: 256 threads, 256x256 output tile, each
//    wave 128x128 (8x8 v_mfma_f32_16x16x32_bf16 tiles, 256 accumulators pinned in AGPRs), BK = 64,
//    two 64-KB LDS stages filled by LDS-DMA two K-tiles ahead, two barriers per K-tile.
//  * LDS image of an operand K-tile: 64 k-rows x 512 B (256 columns), each row one coalesced 512-B
//    segment of the source.  16-B chunk c of row r sits at chunk c ^ sw(r),
//    sw(r) = 2 ((r & 3) | ((r >> 1) & 4)).
//  * MFMA fragments (8 consecutive k of one column per lane) by ds_read_b64_tr_b16: lane 4q + p of
//    a 16-lane group addresses k-row q, columns 4p..4p+3 of its block, and every lane receives one
//    column's 4 k values; reads h = 0, 1 (k-rows 8g + 4h + 0..3 for group g) make one fragment.
//    A half-wave's 32 lanes touch k-rows 8g + q (g in {0, 1}, q in 0..3) at one 32-B piece each;
//    sw maps the 8 rows to 8 distinct even chunk offsets, so the 256 B fall into 64 distinct banks.
//    sw is the same for every read of a lane (it depends on q and g & 1 only).
//  * all fragment reads and MFMAs are inline asm (issue order = source order); the reads are
//    counted by explicit lgkmcnt waits.  (The ds_read_tr builtin makes hipcc wait vmcnt(0) first:
//    it cannot tell the buffer being read from the one the DMA in flight fills.)
//  * split-K over the tokens (K = 118,272 for a 1,024 + 512 caption batch): tiles x split ~ one
//    workgroup per CU, partial tiles in f32 slabs summed in fixed order by gemm_tn_fixup
//    (deterministic), which applies the row scale.  split == 1 stores C directly.
#include "ce_device.h"
#include "ce_kernels.h"
#include "knobs.h"

#include <algorithm>
#include <type_traits>
#include <utility>

namespace ce {

namespace {

constexpr int TN_T = 256, TN_BK = 64;
constexpr int TN_OP = TN_BK * TN_T * 2;     // 32 KB: one operand's K-tile image
constexpr int TN_STAGE = 2 * TN_OP;         // A + B
constexpr int TN_SLAB = TN_T * TN_T;        // f32 elements of one partial tile

template <class F, int... I>
__device__ __forceinline__ void tn_unroll_impl(F& f, std::integer_sequence<int, I...>) {
    (f(std::integral_constant<int, I>{}), ...);
}
// f(integral_constant<int, i>) for i = 0 .. N-1, each i a constant expression
template <int N, class F>
__device__ __forceinline__ void tn_unroll(F&& f) {
    tn_unroll_impl(f, std::make_integer_sequence<int, N>{});
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t tn_srd(const void* base, int nbytes) {
    const uint64_t b = reinterpret_cast<uint64_t>(base);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)b);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32));
    const int n = __builtin_amdgcn_readfirstlane(nbytes);
    return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(((uint64_t)hi << 32) | lo), (short)0, n,
                                             0x00020000);
}

__device__ __forceinline__ void tn_barrier() {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

// blocks b and b + 8 share an XCD: give each XCD a contiguous range of workgroup ids (the tiles of
// one K-chunk, which share A and B column panels at the same k)
__device__ __forceinline__ int tn_xcd_remap(int bid, int nwg) {
    const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

template <int OFF>
__device__ __forceinline__ void tn_tr(s16x4& r, unsigned addr) {
    asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(r) : "v"(addr), "n"(OFF));
}

template <int N>
__device__ __forceinline__ void tn_wait_lgkm() {
    asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ bf16x8 tn_frag(const s16x4& lo, const s16x4& hi) {
    typedef __attribute__((ext_vector_type(8))) short s16x8;
    return __builtin_bit_cast(bf16x8, (s16x8)__builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
}

#define CE_TN_MFMA(ACC, BV, AV) \
    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(ACC) : "v"(BV), "v"(AV))

// One workgroup: output tile (tm, tn), K-tiles [kt0, kt1) of chunk `chunk`.
// Per K-tile (set s = k-rows 32s .. 32s+31 of the tile; a set is 8 A and 8 B fragments):
//   B1: MFMA(set0, rows 0-3)  + 32 reads (set1 of this K-tile)        -> lgkmcnt(0), barrier
//   B2: MFMA(set0, rows 4-7) + MFMA(set1, rows 0-3) + 16 DMA (K-tile t+2 -> this stage)
//                                                                      -> vmcnt(16), barrier
//   B3: MFMA(set1, rows 4-7)  + 32 reads (set0 of K-tile t+1, other stage)
// A set's 32 reads in order: B blocks 0-7 (h = 0, 1), then A blocks 0-7.
__global__ __launch_bounds__(256, 1) void gemm_tn_w4(TnParams p) {
    __shared__ __attribute__((aligned(16))) char smem[2 * TN_STAGE];
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave >> 1, wn = wave & 1;
    const int tiles_n = p.N / TN_T;
    const int tiles = (p.M / TN_T) * tiles_n;
    const int nwg = tiles * p.split;
    const int wgid = tn_xcd_remap(blockIdx.x, nwg);
    const int chunk = wgid / tiles, tile = wgid - chunk * tiles;
    const int tm = tile / tiles_n, tn = tile - tm * tiles_n;
    const int m0 = tm * TN_T, n0 = tn * TN_T;
    const int nkt = (p.K + TN_BK - 1) / TN_BK;
    const int kt0 = (int)((long)chunk * nkt / p.split);
    const int nk = (int)((long)(chunk + 1) * nkt / p.split) - kt0;

    // staging: DMA j (0..7) of wave w copies k-rows 8j + 2w + (lane >> 5) of the K-tile, LDS
    // chunk lane & 31 of the row, from source chunk (lane & 31) ^ sw(row); sw(row) depends on j
    // only through bit 3 of the row = j & 1
    const int r0 = 2 * wave + (lane >> 5), cpos = lane & 31;
    const int lda2 = (int)p.lda * 2, ldb2 = (int)p.ldb * 2;
    const int voA0 = r0 * lda2 + ((cpos ^ (2 * (r0 & 3))) << 4);
    const int voA1 = r0 * lda2 + ((cpos ^ (2 * ((r0 & 3) | 4))) << 4);
    const int voB0 = r0 * ldb2 + ((cpos ^ (2 * (r0 & 3))) << 4);
    const int voB1 = r0 * ldb2 + ((cpos ^ (2 * ((r0 & 3) | 4))) << 4);
    // descriptors from the tile's first column: rows past K read as zero (the clip at K rows)
    const __amdgpu_buffer_rsrc_t srdA = tn_srd(p.A + m0, (int)(((long)p.K * p.lda - m0) * 2));
    const __amdgpu_buffer_rsrc_t srdB = tn_srd(p.B + n0, (int)(((long)p.K * p.ldb - n0) * 2));
    char* const lds = smem;
    auto dma = [&](int kt, int buf, auto jc) __attribute__((always_inline)) {
        constexpr int j = decltype(jc)::value;     // 0..7: A, 8..15: B
        constexpr int jj = j & 7;
        const bool live = kt < nk;
        char* dst = lds + buf * TN_STAGE + (j < 8 ? 0 : TN_OP) + jj * 4096 + wave * 1024;
        if constexpr (j < 8) {
            const int so = live ? (kt0 + kt) * TN_BK * lda2 + jj * 8 * lda2 : 0x7ff00000;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(srdA, (CE_LDS void*)dst, 16, (jj & 1) ? voA1 : voA0, so, 0, 0);
        } else {
            const int so = live ? (kt0 + kt) * TN_BK * ldb2 + jj * 8 * ldb2 : 0x7ff00000;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(srdB, (CE_LDS void*)dst, 16, (jj & 1) ? voB1 : voB0, so, 0, 0);
        }
    };

    // fragment addresses: lane 4q + pp of group g reads k-row 8g + q (+ 4h, + 32s), columns of
    // block c at chunk (c0 / 8 + pp / 2) ^ fx, fx = sw(row) = 2 (q | 4 (g & 1))
    const int g = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
    const int fx = 2 * (q | ((g & 1) << 2));
    const unsigned lds0 = (unsigned)(uintptr_t)(CE_LDS void*)lds;
    const unsigned lrow = lds0 + (8 * g + q) * 512 + pp * 8;
    unsigned abase[8], bbase[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        abase[i] = lrow + ((wm * 16 + ((2 * i) ^ fx)) << 4);
        bbase[i] = lrow + TN_OP + ((wn * 16 + ((2 * i) ^ fx)) << 4);
    }

    f32x4 acc[8][8];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    s16x4 fa[2][8][2], fb[2][8][2];     // [set][block][h]

    // read r (0..31) of set S from stage BUF
    auto rd = [&](auto sc, auto bc, auto rc) __attribute__((always_inline)) {
        (void)fa; (void)fb; (void)abase; (void)bbase;   // captured before the dependent uses below
        constexpr int S = decltype(sc)::value, BUF = decltype(bc)::value, r = decltype(rc)::value;
        constexpr int blk = (r & 15) >> 1, h = r & 1;
        constexpr int off = S * 32 * 512 + h * 4 * 512;
        if constexpr (r < 16) tn_tr<off>(fb[S][blk][h], bbase[blk] + BUF * TN_STAGE);
        else tn_tr<off>(fa[S][blk][h], abase[blk] + BUF * TN_STAGE);
    };
    auto mfma = [&](auto sc, int i, int j) __attribute__((always_inline)) {
        (void)acc; (void)fa; (void)fb;
        constexpr int S = decltype(sc)::value;
        CE_TN_MFMA(acc[i][j], tn_frag(fb[S][j][0], fb[S][j][1]), tn_frag(fa[S][i][0], fa[S][i][1]));
    };
    using C0 = std::integral_constant<int, 0>;
    using C1 = std::integral_constant<int, 1>;

    // one K-tile on stage BUF; kt relative to kt0
    auto ktile = [&](int kt, auto bc) __attribute__((always_inline)) {
        constexpr int BUF = decltype(bc)::value;
        using NB = std::integral_constant<int, BUF ^ 1>;
        // ---- B1: MFMA(set0, rows 0-3); set1 of this K-tile read under it ----
        tn_unroll<32>([&](auto sc2) __attribute__((always_inline)) {
            constexpr int s2 = decltype(sc2)::value, i = s2 >> 3, j = s2 & 7;
            // set0's A block i is read 17 + 2i of the 32 issued in B3; s2 set1 reads followed it
            if constexpr (j == 0) {
                constexpr int n = 14 - 2 * i + s2;
                tn_wait_lgkm<(n < 15 ? n : 15)>();
                __builtin_amdgcn_sched_barrier(0);
            }
            mfma(C0{}, i, j);
            rd(C1{}, bc, sc2);
        });
        tn_wait_lgkm<0>();
        tn_barrier();
        __builtin_amdgcn_sched_barrier(0);
        // ---- B2: MFMA(set0, rows 4-7) + MFMA(set1, rows 0-3); DMA of K-tile kt + 2 ----
        tn_unroll<64>([&](auto sc2) __attribute__((always_inline)) {
            constexpr int s2 = decltype(sc2)::value, i = (s2 >> 3) & 3, j = s2 & 7;
            if constexpr (s2 < 32) mfma(C0{}, 4 + i, j);
            else mfma(C1{}, i, j);
            if constexpr ((s2 & 3) == 3) dma(kt + 2, BUF, std::integral_constant<int, (s2 >> 2)>{});
        });
        asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
        tn_barrier();
        __builtin_amdgcn_sched_barrier(0);
        // ---- B3: MFMA(set1, rows 4-7); set0 of K-tile kt + 1 read under it ----
        tn_unroll<32>([&](auto sc2) __attribute__((always_inline)) {
            constexpr int s2 = decltype(sc2)::value, i = s2 >> 3, j = s2 & 7;
            mfma(C1{}, 4 + i, j);
            rd(C0{}, NB{}, sc2);
        });
    };

    // prologue: K-tiles 0 and 1 in flight, set0 of K-tile 0
    tn_unroll<16>([&](auto jc) { dma(0, 0, jc); });
    tn_unroll<16>([&](auto jc) { dma(1, 1, jc); });
    asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    tn_barrier();
    tn_unroll<32>([&](auto rc) { rd(C0{}, C0{}, rc); });

    int kt = 0;
    for (; kt + 1 < nk; kt += 2) {
        ktile(kt, C0{});
        ktile(kt + 1, C1{});
    }
    if (kt < nk) ktile(kt, C0{});
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");

    // lane holds C[m = 16i + (lane & 15)][n = 16j + 4 (lane >> 4) .. +3] of the wave's quadrant
    const int fr = lane & 15, fq = lane >> 4;
    const int mq = wm * 128 + fr, nq = wn * 128 + fq * 4;
    if (p.split == 1) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int m = m0 + mq + i * 16;
            const float sc = m < p.scale_rows ? p.scale : 1.f;
            float* dst = p.C + (long)m * p.ldc + n0 + nq;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const f32x4 v = acc[i][j];
                *reinterpret_cast<float4*>(dst + j * 16) = make_float4(v[0] * sc, v[1] * sc, v[2] * sc, v[3] * sc);
            }
        }
    } else {
        float* slab = p.part + ((long)tile * p.split + chunk) * TN_SLAB;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            float* dst = slab + (mq + i * 16) * TN_T + nq;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const f32x4 v = acc[i][j];
                *reinterpret_cast<float4*>(dst + j * 16) = make_float4(v[0], v[1], v[2], v[3]);
            }
        }
    }
}
#undef CE_TN_MFMA

// C[m][n] = scale_m * sum over chunks c (in order) of slab[tile][c][m % 256][n % 256]; one float4
// per thread
__global__ __launch_bounds__(256) void gemm_tn_fixup(TnParams p) {
    const long idx = (long)blockIdx.x * 256 + threadIdx.x;
    const int n4 = p.N >> 2;
    if (idx >= (long)p.M * n4) return;
    const int m = (int)(idx / n4);
    const int n = (int)(idx - (long)m * n4) * 4;
    const int tile = (m / TN_T) * (p.N / TN_T) + n / TN_T;
    const float* src = p.part + (long)tile * p.split * TN_SLAB + (m % TN_T) * TN_T + (n % TN_T);
    float4 s = *reinterpret_cast<const float4*>(src);
    for (int c = 1; c < p.split; ++c) {
        const float4 v = *reinterpret_cast<const float4*>(src + (long)c * TN_SLAB);
        s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
    const float sc = m < p.scale_rows ? p.scale : 1.f;
    *reinterpret_cast<float4*>(p.C + (long)m * p.ldc + n) = make_float4(s.x * sc, s.y * sc, s.z * sc, s.w * sc);
}

int tn_num_cus() { return device_cus(); }     // cached per device (knobs.h)

}  // namespace

int gemm_tn_split(int M, int N, int K, long part_elems) {
    if (M <= 0 || N <= 0 || K <= 0 || M % TN_T || N % TN_T) return 0;
    const int tiles = (M / TN_T) * (N / TN_T);
    const int nkt = (K + TN_BK - 1) / TN_BK;
    int split = tn_num_cus() / tiles;                       // one workgroup per CU
    split = std::min(split, nkt / 8);                        // >= 8 K-tiles per chunk
    split = (int)std::min<long>(split, part_elems / ((long)tiles * TN_SLAB));
    return std::max(split, 1);
}

hipError_t launch_gemm_tn(const TnParams& p0, hipStream_t s) {
    TnParams p = p0;
    if (!p.A || !p.B || !p.C || p.M <= 0 || p.N <= 0 || p.K <= 0 || p.M % TN_T || p.N % TN_T || p.lda < p.M ||
        p.ldb < p.N || p.ldc < p.N || p.lda % 8 || p.ldb % 8 || p.ldc % 4 ||
        (reinterpret_cast<uintptr_t>(p.A) | reinterpret_cast<uintptr_t>(p.B) | reinterpret_cast<uintptr_t>(p.C)) % 16)
        return hipErrorInvalidValue;
    // byte offsets of the DMAs are 32-bit (the past-K sentinel sits above 0x7ff00000)
    if ((long)p.K * p.lda * 2 > 0x7fe00000L || (long)p.K * p.ldb * 2 > 0x7fe00000L) return hipErrorInvalidValue;
    p.split = p.part ? gemm_tn_split(p.M, p.N, p.K, p.part_elems) : 1;
    const int tiles = (p.M / TN_T) * (p.N / TN_T);
    hipLaunchKernelGGL(gemm_tn_w4, dim3(tiles * p.split), dim3(256), 0, s, p);
    if (p.split > 1) {
        const long n4 = (long)p.M * p.N / 4;
        hipLaunchKernelGGL(gemm_tn_fixup, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, s, p);
    }
    return hipGetLastError();
}

}  // namespace ce
