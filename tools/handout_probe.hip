// Run-time block hand-out probe (VERDICT r05 "a lost-block race was removed,
// not diagnosed").  Round 5's persistent attention variant 4989 handed q-blocks out from nine int
// counters in one cache line (sched[0..7]: per-XCD ranges, sched[8]: finished workgroups; the last
// workgroup out reset all nine to 0 with plain stores) and lost a block about once in 24 runs.  This
// program runs the same protocol without the attention arithmetic -- each block is a short timed spin
// and a count -- over thousands of launches and checks that every block is handed out exactly once,
// under three ways of resetting the counters between launches:
//   mode 0  the last workgroup out stores 0 to the nine counters (plain stores: round 5's code)
//   mode 1  the last workgroup out resets them with atomic exchanges (device scope)
//   mode 2  the host clears them with hipMemsetAsync before every launch (no in-kernel reset)
// and two layouts: the nine counters in one 128-B line (layout 0, round 5's) or one line each (1).
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/handout_probe tools/handout_probe.hip
//   tools/handout_probe <mode> <layout> <launches> [spin]
// Prints launches with a lost or duplicated block and the first few offending blocks.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                                  \
    do {                                                                                          \
        hipError_t e_ = (x);                                                                      \
        if (e_ != hipSuccess) {                                                                   \
            fprintf(stderr, "%s: %s (%s:%d)\n", #x, hipGetErrorString(e_), __FILE__, __LINE__);   \
            exit(1);                                                                              \
        }                                                                                         \
    } while (0)

__global__ __launch_bounds__(256) void handout_k(int* __restrict__ sched, int stride, int nblk, int mode, int spin,
                                                 int* __restrict__ count, int* __restrict__ owner) {
    __shared__ int s_next;
    const int G = gridDim.x, bid = blockIdx.x, xcd = bid & 7;
    const int own_lo = (int)((long)xcd * nblk / 8), own_hi = (int)((long)(xcd + 1) * nblk / 8);
    auto grab = [&]() {
        // wave 0, lane 0: own XCD's counter first, then the other XCDs' in turn (round 5's order)
        if (threadIdx.x == 0) {
            int got = -1;
            if (own_lo < own_hi) {
                const int k = atomicAdd(&sched[xcd * stride], 1);
                if (own_lo + k < own_hi) got = own_lo + k;
            }
            for (int j = 1; j < 8 && got < 0; ++j) {
                const int x = (xcd + j) & 7;
                const int lo = (int)((long)x * nblk / 8), hi = (int)((long)(x + 1) * nblk / 8);
                if (lo >= hi) continue;
                const int kk = atomicAdd(&sched[x * stride], 1);
                if (lo + kk < hi) got = lo + kk;
            }
            s_next = got;
        }
        __syncthreads();
        const int g = s_next;
        __syncthreads();          // every wave read it before the next grab overwrites it
        return g;
    };
    for (int blk = grab(); blk >= 0; blk = grab()) {
        // the block's "work": a spin of a few microseconds, then one count per block
        const long long t0 = clock64();
        while (clock64() - t0 < spin) __builtin_amdgcn_s_sleep(1);
        if (threadIdx.x == 0) {
            atomicAdd(&count[blk], 1);
            owner[blk] = bid;
        }
    }
    if (mode != 2 && threadIdx.x == 0 && atomicAdd(&sched[8 * stride], 1) == G - 1) {
        for (int i = 0; i < 9; ++i) {
            if (mode == 0) sched[i * stride] = 0;
            else atomicExch(&sched[i * stride], 0);
        }
    }
}

int main(int argc, char** argv) {
    if (argc < 4) {
        fprintf(stderr, "usage: %s <mode 0|1|2> <layout 0|1> <launches> [spin cycles]\n", argv[0]);
        return 2;
    }
    const int mode = atoi(argv[1]), layout = atoi(argv[2]), launches = atoi(argv[3]);
    const int spin = argc > 4 ? atoi(argv[4]) : 2000;
    const int stride = layout ? 32 : 1;              // ints: 128 B apart or adjacent
    int ncu = 0;
    CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    const int G = ncu * 3;                           // three workgroups per CU, as variant 4989
    const int nblk = 5 * 16 * 64;                    // L = 577 (5 q-blocks) x 16 heads x B = 64
    int *sched, *count, *owner;
    CHECK(hipMalloc(&sched, 9 * 32 * sizeof(int)));
    CHECK(hipMalloc(&count, nblk * sizeof(int)));
    CHECK(hipMalloc(&owner, nblk * sizeof(int)));
    CHECK(hipMemset(sched, 0, 9 * 32 * sizeof(int)));
    std::vector<int> h(nblk);
    int bad_launches = 0;
    long lost = 0, dup = 0;
    for (int it = 0; it < launches; ++it) {
        CHECK(hipMemsetAsync(count, 0, nblk * sizeof(int), 0));
        if (mode == 2) CHECK(hipMemsetAsync(sched, 0, 9 * 32 * sizeof(int), 0));
        hipLaunchKernelGGL(handout_k, dim3(G), dim3(256), 0, 0, sched, stride, nblk, mode, spin, count, owner);
        CHECK(hipGetLastError());
        CHECK(hipMemcpy(h.data(), count, nblk * sizeof(int), hipMemcpyDeviceToHost));
        int l = 0, d = 0, first = -1;
        for (int b = 0; b < nblk; ++b) {
            if (h[b] == 0) { ++l; if (first < 0) first = b; }
            if (h[b] > 1) ++d;
        }
        if (l || d) {
            ++bad_launches;
            lost += l;
            dup += d;
            if (bad_launches <= 5) printf("launch %d: %d lost, %d duplicated (first lost block %d)\n", it, l, d, first);
        }
        if ((it + 1) % 500 == 0) {
            printf("mode %d layout %d: %d launches, %d bad so far\n", mode, layout, it + 1, bad_launches);
            fflush(stdout);
        }
    }
    printf("RESULT mode %d layout %d grid %d blocks %d spin %d: %d of %d launches bad, %ld lost, %ld duplicated\n",
           mode, layout, G, nblk, spin, bad_launches, launches, lost, dup);
    return 0;
}
