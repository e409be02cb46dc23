// tune_tree3.hip -- the C3 combine (8 x 32 MiB f32 leaves -> 32 MiB, fixed
// tree, SUM) against the ceilings of its own traffic on the same buffers:
// the 8 leaf reads alone, the 32 MiB result write alone, and one 256 MiB
// stream read (the same bytes as the 8 leaves, one stream).  Leaves sit in
// one allocation 4 KiB apart as in the product's staging pool; 4 such sets
// rotate, so no launch finds its operands in the 256 MiB Infinity Cache.
// Variants run interleaved in one process; median of R rounds x 20 launches.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <algorithm>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));
#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

struct P8 { const f32x4 *s[8]; f32x4 *d; long nvec; };

// MODE 0: tree + store (the product's k_tree_body); 1: the 8 reads only;
// 2: the store only.  CAP: static LDS per block to cap residency (0 = none).
// X > 0: a block's U 4-KiB segments spread over consecutive blocks (XCDs).
template <int U, int MODE, int CAPKIB, int X>
__global__ void __launch_bounds__(256) k_t(P8 p)
{
    __shared__ char lds_cap[CAPKIB ? CAPKIB * 1024 : 1];
    if (p.nvec < 0) lds_cap[threadIdx.x] = 0;
    const long nthr = (long)gridDim.x * 256;
    f32x4 acc = {0, 0, 0, 0};
    for (long c0 = (long)blockIdx.x * 256 * U + threadIdx.x; c0 < p.nvec; c0 += nthr * U) {
        f32x4 x[U][8];
        long cs[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (X) {
                const long b = blockIdx.x;
                cs[u] = (((b / X) * U + u) * X + b % X) * 256 + threadIdx.x;
            } else {
                cs[u] = c0 + (long)u * 256;
            }
        }
        if (MODE != 2) {
#pragma unroll
            for (int u = 0; u < U; ++u)
                if (cs[u] < p.nvec)
#pragma unroll
                    for (int q = 0; q < 8; ++q) x[u][q] = __builtin_nontemporal_load(p.s[q] + cs[u]);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (cs[u] >= p.nvec) continue;
            if (MODE == 2) {
                __builtin_nontemporal_store((f32x4){1.f, 2.f, 3.f, (float)u}, p.d + cs[u]);
                continue;
            }
#pragma unroll
            for (int h = 1; h < 8; h <<= 1)
#pragma unroll
                for (int q = 0; q + h < 8; q += 2 * h) x[u][q] = x[u][q] + x[u][q + h];
            if (MODE == 0) __builtin_nontemporal_store(x[u][0], p.d + cs[u]);
            else acc += x[u][0];
        }
        if (X) break;   // exact grid, one pass
    }
    if (MODE == 1 && acc.x == 1234.5f) p.d[threadIdx.x] = acc;
}

// persistent grid, software-pipelined: the loads of the next batch are in
// flight while the current batch is combined and stored
template <int U>
__global__ void __launch_bounds__(256) k_t_pipe(P8 p)
{
    __shared__ char lds_cap[56 * 1024];
    if (p.nvec < 0) lds_cap[threadIdx.x] = 0;
    const long nthr = (long)gridDim.x * 256;
    long c0 = (long)blockIdx.x * 256 * U + threadIdx.x;
    f32x4 cur[U][8], nxt[U][8];
#pragma unroll
    for (int u = 0; u < U; ++u)
        if (c0 + u * 256 < p.nvec)
#pragma unroll
            for (int q = 0; q < 8; ++q) cur[u][q] = __builtin_nontemporal_load(p.s[q] + c0 + u * 256);
    for (; c0 < p.nvec; c0 += nthr * U) {
        const long c1 = c0 + nthr * U;
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (c1 + u * 256 < p.nvec)
#pragma unroll
                for (int q = 0; q < 8; ++q) nxt[u][q] = __builtin_nontemporal_load(p.s[q] + c1 + u * 256);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (c0 + u * 256 >= p.nvec) continue;
#pragma unroll
            for (int h = 1; h < 8; h <<= 1)
#pragma unroll
                for (int q = 0; q + h < 8; q += 2 * h) cur[u][q] = cur[u][q] + cur[u][q + h];
            __builtin_nontemporal_store(cur[u][0], p.d + c0 + u * 256);
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int q = 0; q < 8; ++q) cur[u][q] = nxt[u][q];
    }
}

// one 256 MiB stream read (p.s[0] spans all 8 leaves of the set)
template <int U>
__global__ void __launch_bounds__(256) k_read1(P8 p)
{
    const long n = p.nvec * 8;
    const long nthr = (long)gridDim.x * 256;
    f32x4 acc = {0, 0, 0, 0};
    for (long c0 = (long)blockIdx.x * 256 * U + threadIdx.x; c0 < n; c0 += nthr * U) {
        f32x4 x[U];
#pragma unroll
        for (int u = 0; u < U; ++u) x[u] = c0 + u * 256 < n ? __builtin_nontemporal_load(p.s[0] + c0 + u * 256) : acc;
#pragma unroll
        for (int u = 0; u < U; ++u) acc += x[u];
    }
    if (acc.x == 1234.5f) p.d[threadIdx.x] = acc;
}

typedef void (*KF)(P8);
struct Var { const char *name; KF f; int U; double moved_leaves; int one_stream; long grid; };

int main(int argc, char **argv)
{
    const long leaf = 32L << 20, stag = 4096;
    const int sets = 4, rounds = argc > 1 ? atoi(argv[1]) : 7;
    std::vector<P8> ps(sets), ps1(sets);
    for (int s = 0; s < sets; ++s) {
        char *big;
        const size_t bytes = 9 * (leaf + stag);
        CHECK(hipMalloc(&big, bytes));
        CHECK(hipMemset(big, 0x3c, bytes));
        for (int q = 0; q < 8; ++q) ps[s].s[q] = (const f32x4 *)(big + q * (leaf + stag));
        ps[s].d = (f32x4 *)(big + 8 * (leaf + stag));
        ps[s].nvec = leaf / 16;
        ps1[s] = ps[s];
        char *one;   // one contiguous 256 MiB stream
        CHECK(hipMalloc(&one, 8 * leaf));
        CHECK(hipMemset(one, 0x3c, 8 * leaf));
        ps1[s].s[0] = (const f32x4 *)one;
    }
    Var vars[] = {
        {"tree U2 cap56 (product)", k_t<2, 0, 56, 0>, 2, 9, 0},
        {"tree U2 cap56 X8", k_t<2, 0, 56, 8>, 2, 9, 0},
        {"tree U1 uncapped", k_t<1, 0, 0, 0>, 1, 9, 0},
        {"tree U2 cap40", k_t<2, 0, 40, 0>, 2, 9, 0},
        {"tree U1 cap56", k_t<1, 0, 56, 0>, 1, 9, 0},
        {"read8 U2 cap56", k_t<2, 1, 56, 0>, 2, 8, 0},
        {"read8 U1 uncapped", k_t<1, 1, 0, 0>, 1, 8, 0},
        {"read8 U2 uncapped", k_t<2, 1, 0, 0>, 2, 8, 0},
        {"write32 U1", k_t<1, 2, 0, 0>, 1, 1, 0},
        {"write32 U2 X8", k_t<2, 2, 0, 8>, 2, 1, 0},
        {"pipe U1 g512", k_t_pipe<1>, 1, 9, 0, 512},
        {"pipe U2 g512", k_t_pipe<2>, 2, 9, 0, 512},
        {"pipe U1 g1024", k_t_pipe<1>, 1, 9, 0, 1024},
        {"pipe U1 g2048", k_t_pipe<1>, 1, 9, 0, 2048},
    };
    const int NV = sizeof(vars) / sizeof(vars[0]);
    // the tree variants agree with each other on set 0 (0x3c3c3c3c x 8, exact)
    {
        float a;
        unsigned ua = 0x3c3c3c3cu;
        memcpy(&a, &ua, 4);
        const float want = ((a + a) + (a + a)) + ((a + a) + (a + a));
        std::vector<float> h(1024);
        for (int v = 0; v < NV; ++v) {
            if (vars[v].moved_leaves != 9) continue;
            CHECK(hipMemset(ps[0].d, 0, leaf));
            long blocks = vars[v].grid ? vars[v].grid : ps[0].nvec / (256L * vars[v].U);
            hipLaunchKernelGGL(vars[v].f, dim3(blocks), dim3(256), 0, 0, ps[0]);
            CHECK(hipDeviceSynchronize());
            for (long off : {0L, leaf / 2, leaf - 4096}) {
                CHECK(hipMemcpy(h.data(), (char *)ps[0].d + off, 4096, hipMemcpyDeviceToHost));
                for (int i = 0; i < 1024; ++i)
                    if (h[i] != want) { printf("MISMATCH %s at byte %ld: %g\n", vars[v].name, off + 4 * i, h[i]); return 1; }
            }
        }
        printf("tree variants correct\n");
    }
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    std::vector<std::vector<float>> t(NV);
    for (int r = 0; r < rounds; ++r) {
        for (int v = 0; v < NV; ++v) {
            const std::vector<P8> &pp = vars[v].one_stream ? ps1 : ps;
            const long blocks = vars[v].grid ? vars[v].grid : (vars[v].one_stream ? pp[0].nvec * 8 : pp[0].nvec) / (256L * vars[v].U);
            for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(vars[v].f, dim3(blocks), dim3(256), 0, 0, pp[w % sets]);
            CHECK(hipEventRecord(e0, 0));
            for (int i = 0; i < 20; ++i) hipLaunchKernelGGL(vars[v].f, dim3(blocks), dim3(256), 0, 0, pp[i % sets]);
            CHECK(hipEventRecord(e1, 0));
            CHECK(hipEventSynchronize(e1));
            float ms;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            t[v].push_back(ms / 20);
        }
        fprintf(stderr, "round %d done\n", r);
    }
    printf("%-26s %8s %8s %8s %6s\n", "variant", "med_us", "min_us", "TB/s", "of8");
    for (int v = 0; v < NV; ++v) {
        auto x = t[v];
        std::sort(x.begin(), x.end());
        const double med = x[x.size() / 2], tbs = vars[v].moved_leaves * leaf / (med * 1e-3) / 1e12;
        printf("%-26s %8.2f %8.2f %8.3f %6.3f\n", vars[v].name, med * 1e3, x[0] * 1e3, tbs, tbs / 8);
    }
    return 0;
}
