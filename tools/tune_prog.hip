// tune_prog.hip -- why does the 8-leaf combine (config 3/5 shape) reach ~73 %
// of HBM peak when the 2-leaf op at the same launch size reaches ~78 %?
// Sweeps, for SUM f32 over 8 leaves -> 1 (tree order), the knobs that change
// how many DRAM pages are open at once and how many bytes are in flight:
//   U      16-byte chunks per lane per iteration (loads in flight per leaf)
//   B      threads per block
//   GRID   one pass over the data, or persistent (CUs x resident blocks)
//   ORDER  leaf-major issue (all chunks of leaf 0, then leaf 1 ...) or
//          chunk-major (chunk u of every leaf, then u+1)
//   XCD    consecutive chunk ranges to consecutive blocks (default), or
//          remapped so each XCD (blockIdx % 8) walks one contiguous eighth
//   STAG   bytes between consecutive leaf slots beyond the leaf size
// Rotating buffer sets keep every launch out of the Infinity Cache.  Prints
// one line per variant: median of 5 rounds x 20 launches (HIP events).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <algorithm>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));
#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

struct P8 { const f32x4 *s[8]; f32x4 *d; long nvec; int xcd; };

template <int U, int B, int ORDER>
__global__ void __launch_bounds__(B) k_tree8(P8 p)
{
    long bid = blockIdx.x;
    const long nb = gridDim.x;
    if (p.xcd && nb % 8 == 0) bid = (bid % 8) * (nb / 8) + bid / 8;   // XCD j walks blocks [j*nb/8, (j+1)*nb/8)
    const long nthr = nb * B;
    for (long c0 = bid * B * U + threadIdx.x; c0 < p.nvec; c0 += nthr * U) {
        f32x4 x[U][8];
        if (ORDER == 0) {
#pragma unroll
            for (int q = 0; q < 8; ++q)
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const long c = c0 + (long)u * B;
                    if (c < p.nvec) x[u][q] = __builtin_nontemporal_load(p.s[q] + c);
                }
        } else {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const long c = c0 + (long)u * B;
                if (c < p.nvec)
#pragma unroll
                    for (int q = 0; q < 8; ++q) x[u][q] = __builtin_nontemporal_load(p.s[q] + c);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long c = c0 + (long)u * B;
            if (c < p.nvec) {
#pragma unroll
                for (int h = 1; h < 8; h <<= 1)
#pragma unroll
                    for (int q = 0; q + h < 8; q += 2 * h) x[u][q] = x[u][q] + x[u][q + h];
                __builtin_nontemporal_store(x[u][0], p.d + c);
            }
        }
    }
}

typedef void (*KF)(P8);
struct Var { char name[64]; KF f; int U, B; };

template <int U, int B, int ORDER>
static Var var()
{
    Var v;
    snprintf(v.name, sizeof v.name, "U%d B%d %s", U, B, ORDER ? "chunk-major" : "leaf-major");
    v.f = k_tree8<U, B, ORDER>;
    v.U = U; v.B = B;
    return v;
}

int main(int argc, char **argv)
{
    long leaf_mib = argc > 1 ? atol(argv[1]) : 32;
    const long leaf = leaf_mib << 20;
    const int sets = leaf_mib <= 64 ? 4 : 2;
    int ncu = 0;
    CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    std::vector<Var> vars = { var<1, 256, 1>(), var<2, 256, 1>(), var<2, 256, 0>(), var<4, 256, 1>(),
                              var<1, 512, 1>(), var<2, 512, 1>(), var<1, 1024, 1>(), var<2, 128, 1>() };
    const long stags[] = {0, 4096, 65536 + 4096, (1L << 20) + 4096};
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
    for (long stag : stags) {
        std::vector<P8> ps(sets);
        std::vector<char *> bigs;
        for (auto &p : ps) {
            char *big;
            CHECK(hipMalloc(&big, 8 * (leaf + stag) + leaf));
            CHECK(hipMemset(big, 0x3c, 8 * (leaf + stag) + leaf));
            bigs.push_back(big);
            for (int q = 0; q < 8; ++q) p.s[q] = (const f32x4 *)(big + q * (leaf + stag));
            p.d = (f32x4 *)(big + 8 * (leaf + stag));
            p.nvec = leaf / 16;
            p.xcd = 0;
        }
        for (int grid = 0; grid < 2; ++grid)
            for (int xcd = 0; xcd < 2; ++xcd)
                for (auto &v : vars) {
                    if (stag != 4096 && (grid || xcd)) continue;   // layout sweep on the default launch only
                    long blocks = (ps[0].nvec + (long)v.B * v.U - 1) / ((long)v.B * v.U);
                    int occ = 0;
                    CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, (const void *)v.f, v.B, 0));
                    if (grid) blocks = std::min(blocks, (long)ncu * occ);
                    blocks = (blocks + 7) / 8 * 8;
                    for (auto &p : ps) p.xcd = xcd;
                    std::vector<float> t;
                    for (int r = 0; r < 5; ++r) {
                        for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(v.f, dim3(blocks), dim3(v.B), 0, 0, ps[w % sets]);
                        CHECK(hipEventRecord(e0, 0));
                        for (int i = 0; i < 20; ++i) hipLaunchKernelGGL(v.f, dim3(blocks), dim3(v.B), 0, 0, ps[i % sets]);
                        CHECK(hipEventRecord(e1, 0));
                        CHECK(hipEventSynchronize(e1));
                        float ms;
                        CHECK(hipEventElapsedTime(&ms, e0, e1));
                        t.push_back(ms / 20);
                    }
                    std::sort(t.begin(), t.end());
                    const double med = t[t.size() / 2], bytes = 9.0 * leaf;
                    printf("{\"leaf_mib\": %ld, \"stagger\": %ld, \"variant\": \"%s\", \"grid\": \"%s\", \"xcd_remap\": %d, "
                           "\"blocks\": %ld, \"occupancy_blocks_per_cu\": %d, \"us\": %.2f, \"frac\": %.4f}\n",
                           leaf_mib, stag, v.name, grid ? "persistent" : "one-pass", xcd, blocks, occ, med * 1e3,
                           bytes / (med * 1e-3) / 8e12);
                    fflush(stdout);
                }
        for (char *b : bigs) CHECK(hipFree(b));
    }
    return 0;
}
