// tune_occ.hip -- does the k = 8 combine (C3 / C5 shape) run faster with
// FEWER bytes in flight?  At full occupancy the fixed-tree kernel keeps about
// 75 MB of loads outstanding (512 Ki resident lanes x 9 streams x 16 B),
// ten times what Little's law needs at 8 TB/s, and every HBM channel then
// juggles rows from 9 streams.  This caps the resident blocks per CU with
// dynamic LDS (160 KiB per CU / bytes per block) and sweeps:
//   OCC    resident 256-thread blocks per CU: 1, 2, 3, 4, 6, 8 (0 = uncapped)
//   GRID   one pass over the data, or persistent (CUs x OCC blocks, grid-stride)
//   U      16-byte chunks per lane per leaf in flight: 1, 2, 3, 4, 6
// for k = 8 (8 x 32 MiB -> 32 MiB, SUM f32, tree order) and, as a control,
// k = 2 (256 MiB SUM f32, the C2 kernel's shape).  Rotating buffer sets keep
// launches out of the Infinity Cache.  One JSON line per variant: median of
// 5 rounds x 20 launches (HIP events).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <vector>

#include "mvx_hip.h"   // the product's combine (libmvx_hip.so) on the same buffers

typedef float f32x4 __attribute__((ext_vector_type(4)));
#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

struct P8 { const f32x4 *s[8]; f32x4 *d; long nvec; };

template <int K, int U>
__global__ void __launch_bounds__(256) k_tree(P8 p)
{
    extern __shared__ char lds_cap[];   // only there to cap residency
    if (p.nvec < 0) lds_cap[threadIdx.x] = 0;
    const long nthr = (long)gridDim.x * 256;
    for (long c0 = (long)blockIdx.x * 256 * U + threadIdx.x; c0 < p.nvec; c0 += nthr * U) {
        f32x4 x[U][K];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long c = c0 + (long)u * 256;
            if (c < p.nvec)
#pragma unroll
                for (int q = 0; q < K; ++q) x[u][q] = __builtin_nontemporal_load(p.s[q] + c);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long c = c0 + (long)u * 256;
            if (c < p.nvec) {
#pragma unroll
                for (int h = 1; h < K; h <<= 1)
#pragma unroll
                    for (int q = 0; q + h < K; q += 2 * h) x[u][q] = x[u][q] + x[u][q + h];
                __builtin_nontemporal_store(x[u][0], p.d + c);
            }
        }
    }
}

// the same loop with the residency cap as 52 KiB of static LDS (what the
// product's k_tree_body does) instead of a dynamic reservation at launch
template <int K, int U>
__global__ void __launch_bounds__(256) k_tree_static(P8 p)
{
    __shared__ char lds_cap[52 * 1024];
    if (p.nvec < 0) lds_cap[threadIdx.x] = 0;
    const long nthr = (long)gridDim.x * 256;
    for (long c0 = (long)blockIdx.x * 256 * U + threadIdx.x; c0 < p.nvec; c0 += nthr * U) {
        f32x4 x[U][K];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long c = c0 + (long)u * 256;
            if (c < p.nvec)
#pragma unroll
                for (int q = 0; q < K; ++q) x[u][q] = __builtin_nontemporal_load(p.s[q] + c);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long c = c0 + (long)u * 256;
            if (c < p.nvec) {
#pragma unroll
                for (int h = 1; h < K; h <<= 1)
#pragma unroll
                    for (int q = 0; q + h < K; q += 2 * h) x[u][q] = x[u][q] + x[u][q + h];
                __builtin_nontemporal_store(x[u][0], p.d + c);
            }
        }
    }
}

typedef void (*KF)(P8);

int main(int argc, char **argv)
{
    int ncu = 0;
    CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    struct Shape { int k; long leaf; int sets; };
    const Shape shapes[] = { {8, 32L << 20, 4}, {8, 64L << 20, 2}, {2, 256L << 20, 4} };
    const long stag = 4096;
    for (const Shape &sh : shapes) {
        std::vector<P8> ps(sh.sets);
        std::vector<char *> bigs;
        for (auto &p : ps) {
            char *big;
            const size_t bytes = (size_t)(sh.k + 1) * (sh.leaf + stag);
            CHECK(hipMalloc(&big, bytes));
            CHECK(hipMemset(big, 0x3c, bytes));
            bigs.push_back(big);
            for (int q = 0; q < 8; ++q) p.s[q] = (const f32x4 *)(big + (q < sh.k ? q : 0) * (sh.leaf + stag));
            p.d = (f32x4 *)(big + sh.k * (sh.leaf + stag));
            if (getenv("DST_SEPARATE")) {       // the result in its own allocation (the product's recvbuf)
                char *d;
                CHECK(hipMalloc(&d, sh.leaf));
                bigs.push_back(d);
                p.d = (f32x4 *)d;
            }
            p.nvec = sh.leaf / 16;
        }
        const int Us[] = {1, 2, 4};
        for (int U : Us) {
            if (getenv("PRODUCT_ONLY")) break;
            KF f = sh.k == 8 ? (U == 1 ? k_tree<8, 1> : U == 2 ? k_tree<8, 2> : U == 3 ? k_tree<8, 3> : U == 4 ? k_tree<8, 4> : k_tree<8, 6>)
                             : (U == 1 ? k_tree<2, 1> : U == 2 ? k_tree<2, 2> : U == 3 ? k_tree<2, 3> : U == 4 ? k_tree<2, 4> : k_tree<2, 6>);
            const int occs[] = {0, 3};
            for (int grid = 0; grid < 1; ++grid)   // persistent grids lost everywhere (first sweep)
                for (int occ : occs) {
                    if (grid && !occ) continue;
                    if (getenv("ONLY_U2CAP3") && (U != 2 || occ != 3)) continue;
                    const size_t lds = occ ? (size_t)(160 * 1024 / occ) & ~(size_t)1023 : 0;
                    if (lds > 64 * 1024 && hipFuncSetAttribute((const void *)f, hipFuncAttributeMaxDynamicSharedMemorySize,
                                                               (int)lds) != hipSuccess) {
                        (void)hipGetLastError();
                        continue;
                    }
                    int real = 0;
                    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&real, (const void *)f, 256, lds) != hipSuccess) {
                        (void)hipGetLastError();
                        continue;
                    }
                    long blocks = (ps[0].nvec + 256L * U - 1) / (256L * U);
                    if (grid) blocks = std::min(blocks, (long)ncu * real);
                    std::vector<float> t;
                    bool bad = false;
                    for (int r = 0; r < 5 && !bad; ++r) {
                        for (int w = 0; w < 3; ++w)
                            hipLaunchKernelGGL(f, dim3(blocks), dim3(256), lds, 0, ps[w % sh.sets]);
                        if (hipGetLastError() != hipSuccess) { bad = true; break; }
                        CHECK(hipEventRecord(e0, 0));
                        for (int i = 0; i < 20; ++i)
                            hipLaunchKernelGGL(f, dim3(blocks), dim3(256), lds, 0, ps[i % sh.sets]);
                        CHECK(hipEventRecord(e1, 0));
                        CHECK(hipEventSynchronize(e1));
                        float ms;
                        CHECK(hipEventElapsedTime(&ms, e0, e1));
                        t.push_back(ms / 20);
                    }
                    if (bad) continue;
                    std::sort(t.begin(), t.end());
                    const double med = t[t.size() / 2], bytes = (double)(sh.k + 1) * sh.leaf;
                    printf("{\"k\": %d, \"leaf_mib\": %ld, \"U\": %d, \"grid\": \"%s\", \"occ_cap\": %d, "
                           "\"blocks_per_cu\": %d, \"lds\": %zu, \"blocks\": %ld, \"us\": %.2f, \"frac\": %.4f}\n",
                           sh.k, sh.leaf >> 20, U, grid ? "persistent" : "one-pass", occ, real, lds, blocks,
                           med * 1e3, bytes / (med * 1e-3) / 8e12);
                    fflush(stdout);
                }
        }
        if (sh.k == 2 && getenv("K2_SWEEP")) {   // the plain op: U x resident blocks (by LDS reservation)
            const int kib[] = {0, 36, 44, 56, 88};   // ~ 8 (regs), 4, 3, 2, 1 blocks per CU
            KF fs[] = {k_tree<2, 1>, k_tree<2, 2>, k_tree<2, 3>, k_tree<2, 4>, k_tree<2, 6>};
            const int us[] = {1, 2, 3, 4, 6};
            for (int ui = 0; ui < 5; ++ui)
                for (int kb : kib) {
                    KF f = fs[ui];
                    const size_t lds = (size_t)kb * 1024;
                    if (lds > 64 * 1024 && hipFuncSetAttribute((const void *)f, hipFuncAttributeMaxDynamicSharedMemorySize,
                                                               (int)lds) != hipSuccess) {
                        (void)hipGetLastError();
                        continue;
                    }
                    int real = 0;
                    CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&real, (const void *)f, 256, lds));
                    std::vector<float> t;
                    const long blocks = (ps[0].nvec + 256L * us[ui] - 1) / (256L * us[ui]);
                    for (int r = 0; r < 5; ++r) {
                        for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(f, dim3(blocks), dim3(256), lds, 0, ps[w % sh.sets]);
                        CHECK(hipEventRecord(e0, 0));
                        for (int i = 0; i < 20; ++i) hipLaunchKernelGGL(f, dim3(blocks), dim3(256), lds, 0, ps[i % sh.sets]);
                        CHECK(hipEventRecord(e1, 0));
                        CHECK(hipEventSynchronize(e1));
                        float ms;
                        CHECK(hipEventElapsedTime(&ms, e0, e1));
                        t.push_back(ms / 20);
                    }
                    std::sort(t.begin(), t.end());
                    const double med = t[t.size() / 2], bytes = (double)(sh.k + 1) * sh.leaf;
                    printf("{\"k\": 2, \"leaf_mib\": %ld, \"variant\": \"U%d lds %d KiB\", \"blocks_per_cu\": %d, "
                           "\"us\": %.2f, \"frac\": %.4f}\n", sh.leaf >> 20, us[ui], kb, real, med * 1e3,
                           bytes / (med * 1e-3) / 8e12);
                    fflush(stdout);
                }
        }
        if (sh.k == 8 && getenv("LDS_SWEEP")) {   // U = 2, dynamic LDS from 24 to 80 KiB
            const int kib[] = {24, 32, 40, 41, 44, 48, 50, 52, 53, 54, 56, 60, 64, 72, 80};
            for (int kb : kib) {
                const size_t lds = (size_t)kb * 1024;
                if (lds > 64 * 1024 && hipFuncSetAttribute((const void *)k_tree<8, 2>,
                                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess) {
                    (void)hipGetLastError();
                    continue;
                }
                int real = 0;
                CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&real, (const void *)k_tree<8, 2>, 256, lds));
                std::vector<float> t;
                const long blocks = ps[0].nvec / 512;
                for (int r = 0; r < 5; ++r) {
                    for (int w = 0; w < 3; ++w) hipLaunchKernelGGL((k_tree<8, 2>), dim3(blocks), dim3(256), lds, 0, ps[w % sh.sets]);
                    CHECK(hipEventRecord(e0, 0));
                    for (int i = 0; i < 20; ++i) hipLaunchKernelGGL((k_tree<8, 2>), dim3(blocks), dim3(256), lds, 0, ps[i % sh.sets]);
                    CHECK(hipEventRecord(e1, 0));
                    CHECK(hipEventSynchronize(e1));
                    float ms;
                    CHECK(hipEventElapsedTime(&ms, e0, e1));
                    t.push_back(ms / 20);
                }
                std::sort(t.begin(), t.end());
                const double med = t[t.size() / 2], bytes = (double)(sh.k + 1) * sh.leaf;
                printf("{\"k\": %d, \"leaf_mib\": %ld, \"variant\": \"U2 dynamic lds %d KiB\", \"blocks_per_cu\": %d, "
                       "\"us\": %.2f, \"frac\": %.4f}\n", sh.k, sh.leaf >> 20, kb, real, med * 1e3,
                       bytes / (med * 1e-3) / 8e12);
                fflush(stdout);
            }
        }
        if (sh.k == 8) {   // static-LDS variant of U = 2
            std::vector<float> t;
            const long blocks = ps[0].nvec / 512;
            for (int r = 0; r < 5; ++r) {
                for (int w = 0; w < 3; ++w) hipLaunchKernelGGL((k_tree_static<8, 2>), dim3(blocks), dim3(256), 0, 0, ps[w % sh.sets]);
                CHECK(hipEventRecord(e0, 0));
                for (int i = 0; i < 20; ++i) hipLaunchKernelGGL((k_tree_static<8, 2>), dim3(blocks), dim3(256), 0, 0, ps[i % sh.sets]);
                CHECK(hipEventRecord(e1, 0));
                CHECK(hipEventSynchronize(e1));
                float ms;
                CHECK(hipEventElapsedTime(&ms, e0, e1));
                t.push_back(ms / 20);
            }
            std::sort(t.begin(), t.end());
            const double med = t[t.size() / 2], bytes = (double)(sh.k + 1) * sh.leaf;
            printf("{\"k\": %d, \"leaf_mib\": %ld, \"variant\": \"static-lds U2\", \"us\": %.2f, \"frac\": %.4f}\n",
                   sh.k, sh.leaf >> 20, med * 1e3, bytes / (med * 1e-3) / 8e12);
        }
        {   // the product kernel (mvx_op_combine: the launched template and
            // residency of libmvx_hip.so) on exactly these buffers
            std::vector<float> t;
            for (int r = 0; r < 5; ++r) {
                for (int w = 0; w < 3; ++w) {
                    const P8 &p = ps[w % sh.sets];
                    if (mvx_op_combine(102, 10, (const void *const *)p.s, nullptr, sh.k, MVX_SHAPE_TREE, p.d,
                                       (size_t)p.nvec * 4, nullptr)) { printf("combine failed\n"); exit(1); }
                }
                CHECK(hipEventRecord(e0, 0));
                for (int i = 0; i < 20; ++i) {
                    const P8 &p = ps[i % sh.sets];
                    mvx_op_combine(102, 10, (const void *const *)p.s, nullptr, sh.k, MVX_SHAPE_TREE, p.d,
                                   (size_t)p.nvec * 4, nullptr);
                }
                CHECK(hipEventRecord(e1, 0));
                CHECK(hipEventSynchronize(e1));
                float ms;
                CHECK(hipEventElapsedTime(&ms, e0, e1));
                t.push_back(ms / 20);
            }
            std::sort(t.begin(), t.end());
            const double med = t[t.size() / 2], bytes = (double)(sh.k + 1) * sh.leaf;
            unsigned lb = 0;
            size_t ll = 0;
            int locc = 0;
            mvx_hip_last_launch(&lb, &ll, &locc);
            printf("{\"k\": %d, \"leaf_mib\": %ld, \"variant\": \"product %s\", \"blocks\": %u, \"lds\": %zu, "
                   "\"blocks_per_cu\": %d, \"us\": %.2f, \"frac\": %.4f}\n",
                   sh.k, sh.leaf >> 20, mvx_hip_last_kernel_symbol(), lb, ll, locc, med * 1e3, bytes / (med * 1e-3) / 8e12);
            fflush(stdout);
        }
        for (char *b : bigs) CHECK(hipFree(b));
    }
    return 0;
}
