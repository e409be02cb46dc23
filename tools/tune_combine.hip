// tune_combine.hip -- sweep unroll / block size of the k-leaf f32 SUM tree
// (config-3 shape: 8 leaves of 32 MiB -> 32 MiB; config-4 shape: 4 x 256 MiB).
// Rotating buffer sets keep every launch out of the Infinity Cache.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include <algorithm>

typedef float f32x4 __attribute__((ext_vector_type(4)));
#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

struct P8 { const f32x4 *s[8]; f32x4 *d; long nvec; };

template <int K, int U, int B>
__global__ void __launch_bounds__(B) k_tree(P8 p)
{
    const long nthr = (long)gridDim.x * B;
    for (long c0 = (long)blockIdx.x * B * U + threadIdx.x; c0 < p.nvec; c0 += nthr * U) {
        f32x4 x[U][K];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            long c = c0 + (long)u * B;
            if (c < p.nvec) {
#pragma unroll
                for (int q = 0; q < K; ++q) x[u][q] = __builtin_nontemporal_load(p.s[q] + c);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            long c = c0 + (long)u * B;
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
struct Var { const char *name; KF f; int U, B, K; };
#define V(K, U, B) { "K" #K " U" #U " B" #B, k_tree<K, U, B>, U, B, K }

int main()
{
    struct Shape { int K; long leaf; int sets; } shapes[] = {{8, 32L << 20, 4}, {4, 256L << 20, 2}, {8, 64L << 20, 2}};
    Var vars[] = { V(8, 1, 256), V(8, 2, 256), V(8, 4, 256), V(8, 1, 512), V(8, 2, 512), V(8, 1, 128), V(8, 2, 128),
                   V(4, 1, 256), V(4, 2, 256), V(4, 4, 256), V(4, 2, 512) };
    const int NV = sizeof(vars) / sizeof(vars[0]);
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
    for (auto &sh : shapes) {
        std::vector<P8> sets(sh.sets);
        for (auto &ps : sets) {
            for (int q = 0; q < sh.K; ++q) { f32x4 *b; CHECK(hipMalloc(&b, sh.leaf)); CHECK(hipMemset(b, 0x3c, sh.leaf)); ps.s[q] = b; }
            CHECK(hipMalloc(&ps.d, sh.leaf));
            ps.nvec = sh.leaf / 16;
        }
        std::vector<std::vector<float>> t(NV);
        for (int r = 0; r < 5; ++r)
            for (int v = 0; v < NV; ++v) {
                if (vars[v].K != sh.K) continue;
                long blocks = (sets[0].nvec + (long)vars[v].B * vars[v].U - 1) / ((long)vars[v].B * vars[v].U);
                for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(vars[v].f, dim3(blocks), dim3(vars[v].B), 0, 0, sets[w % sh.sets]);
                CHECK(hipEventRecord(e0, 0));
                for (int i = 0; i < 20; ++i) hipLaunchKernelGGL(vars[v].f, dim3(blocks), dim3(vars[v].B), 0, 0, sets[i % sh.sets]);
                CHECK(hipEventRecord(e1, 0)); CHECK(hipEventSynchronize(e1));
                float ms; CHECK(hipEventElapsedTime(&ms, e0, e1)); t[v].push_back(ms / 20);
            }
        for (int v = 0; v < NV; ++v) {
            if (t[v].empty()) continue;
            std::sort(t[v].begin(), t[v].end());
            float med = t[v][t[v].size() / 2];
            double bytes = (double)(sh.K + 1) * sh.leaf;
            printf("leaf %4ld MiB  %-14s med %8.1f us  %6.3f TB/s\n", sh.leaf >> 20, vars[v].name, med * 1e3, bytes / (med * 1e-3) / 1e12);
        }
        for (auto &ps : sets) { for (int q = 0; q < sh.K; ++q) hipFree((void *)ps.s[q]); hipFree(ps.d); }
    }
    return 0;
}
