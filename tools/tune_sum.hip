// tune_sum.hip -- standalone sweep of launch/streaming variants of the
// 2-operand f32 SUM kernel (the config-2 hot kernel) on one MI355X.
// Variants are timed interleaved in one process (guide rule 24).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include <algorithm>

typedef float f32x4 __attribute__((ext_vector_type(4)));

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

template <int U, int NTL, int NTS, int CONTIG>
__global__ void __launch_bounds__(256) k_sum(const f32x4 *__restrict__ in, f32x4 *__restrict__ io, long nvec)
{
    const long nthr = (long)gridDim.x * 256;
    if (CONTIG) {   // each block streams one contiguous slab
        const long per = (nvec + gridDim.x - 1) / gridDim.x;
        const long lo = blockIdx.x * per;
        const long hi = lo + per < nvec ? lo + per : nvec;
        for (long c0 = lo + threadIdx.x; c0 < hi; c0 += 256 * U) {
            f32x4 a[U], b[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                long c = c0 + u * 256;
                if (c < hi) {
                    a[u] = NTL ? __builtin_nontemporal_load(&io[c]) : io[c];
                    b[u] = NTL ? __builtin_nontemporal_load(&in[c]) : in[c];
                }
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                long c = c0 + u * 256;
                if (c < hi) {
                    f32x4 r = a[u] + b[u];
                    if (NTS) __builtin_nontemporal_store(r, &io[c]); else io[c] = r;
                }
            }
        }
        return;
    }
    for (long c0 = (long)blockIdx.x * 256 * U + threadIdx.x; c0 < nvec; c0 += nthr * U) {
        f32x4 a[U], b[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            long c = c0 + u * 256;
            if (c < nvec) {
                a[u] = NTL ? __builtin_nontemporal_load(&io[c]) : io[c];
                b[u] = NTL ? __builtin_nontemporal_load(&in[c]) : in[c];
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            long c = c0 + u * 256;
            if (c < nvec) {
                f32x4 r = a[u] + b[u];
                if (NTS) __builtin_nontemporal_store(r, &io[c]); else io[c] = r;
            }
        }
    }
}

typedef void (*KF)(const f32x4 *, f32x4 *, long);
struct Var { const char *name; KF f; int U; };

#define V(U, L, S, C) { "U" #U " ntl" #L " nts" #S " contig" #C, k_sum<U, L, S, C>, U }

int main(int argc, char **argv)
{
    const long nbytes = 256L << 20, n = nbytes / 4, nvec = n / 4;
    // NB buffer pairs, used round-robin: 2 GiB working set, so neither
    // operand of a launch can still sit in the 256 MiB Infinity Cache
    const int NB = argc > 1 ? atoi(argv[1]) : 4;
    std::vector<f32x4 *> ins(NB), ios(NB);
    for (int b = 0; b < NB; ++b) {
        CHECK(hipMalloc(&ins[b], nbytes));
        CHECK(hipMalloc(&ios[b], nbytes));
        CHECK(hipMemset(ins[b], 0x3c, nbytes));
        CHECK(hipMemset(ios[b], 0x3d, nbytes));
    }
    Var vars[] = {
        V(1, 0, 0, 0), V(2, 0, 0, 0), V(4, 0, 0, 0), V(8, 0, 0, 0),
        V(4, 1, 0, 0), V(4, 0, 1, 0), V(4, 1, 1, 0), V(8, 1, 1, 0), V(2, 1, 1, 0),
        V(4, 0, 0, 1), V(4, 1, 1, 1), V(8, 0, 0, 1), V(1, 1, 0, 0), V(1, 1, 1, 0), V(2, 1, 0, 0),
    };
    const int grids[] = {1024, 2048, 4096, 8192, 16384, 0};  // 0: exact (one pass)
    const int NV = sizeof(vars) / sizeof(vars[0]), NG = sizeof(grids) / sizeof(grids[0]);
    const int reps = 20, rounds = 5;
    std::vector<std::vector<float>> t(NV * NG);
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    for (int r = 0; r < rounds; ++r) {
        for (int v = 0; v < NV; ++v) {
            for (int g = 0; g < NG; ++g) {
                long blocks = grids[g] ? grids[g] : (nvec + 256L * vars[v].U - 1) / (256L * vars[v].U);
                for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(vars[v].f, dim3(blocks), dim3(256), 0, 0, ins[w % NB], ios[w % NB], nvec);
                CHECK(hipEventRecord(e0, 0));
                for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(vars[v].f, dim3(blocks), dim3(256), 0, 0, ins[i % NB], ios[i % NB], nvec);
                CHECK(hipEventRecord(e1, 0));
                CHECK(hipEventSynchronize(e1));
                float ms;
                CHECK(hipEventElapsedTime(&ms, e0, e1));
                t[v * NG + g].push_back(ms / reps);
            }
        }
        fprintf(stderr, "round %d done\n", r);
    }
    printf("%-28s %7s %9s %9s %8s\n", "variant", "grid", "med_us", "min_us", "TB/s");
    for (int v = 0; v < NV; ++v)
        for (int g = 0; g < NG; ++g) {
            auto x = t[v * NG + g];
            std::sort(x.begin(), x.end());
            float med = x[x.size() / 2], mn = x[0];
            printf("%-28s %7d %9.1f %9.1f %8.3f\n", vars[v].name, grids[g], med * 1e3, mn * 1e3, 3.0 * nbytes / (med * 1e-3) / 1e12);
        }
    return 0;
}
