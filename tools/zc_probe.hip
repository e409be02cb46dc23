// zc_probe.hip -- can the op on page-locked host operands skip the DMA
// engines?  A kernel reads both operands straight from page-locked host
// memory over PCIe and writes the result straight back (zero-copy), against
// the product's DMA pipeline (csrc/mvx_hostop.c: 2 H2D + kernel + 1 D2H,
// 10.9 ms at 256 MiB).  Also the one-direction rates a kernel reaches:
// host -> HBM (read over PCIe), HBM -> host (write over PCIe).
// Buffers come from hipHostMalloc (device-accessible by construction).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <algorithm>
#include <chrono>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));
#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

template <int U>
__global__ void __launch_bounds__(256) k_sum(const f32x4 *__restrict__ in, f32x4 *__restrict__ io, long nvec)
{
    const long nthr = (long)gridDim.x * 256;
    for (long c0 = (long)blockIdx.x * 256 * U + threadIdx.x; c0 < nvec; c0 += nthr * U) {
        f32x4 a[U], b[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            long c = c0 + u * 256;
            if (c < nvec) { a[u] = io[c]; b[u] = in[c]; }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            long c = c0 + u * 256;
            if (c < nvec) io[c] = a[u] + b[u];
        }
    }
}

template <int U>
__global__ void __launch_bounds__(256) k_copy(const f32x4 *__restrict__ s, f32x4 *__restrict__ d, long nvec)
{
    const long nthr = (long)gridDim.x * 256;
    for (long c0 = (long)blockIdx.x * 256 * U + threadIdx.x; c0 < nvec; c0 += nthr * U) {
        f32x4 a[U];
#pragma unroll
        for (int u = 0; u < U; ++u) if (c0 + u * 256 < nvec) a[u] = s[c0 + u * 256];
#pragma unroll
        for (int u = 0; u < U; ++u) if (c0 + u * 256 < nvec) d[c0 + u * 256] = a[u];
    }
}

typedef void (*KF)(const f32x4 *, f32x4 *, long);

static float time_it(KF f, int U, long grid, const f32x4 *a, f32x4 *b, long nvec, int reps)
{
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    const long blocks = grid ? grid : (nvec + 256L * U - 1) / (256L * U);
    hipLaunchKernelGGL(f, dim3(blocks), dim3(256), 0, 0, a, b, nvec);
    CHECK(hipDeviceSynchronize());
    std::vector<float> t;
    for (int r = 0; r < reps; ++r) {
        CHECK(hipEventRecord(e0, 0));
        hipLaunchKernelGGL(f, dim3(blocks), dim3(256), 0, 0, a, b, nvec);
        CHECK(hipEventRecord(e1, 0));
        CHECK(hipEventSynchronize(e1));
        float ms;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    CHECK(hipEventDestroy(e0));
    CHECK(hipEventDestroy(e1));
    return t[t.size() / 2];
}

int main(int argc, char **argv)
{
    const long nbytes = 256L << 20, nvec = nbytes / 16;
    const int reps = argc > 1 ? atoi(argv[1]) : 5;
    f32x4 *ha, *hb, *da;
    CHECK(hipHostMalloc((void **)&ha, nbytes, hipHostMallocDefault));
    CHECK(hipHostMalloc((void **)&hb, nbytes, hipHostMallocDefault));
    CHECK(hipMalloc((void **)&da, nbytes));
    float *fa = (float *)ha, *fb = (float *)hb;
    for (long i = 0; i < nbytes / 4; ++i) { fa[i] = (float)((i * 7) % 16) - 8.f; fb[i] = (float)((i * 5) % 16) - 8.f; }
    // correctness of the zero-copy op once
    hipLaunchKernelGGL(k_sum<2>, dim3(nvec / 512), dim3(256), 0, 0, ha, hb, nvec);
    CHECK(hipDeviceSynchronize());
    for (long i = 0; i < nbytes / 4; i += 4097)
        if (fb[i] != (float)((i * 7) % 16) - 8.f + (float)((i * 5) % 16) - 8.f) { printf("MISMATCH at %ld\n", i); return 1; }
    printf("zero-copy op correct\n");
    struct { const char *name; KF f; int U; long grid; int what; } vars[] = {
        {"op host->host U1", k_sum<1>, 1, 0, 0},
        {"op host->host U2", k_sum<2>, 2, 0, 0},
        {"op host->host U4", k_sum<4>, 4, 0, 0},
        {"op host->host U2 g1024", k_sum<2>, 2, 1024, 0},
        {"op host->host U2 g4096", k_sum<2>, 2, 4096, 0},
        {"read host->HBM U2", k_copy<2>, 2, 0, 1},
        {"read host->HBM U4", k_copy<4>, 4, 0, 1},
        {"write HBM->host U2", k_copy<2>, 2, 0, 2},
        {"write HBM->host U4", k_copy<4>, 4, 0, 2},
    };
    for (auto &v : vars) {
        const f32x4 *s = v.what == 2 ? da : ha;
        f32x4 *d = v.what == 0 ? hb : v.what == 1 ? da : hb;
        const float ms = time_it(v.f, v.U, v.grid, s, d, nvec, reps);
        const double pcie = (v.what == 0 ? 3.0 : 1.0) * nbytes;
        printf("{\"variant\": \"%s\", \"ms\": %.3f, \"pcie_GBps\": %.1f}\n", v.name, ms, pcie / (ms * 1e-3) / 1e9);
        fflush(stdout);
    }
    // the DMA engines for comparison: one 256 MiB H2D, one D2H, both at once
    {
        hipStream_t s1, s2;
        CHECK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
        CHECK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
        f32x4 *db;
        CHECK(hipMalloc((void **)&db, nbytes));
        for (int mode = 0; mode < 3; ++mode) {
            std::vector<double> t;
            for (int r = 0; r < reps + 1; ++r) {
                CHECK(hipDeviceSynchronize());
                auto t0 = std::chrono::steady_clock::now();
                if (mode != 1) CHECK(hipMemcpyAsync(da, ha, nbytes, hipMemcpyHostToDevice, s1));
                if (mode != 0) CHECK(hipMemcpyAsync(hb, db, nbytes, hipMemcpyDeviceToHost, s2));
                CHECK(hipDeviceSynchronize());
                if (r) t.push_back(std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
            }
            std::sort(t.begin(), t.end());
            const double sec = t[t.size() / 2];
            printf("{\"variant\": \"DMA %s\", \"ms\": %.3f, \"pcie_GBps\": %.1f}\n",
                   mode == 0 ? "H2D 256 MiB" : mode == 1 ? "D2H 256 MiB" : "H2D + D2H 256 MiB each, concurrent",
                   sec * 1e3, (mode == 2 ? 2.0 : 1.0) * nbytes / sec / 1e9);
        }
    }
    return 0;
}
