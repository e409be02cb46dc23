// zc_window.hip -- does the zero-copy op read registered (hipHostRegister'ed
// malloc) pages slower than hipHostMalloc'd ones because of address
// translation, and does a smaller window of pages in flight help?  The
// 256 MiB SUM float32 op (two host operands read, one written, all over
// PCIe) with the grid capped at B workgroups (each streaming its share in
// 16 KiB steps) for both kinds of memory.  Measurement probe only.
//   ./zc_window > out.jsonl
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <algorithm>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));
#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

// block-contiguous: workgroup b takes chunks [b * per, (b + 1) * per), 4 per lane in flight
__global__ void __launch_bounds__(256) k_sum_blocked(const f32x4 *__restrict__ in, f32x4 *__restrict__ io, long nvec,
                                                      long per)
{
    const long lo = (long)blockIdx.x * per, hi = lo + per < nvec ? lo + per : nvec;
    for (long c0 = lo + threadIdx.x; c0 < hi; c0 += 1024) {
        f32x4 a[4], b[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const long c = c0 + u * 256;
            if (c < hi) { a[u] = io[c]; b[u] = in[c]; }
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const long c = c0 + u * 256;
            if (c < hi) io[c] = a[u] + b[u];
        }
    }
}

// grid-stride: the whole grid sweeps the vector front to back (a window of
// grid * 16 KiB per operand in flight)
__global__ void __launch_bounds__(256) k_sum_stride(const f32x4 *__restrict__ in, f32x4 *__restrict__ io, long nvec)
{
    const long nthr = (long)gridDim.x * 256;
    for (long c0 = (long)blockIdx.x * 1024 + threadIdx.x; c0 < nvec; c0 += nthr * 4) {
        f32x4 a[4], b[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const long c = c0 + u * 256;
            if (c < nvec) { a[u] = io[c]; b[u] = in[c]; }
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const long c = c0 + u * 256;
            if (c < nvec) io[c] = a[u] + b[u];
        }
    }
}

static double run(int mode, int grid, const f32x4 *in, f32x4 *io, long nvec, hipStream_t st)
{
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    std::vector<float> t;
    for (int r = 0; r < 7; ++r) {
        CHECK(hipEventRecord(e0, st));
        if (mode == 0) {
            const long per = (nvec + grid - 1) / grid;
            hipLaunchKernelGGL(k_sum_blocked, dim3(grid), dim3(256), 0, st, in, io, nvec, per);
        } else {
            hipLaunchKernelGGL(k_sum_stride, dim3(grid), dim3(256), 0, st, in, io, nvec);
        }
        CHECK(hipEventRecord(e1, st));
        CHECK(hipEventSynchronize(e1));
        float ms;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        if (r) t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    CHECK(hipEventDestroy(e0));
    CHECK(hipEventDestroy(e1));
    return t[t.size() / 2];
}

int main()
{
    const size_t nbytes = 256ul << 20;
    const long nvec = (long)(nbytes / 16);
    hipStream_t st;
    CHECK(hipStreamCreate(&st));
    for (int kind = 0; kind < 2; ++kind) {
        float *a, *b;
        if (kind == 0) {
            CHECK(hipHostMalloc((void **)&a, nbytes, hipHostMallocDefault));
            CHECK(hipHostMalloc((void **)&b, nbytes, hipHostMallocDefault));
        } else {
            if (posix_memalign((void **)&a, 4096, nbytes) || posix_memalign((void **)&b, 4096, nbytes)) return 1;
            memset(a, 0, nbytes);
            memset(b, 0, nbytes);
            CHECK(hipHostRegister(a, nbytes, hipHostRegisterDefault));
            CHECK(hipHostRegister(b, nbytes, hipHostRegisterDefault));
        }
        for (size_t i = 0; i < nbytes / 4; ++i) { a[i] = 1.0f; b[i] = 2.0f; }
        const int grids[6] = {128, 256, 512, 1024, 2048, 16384};
        for (int mode = 0; mode < 2; ++mode)
            for (int gi = 0; gi < 6; ++gi) {
                const int g = grids[gi];
                const double ms = run(mode, g, (const f32x4 *)a, (f32x4 *)b, nvec, st);
                printf("{\"memory\": \"%s\", \"order\": \"%s\", \"grid\": %d, \"ms\": %.3f, \"GBs\": %.1f}\n",
                       kind ? "registered" : "hipHostMalloc", mode ? "stride" : "blocked", g, ms, 3.0 * nbytes / ms / 1e6);
                fflush(stdout);
            }
        if (kind == 0) {
            CHECK(hipHostFree(a));
            CHECK(hipHostFree(b));
        } else {
            CHECK(hipHostUnregister(a));
            CHECK(hipHostUnregister(b));
            free(a);
            free(b);
        }
    }
    return 0;
}
