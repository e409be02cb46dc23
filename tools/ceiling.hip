// ceiling.hip -- libmvx_ceiling.so: the read-only, write-only and copy rates
// of this GPU's HBM over the bench's own buffers, so bench.py can report the
// config-2 kernel against the measured ceiling of its own 2-read / 1-write
// mix as well as against the 8 TB/s spec peak (DESIGN.md section 5,
// tools/tune_sum3.hip for the sweep that chose these forms: each is the
// fastest form of its stream found there).  Measurement helper only; the
// product never loads it.
//
//   int mvx_ceiling_run(int mode, void *const *a, void *const *b, int sets,
//                       size_t bytes, int reps, void *stream, float *us)
//     mode 0  read a[s] and b[s] (2 x bytes per launch; U = 4, nt loads)
//     mode 1  write b[s]           (1 x bytes; one 16-byte nt store per lane)
//     mode 2  copy a[s] -> b[s]    (2 x bytes; U = 4, nt)
//   sets rotate launch by launch; *us = mean launch time over `reps`
//   launches between two events on `stream`, after 2 untimed launches.
//   bytes must be a multiple of 16 KiB.  Returns 0, or -1 on a bad argument
//   or a HIP error.
#include <hip/hip_runtime.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ void __launch_bounds__(256) k_read2(const f32x4 *__restrict__ a, const f32x4 *__restrict__ b,
                                               f32x4 *__restrict__ sink, long nvec)
{
    const long c0 = (long)blockIdx.x * 1024 + threadIdx.x;
    f32x4 x[4], y[4], acc = {0, 0, 0, 0};
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        x[u] = __builtin_nontemporal_load(a + c0 + u * 256);
        y[u] = __builtin_nontemporal_load(b + c0 + u * 256);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) acc += x[u] + y[u];
    if (acc.x == 1234.5f && acc.y == -1234.5f) sink[threadIdx.x] = acc;   // keeps the loads
    (void)nvec;
}

__global__ void __launch_bounds__(256) k_write1(f32x4 *__restrict__ b, long nvec)
{
    const f32x4 v = {1.f, 2.f, 3.f, (float)blockIdx.x};
    __builtin_nontemporal_store(v, b + (long)blockIdx.x * 256 + threadIdx.x);
    (void)nvec;
}

__global__ void __launch_bounds__(256) k_copy(const f32x4 *__restrict__ a, f32x4 *__restrict__ b, long nvec)
{
    const long c0 = (long)blockIdx.x * 1024 + threadIdx.x;
    f32x4 x[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) x[u] = __builtin_nontemporal_load(a + c0 + u * 256);
#pragma unroll
    for (int u = 0; u < 4; ++u) __builtin_nontemporal_store(x[u], b + c0 + u * 256);
    (void)nvec;
}

static hipError_t launch(int mode, void *a, void *b, long nvec, hipStream_t st)
{
    if (mode == 0)
        hipLaunchKernelGGL(k_read2, dim3(nvec / 1024), dim3(256), 0, st, (const f32x4 *)a, (const f32x4 *)b,
                           (f32x4 *)b, nvec);
    else if (mode == 1)
        hipLaunchKernelGGL(k_write1, dim3(nvec / 256), dim3(256), 0, st, (f32x4 *)b, nvec);
    else
        hipLaunchKernelGGL(k_copy, dim3(nvec / 1024), dim3(256), 0, st, (const f32x4 *)a, (f32x4 *)b, nvec);
    return hipGetLastError();
}

extern "C" int mvx_ceiling_run(int mode, void *const *a, void *const *b, int sets, size_t bytes, int reps,
                               void *stream, float *us)
{
    if (mode < 0 || mode > 2 || !a || !b || sets < 1 || reps < 1 || !us || !bytes || bytes % (16 << 10))
        return -1;
    for (int s = 0; s < sets; ++s)
        if (!a[s] || !b[s] || ((size_t)a[s] | (size_t)b[s]) % 16) return -1;
    const long nvec = (long)(bytes / 16);
    hipStream_t st = (hipStream_t)stream;
    hipEvent_t e0, e1;
    if (hipEventCreate(&e0) != hipSuccess) return -1;
    if (hipEventCreate(&e1) != hipSuccess) { (void)hipEventDestroy(e0); return -1; }
    int rc = 0;
    for (int w = 0; w < 2 && !rc; ++w) rc = launch(mode, a[w % sets], b[w % sets], nvec, st) != hipSuccess;
    if (!rc) rc = hipEventRecord(e0, st) != hipSuccess;
    for (int i = 0; i < reps && !rc; ++i) rc = launch(mode, a[i % sets], b[i % sets], nvec, st) != hipSuccess;
    if (!rc) rc = hipEventRecord(e1, st) != hipSuccess;
    float ms = 0;
    if (!rc) rc = hipEventSynchronize(e1) != hipSuccess || hipEventElapsedTime(&ms, e0, e1) != hipSuccess;
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    if (rc) return -1;
    *us = ms * 1e3f / (float)reps;
    return 0;
}
