// tune_sum2.hip -- cache-policy bits and block size for the config-2 kernel.
// Buffer loads/stores with an explicit aux (gfx950 CPol: sc0 = 1, nt = 2,
// sc1 = 16) vs the __builtin_nontemporal form; 4 rotating buffer pairs.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include <algorithm>

typedef float f32x4 __attribute__((ext_vector_type(4)));
#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

template <int U, int B, int LAUX, int SAUX>
__global__ void __launch_bounds__(B) k_buf(const float *in, float *io, long nvec)
{
    // one descriptor per operand (wave-uniform), 32-bit byte offsets (< 4 GiB)
    __amdgpu_buffer_rsrc_t rin = __builtin_amdgcn_make_buffer_rsrc((void *)in, 0, 0x7fffffff, 0x00020000);
    __amdgpu_buffer_rsrc_t rio = __builtin_amdgcn_make_buffer_rsrc((void *)io, 0, 0x7fffffff, 0x00020000);
    const long nthr = (long)gridDim.x * B;
    for (long c0 = (long)blockIdx.x * B * U + threadIdx.x; c0 < nvec; c0 += nthr * U) {
        f32x4 a[U], b[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int off = (int)((c0 + (long)u * B) * 16);
            a[u] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rio, off, 0, LAUX));
            b[u] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rin, off, 0, LAUX));
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int off = (int)((c0 + (long)u * B) * 16);
            f32x4 r = a[u] + b[u];
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, r), rio, off, 0, SAUX);
        }
    }
}

template <int U, int B>
__global__ void __launch_bounds__(B) k_nt(const f32x4 *in, f32x4 *io, long nvec)
{
    const long nthr = (long)gridDim.x * B;
    for (long c0 = (long)blockIdx.x * B * U + threadIdx.x; c0 < nvec; c0 += nthr * U) {
        f32x4 a[U], b[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            long c = c0 + (long)u * B;
            if (c < nvec) { a[u] = __builtin_nontemporal_load(&io[c]); b[u] = __builtin_nontemporal_load(&in[c]); }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            long c = c0 + (long)u * B;
            if (c < nvec) __builtin_nontemporal_store(a[u] + b[u], &io[c]);
        }
    }
}

typedef void (*KF)(const void *, void *, long);
struct Var { const char *name; KF f; int U, B; };
#define VB(U, B, L, S) { "buf U" #U " B" #B " ld" #L " st" #S, (KF)k_buf<U, B, L, S>, U, B }
#define VN(U, B) { "nt U" #U " B" #B, (KF)k_nt<U, B>, U, B }

int main()
{
    const long nbytes = 256L << 20, nvec = nbytes / 16;
    const int NB = 4;
    std::vector<float *> ins(NB), ios(NB);
    for (int b = 0; b < NB; ++b) {
        CHECK(hipMalloc(&ins[b], nbytes)); CHECK(hipMalloc(&ios[b], nbytes));
        CHECK(hipMemset(ins[b], 0x3c, nbytes)); CHECK(hipMemset(ios[b], 0x3d, nbytes));
    }
    Var vars[] = {
        VN(4, 256), VN(4, 512), VN(4, 1024), VN(2, 512), VN(8, 256), VN(4, 128),
        VB(4, 256, 2, 2), VB(4, 256, 0, 0), VB(4, 256, 3, 2), VB(4, 256, 18, 2), VB(4, 256, 2, 18),
        VB(4, 256, 19, 19), VB(4, 256, 16, 16), VB(4, 256, 1, 2), VB(4, 512, 2, 2), VB(8, 256, 2, 2),
    };
    const int NV = sizeof(vars) / sizeof(vars[0]);
    std::vector<std::vector<float>> t(NV);
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
    for (int r = 0; r < 7; ++r)
        for (int v = 0; v < NV; ++v) {
            long blocks = (nvec + (long)vars[v].B * vars[v].U - 1) / ((long)vars[v].B * vars[v].U);
            for (int w = 0; w < 4; ++w) hipLaunchKernelGGL(vars[v].f, dim3(blocks), dim3(vars[v].B), 0, 0, ins[w % NB], ios[w % NB], nvec);
            CHECK(hipEventRecord(e0, 0));
            for (int i = 0; i < 20; ++i) hipLaunchKernelGGL(vars[v].f, dim3(blocks), dim3(vars[v].B), 0, 0, ins[i % NB], ios[i % NB], nvec);
            CHECK(hipEventRecord(e1, 0)); CHECK(hipEventSynchronize(e1));
            float ms; CHECK(hipEventElapsedTime(&ms, e0, e1)); t[v].push_back(ms / 20);
        }
    for (int v = 0; v < NV; ++v) {
        std::sort(t[v].begin(), t[v].end());
        float med = t[v][t[v].size() / 2], mn = t[v][0];
        printf("%-24s med %7.1f us  min %7.1f us  %6.3f TB/s\n", vars[v].name, med * 1e3, mn * 1e3, 3.0 * nbytes / (med * 1e-3) / 1e12);
    }
    return 0;
}
