// tune_sum3.hip -- the config-2 kernel (256 MiB f32 SUM, inout += in) against
// the read-only, write-only and copy ceilings of the same GPU, and the
// load/store forms round 2's sweep (tune_sum.hip) did not try:
//   * buffer loads / stores with explicit cache-policy bits (aux: 1 = sc0,
//     2 = nt, 16 = sc1) instead of global_load ... nt;
//   * LDS-DMA loads (global_load_lds_dwordx4, nt) into a wave-private LDS
//     slab, read back by the same lane.
// Every variant is timed interleaved with the others in one process, over
// NB buffer pairs used round-robin (2 GiB at NB = 4: nothing served from the
// 256 MiB Infinity Cache).  Prints one line per variant: median / min us and
// the rate of the bytes the variant moves.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include <algorithm>
#include <string.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

// production form: global_load/store_dwordx4 ... nt, U chunks per lane in flight
template <int U>
__global__ void __launch_bounds__(256) k_glob(const f32x4 *__restrict__ in, f32x4 *__restrict__ io, long nvec)
{
    const long nthr = (long)gridDim.x * 256;
    for (long c0 = (long)blockIdx.x * 256 * U + threadIdx.x; c0 < nvec; c0 += nthr * U) {
        f32x4 a[U], b[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            long c = c0 + u * 256;
            if (c < nvec) { a[u] = __builtin_nontemporal_load(&io[c]); b[u] = __builtin_nontemporal_load(&in[c]); }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            long c = c0 + u * 256;
            if (c < nvec) __builtin_nontemporal_store(a[u] + b[u], &io[c]);
        }
    }
}

// buffer loads / stores with cache-policy bits LA (loads) and SA (stores)
template <int U, int LA, int SA>
__global__ void __launch_bounds__(256) k_buf(const f32x4 *__restrict__ in, f32x4 *__restrict__ io, long nvec)
{
    const __amdgpu_buffer_rsrc_t ri = __builtin_amdgcn_make_buffer_rsrc((void *)in, 0, (int)(nvec * 16 > 0x7fffffff ? 0x7fffffff : nvec * 16), 0x00020000);
    const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc((void *)io, 0, (int)(nvec * 16 > 0x7fffffff ? 0x7fffffff : nvec * 16), 0x00020000);
    const long nthr = (long)gridDim.x * 256;
    for (long c0 = (long)blockIdx.x * 256 * U + threadIdx.x; c0 < nvec; c0 += nthr * U) {
        u32x4 a[U], b[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int off = (int)((c0 + u * 256) * 16);
            a[u] = __builtin_amdgcn_raw_buffer_load_b128(ro, off, 0, LA);   // out of range: reads 0
            b[u] = __builtin_amdgcn_raw_buffer_load_b128(ri, off, 0, LA);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int off = (int)((c0 + u * 256) * 16);
            f32x4 r = __builtin_bit_cast(f32x4, a[u]) + __builtin_bit_cast(f32x4, b[u]);
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, r), ro, off, 0, SA);  // out of range: dropped
        }
    }
}

// LDS-DMA: each wave stages its U chunks of both operands in its own slab
// (lane-linear, so every lane reads back what its own load wrote)
template <int U>
__global__ void __launch_bounds__(256) k_glds(const f32x4 *__restrict__ in, f32x4 *__restrict__ io, long nvec)
{
    __shared__ f32x4 slab[4][2 * U][64];
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    const long nthr = (long)gridDim.x * 256;
    for (long c0 = (long)blockIdx.x * 256 * U + threadIdx.x; c0 < nvec; c0 += nthr * U) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            long c = c0 + u * 256;
            if (c > nvec - 1) c = nvec - 1;   // whole waves issue: clamp, never store past the end
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)(io + c),
                                             (__attribute__((address_space(3))) void *)&slab[w][2 * u][0], 16, 0, 2);
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)(in + c),
                                             (__attribute__((address_space(3))) void *)&slab[w][2 * u + 1][0], 16, 0, 2);
        }
        __builtin_amdgcn_s_waitcnt(0x0070);   // vmcnt(0) expcnt(7) lgkmcnt(0): every LDS-DMA landed
#pragma unroll
        for (int u = 0; u < U; ++u) {
            long c = c0 + u * 256;
            f32x4 r = slab[w][2 * u][l] + slab[w][2 * u + 1][l];
            if (c < nvec) __builtin_nontemporal_store(r, &io[c]);
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0) before the slab is refilled
    }
}

// ceilings: read both operands only (one dword per thread out), write only, copy
template <int U>
__global__ void __launch_bounds__(256) k_read2(const f32x4 *__restrict__ in, f32x4 *__restrict__ io, long nvec)
{
    const long nthr = (long)gridDim.x * 256;
    f32x4 acc = {0, 0, 0, 0};
    for (long c0 = (long)blockIdx.x * 256 * U + threadIdx.x; c0 < nvec; c0 += nthr * U) {
        f32x4 a[U], b[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            long c = c0 + u * 256;
            if (c < nvec) { a[u] = __builtin_nontemporal_load(&io[c]); b[u] = __builtin_nontemporal_load(&in[c]); }
            else a[u] = b[u] = acc;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) acc += a[u] + b[u];
    }
    if (acc.x == 1234.5f) io[threadIdx.x] = acc;   // never true for the fill pattern; keeps the loads
}

template <int U>
__global__ void __launch_bounds__(256) k_write(const f32x4 *__restrict__ in, f32x4 *__restrict__ io, long nvec)
{
    const long nthr = (long)gridDim.x * 256;
    const f32x4 v = {1.f, 2.f, 3.f, (float)blockIdx.x};
    for (long c0 = (long)blockIdx.x * 256 * U + threadIdx.x; c0 < nvec; c0 += nthr * U)
#pragma unroll
        for (int u = 0; u < U; ++u) {
            long c = c0 + u * 256;
            if (c < nvec) __builtin_nontemporal_store(v, &io[c]);
        }
}

// write ceiling through buffer stores with cache-policy bits SA
template <int U, int SA>
__global__ void __launch_bounds__(256) k_bwrite(const f32x4 *__restrict__ in, f32x4 *__restrict__ io, long nvec)
{
    const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc((void *)io, 0, (int)(nvec * 16 > 0x7fffffff ? 0x7fffffff : nvec * 16), 0x00020000);
    const long nthr = (long)gridDim.x * 256;
    const f32x4 v = {1.f, 2.f, 3.f, (float)blockIdx.x};
    for (long c0 = (long)blockIdx.x * 256 * U + threadIdx.x; c0 < nvec; c0 += nthr * U)
#pragma unroll
        for (int u = 0; u < U; ++u)
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), ro, (int)((c0 + u * 256) * 16), 0, SA);
}

// write ceiling, plain (cached) global stores
template <int U>
__global__ void __launch_bounds__(256) k_write_c(const f32x4 *__restrict__ in, f32x4 *__restrict__ io, long nvec)
{
    const long nthr = (long)gridDim.x * 256;
    const f32x4 v = {1.f, 2.f, 3.f, (float)blockIdx.x};
    for (long c0 = (long)blockIdx.x * 256 * U + threadIdx.x; c0 < nvec; c0 += nthr * U)
#pragma unroll
        for (int u = 0; u < U; ++u) {
            long c = c0 + u * 256;
            if (c < nvec) io[c] = v;
        }
}

template <int U>
__global__ void __launch_bounds__(256) k_copy(const f32x4 *__restrict__ in, f32x4 *__restrict__ io, long nvec)
{
    const long nthr = (long)gridDim.x * 256;
    for (long c0 = (long)blockIdx.x * 256 * U + threadIdx.x; c0 < nvec; c0 += nthr * U) {
        f32x4 b[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            long c = c0 + u * 256;
            if (c < nvec) b[u] = __builtin_nontemporal_load(&in[c]);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            long c = c0 + u * 256;
            if (c < nvec) __builtin_nontemporal_store(b[u], &io[c]);
        }
    }
}

// MAP 1: a lane's U chunks one grid-width apart (c0 + u * nthr), so the
// chunks in flight across the chip at one time form U compact windows of
// grid x 4 KiB rather than one window of grid x U x 4 KiB
template <int U, int MAP>
__global__ void __launch_bounds__(256) k_sum_map(const f32x4 *__restrict__ in, f32x4 *__restrict__ io, long nvec)
{
    const long nthr = (long)gridDim.x * 256;
    const long step = MAP ? nthr : 256;
    const long base = MAP ? (long)blockIdx.x * 256 : (long)blockIdx.x * 256 * U;
    for (long c0 = base + threadIdx.x; c0 < nvec; c0 += nthr * U) {
        f32x4 a[U], b[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            long c = c0 + u * step;
            if (c < nvec) { a[u] = __builtin_nontemporal_load(&io[c]); b[u] = __builtin_nontemporal_load(&in[c]); }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            long c = c0 + u * step;
            if (c < nvec) __builtin_nontemporal_store(a[u] + b[u], &io[c]);
        }
    }
}

template <int U, int MAP>
__global__ void __launch_bounds__(256) k_write_map(const f32x4 *__restrict__ in, f32x4 *__restrict__ io, long nvec)
{
    const long nthr = (long)gridDim.x * 256;
    const long step = MAP ? nthr : 256;
    const long base = MAP ? (long)blockIdx.x * 256 : (long)blockIdx.x * 256 * U;
    const f32x4 v = {1.f, 2.f, 3.f, (float)blockIdx.x};
    for (long c0 = base + threadIdx.x; c0 < nvec; c0 += nthr * U)
#pragma unroll
        for (int u = 0; u < U; ++u) {
            long c = c0 + u * step;
            if (c < nvec) __builtin_nontemporal_store(v, &io[c]);
        }
}

// MAP 2: each wave's U chunks contiguous (wave w of block b covers chunks
// [b*256*U + w*64*U, +64*U)), one pass (exact grid)
template <int U>
__global__ void __launch_bounds__(256) k_sum_wc(const f32x4 *__restrict__ in, f32x4 *__restrict__ io, long nvec)
{
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    const long c0 = (long)blockIdx.x * 256 * U + (long)w * 64 * U + l;
    f32x4 a[U], b[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        long c = c0 + u * 64;
        if (c < nvec) { a[u] = __builtin_nontemporal_load(&io[c]); b[u] = __builtin_nontemporal_load(&in[c]); }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        long c = c0 + u * 64;
        if (c < nvec) __builtin_nontemporal_store(a[u] + b[u], &io[c]);
    }
}

template <int U>
__global__ void __launch_bounds__(256) k_write_wc(const f32x4 *__restrict__ in, f32x4 *__restrict__ io, long nvec)
{
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    const long c0 = (long)blockIdx.x * 256 * U + (long)w * 64 * U + l;
    const f32x4 v = {1.f, 2.f, 3.f, (float)blockIdx.x};
#pragma unroll
    for (int u = 0; u < U; ++u) {
        long c = c0 + u * 64;
        if (c < nvec) __builtin_nontemporal_store(v, &io[c]);
    }
}

// the same with 64-thread blocks (one wave per block)
template <int U>
__global__ void __launch_bounds__(64) k_sum_w64(const f32x4 *__restrict__ in, f32x4 *__restrict__ io, long nvec)
{
    const long c0 = (long)blockIdx.x * 64 * U + threadIdx.x;
    f32x4 a[U], b[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        long c = c0 + u * 64;
        if (c < nvec) { a[u] = __builtin_nontemporal_load(&io[c]); b[u] = __builtin_nontemporal_load(&in[c]); }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        long c = c0 + u * 64;
        if (c < nvec) __builtin_nontemporal_store(a[u] + b[u], &io[c]);
    }
}

// X: the U 4-KiB segments of block b are g = ((b / X) * U + u) * X + b % X,
// so consecutive segments go to consecutive blocks, i.e. round-robin over
// the XCDs exactly as in a one-segment-per-block (U = 1) launch, while each
// lane keeps 2U loads in flight.  Exact grid, nvec a multiple of 256*U*X.
template <int U, int X, int WRITE_ONLY>
__global__ void __launch_bounds__(256) k_sum_x(const f32x4 *__restrict__ in, f32x4 *__restrict__ io, long nvec)
{
    const long b = blockIdx.x;
    const long g0 = (b / X) * U * X + b % X;
    f32x4 a[U], bb[U];
    if (!WRITE_ONLY) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            long c = (g0 + (long)u * X) * 256 + threadIdx.x;
            a[u] = __builtin_nontemporal_load(&io[c]); bb[u] = __builtin_nontemporal_load(&in[c]);
        }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        long c = (g0 + (long)u * X) * 256 + threadIdx.x;
        f32x4 r;
        if (WRITE_ONLY) r = (f32x4){1.f, 2.f, 3.f, (float)b};
        else r = a[u] + bb[u];
        __builtin_nontemporal_store(r, &io[c]);
    }
}

typedef void (*KF)(const f32x4 *, f32x4 *, long);
struct Var { const char *name; KF f; int U; int moved; long grid; };   // moved: vectors of 256 MiB per launch; grid 0 = one pass

int main(int argc, char **argv)
{
    const long nbytes = 256L << 20, nvec = nbytes / 16;
    const int NB = argc > 1 ? atoi(argv[1]) : 4;
    std::vector<f32x4 *> ins(NB), ios(NB);
    for (int b = 0; b < NB; ++b) {
        CHECK(hipMalloc(&ins[b], nbytes));
        CHECK(hipMalloc(&ios[b], nbytes));
        CHECK(hipMemset(ins[b], 0x3c, nbytes));
        CHECK(hipMemset(ios[b], 0x3d, nbytes));
    }
    Var vars[] = {
        {"glob U4 nt (product)", k_glob<4>, 4, 3},
        {"glob U2 nt", k_glob<2>, 2, 3},
        {"buf U4 ld nt st nt", k_buf<4, 2, 2>, 4, 3},
        {"buf U4 ld 0 st nt", k_buf<4, 0, 2>, 4, 3},
        {"buf U4 ld sc1nt st sc1nt", k_buf<4, 18, 18>, 4, 3},
        {"buf U4 ld sc0sc1nt st nt", k_buf<4, 19, 2>, 4, 3},
        {"buf U4 ld nt st sc0sc1nt", k_buf<4, 2, 19>, 4, 3},
        {"buf U8 ld nt st nt", k_buf<8, 2, 2>, 8, 3},
        {"glds U2 nt", k_glds<2>, 2, 3},
        {"glds U4 nt", k_glds<4>, 4, 3},
        {"read2 U4 nt (ceiling)", k_read2<4>, 4, 2},
        {"write U4 nt (ceiling)", k_write<4>, 4, 1},
        {"copy U4 nt (ceiling)", k_copy<4>, 4, 2},
    };
    Var ceil_vars[] = {
        {"glob U4 nt (product)", k_glob<4>, 4, 3},
        {"read2 U4 nt", k_read2<4>, 4, 2},
        {"read2 U8 nt", k_read2<8>, 8, 2},
        {"read2 U2 nt", k_read2<2>, 2, 2},
        {"write U4 nt", k_write<4>, 4, 1},
        {"write U1 nt", k_write<1>, 1, 1},
        {"write U8 nt", k_write<8>, 8, 1},
        {"write U4 cached", k_write_c<4>, 4, 1},
        {"bwrite U4 sc1nt", k_bwrite<4, 18>, 4, 1},
        {"bwrite U4 sc0sc1nt", k_bwrite<4, 19>, 4, 1},
        {"bwrite U4 sc0nt", k_bwrite<4, 3>, 4, 1},
        {"bwrite U4 sc1", k_bwrite<4, 16>, 4, 1},
        {"copy U4 nt", k_copy<4>, 4, 2},
    };
    Var map_vars[] = {
        {"sum U4 contig (product)", k_sum_map<4, 0>, 4, 3},
        {"sum U4 ustride", k_sum_map<4, 1>, 4, 3},
        {"sum U4 contig g2048", k_sum_map<4, 0>, 4, 3, 2048},
        {"sum U4 ustride g2048", k_sum_map<4, 1>, 4, 3, 2048},
        {"sum U2 ustride", k_sum_map<2, 1>, 2, 3},
        {"sum U8 ustride", k_sum_map<8, 1>, 8, 3},
        {"sum U1 g2048", k_sum_map<1, 0>, 1, 3, 2048},
        {"sum U1", k_sum_map<1, 0>, 1, 3},
        {"write U1", k_write_map<1, 0>, 1, 1},
        {"write U4 ustride", k_write_map<4, 1>, 4, 1},
        {"write U1 g2048", k_write_map<1, 0>, 1, 1, 2048},
        {"write U1 g1024", k_write_map<1, 0>, 1, 1, 1024},
        {"write U4 contig g512", k_write_map<4, 0>, 4, 1, 512},
    };
    Var wc_vars[] = {
        {"sum U4 contig (product)", k_sum_map<4, 0>, 4, 3},
        {"sum U4 wavecontig", k_sum_wc<4>, 4, 3},
        {"sum U2 wavecontig", k_sum_wc<2>, 2, 3},
        {"sum U8 wavecontig", k_sum_wc<8>, 8, 3},
        {"sum U16 wavecontig", k_sum_wc<16>, 16, 3},
        {"sum U4 w64", k_sum_w64<4>, 4, 3, -4},
        {"sum U8 w64", k_sum_w64<8>, 8, 3, -8},
        {"write U1", k_write_map<1, 0>, 1, 1},
        {"write U4 wavecontig", k_write_wc<4>, 4, 1},
        {"write U2 wavecontig", k_write_wc<2>, 2, 1},
        {"write U8 wavecontig", k_write_wc<8>, 8, 1},
        {"write U16 wavecontig", k_write_wc<16>, 16, 1},
        {"read2 U4", k_read2<4>, 4, 2},
    };
    Var x_vars[] = {
        {"sum U4 contig (product)", k_sum_map<4, 0>, 4, 3},
        {"sum U4 X8", k_sum_x<4, 8, 0>, 4, 3},
        {"sum U2 X8", k_sum_x<2, 8, 0>, 2, 3},
        {"sum U8 X8", k_sum_x<8, 8, 0>, 8, 3},
        {"sum U4 X16", k_sum_x<4, 16, 0>, 4, 3},
        {"sum U4 X32", k_sum_x<4, 32, 0>, 4, 3},
        {"sum U4 X256", k_sum_x<4, 256, 0>, 4, 3},
        {"sum U1", k_sum_map<1, 0>, 1, 3},
        {"write U1", k_write_map<1, 0>, 1, 1},
        {"write U4 X8", k_sum_x<4, 8, 1>, 4, 1},
        {"write U4 X16", k_sum_x<4, 16, 1>, 4, 1},
        {"write U4 X256", k_sum_x<4, 256, 1>, 4, 1},
        {"write U4", k_write_map<4, 0>, 4, 1},
    };
    if (argc > 3 && !strcmp(argv[3], "x")) {
        static_assert(sizeof(x_vars) == sizeof(vars), "same count");
        memcpy(vars, x_vars, sizeof vars);
    }
    if (argc > 3 && !strcmp(argv[3], "wc")) {
        static_assert(sizeof(wc_vars) == sizeof(vars), "same count");
        memcpy(vars, wc_vars, sizeof vars);
    }
    const bool ceil_set = argc > 3 && !strcmp(argv[3], "ceil");
    if (ceil_set) {
        static_assert(sizeof(ceil_vars) == sizeof(vars), "same count");
        memcpy(vars, ceil_vars, sizeof vars);
    }
    if (argc > 3 && !strcmp(argv[3], "map")) {
        static_assert(sizeof(map_vars) == sizeof(vars), "same count");
        memcpy(vars, map_vars, sizeof vars);
    }
    const int NV = sizeof(vars) / sizeof(vars[0]);
    const int reps = 20, rounds = argc > 2 ? atoi(argv[2]) : 7;
    std::vector<std::vector<float>> t(NV);
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    // correctness of the SUM variants on the first buffer pair
    {
        std::vector<float> h(1024);
        for (int v = 0; v < NV; ++v) {
            if (vars[v].moved != 3) continue;
            CHECK(hipMemset(ios[0], 0x3d, nbytes));
            long blocks = vars[v].grid > 0 ? vars[v].grid : vars[v].grid < 0 ? nvec / (64L * vars[v].U) : (nvec + 256L * vars[v].U - 1) / (256L * vars[v].U);
            hipLaunchKernelGGL(vars[v].f, dim3(blocks), dim3(vars[v].grid < 0 ? 64 : 256), 0, 0, ins[0], ios[0], nvec);
            CHECK(hipDeviceSynchronize());
            float a, b;
            unsigned ua = 0x3d3d3d3du, ub = 0x3c3c3c3cu;
            memcpy(&a, &ua, 4); memcpy(&b, &ub, 4);
            for (long off : {0L, nbytes / 2 - 4096, nbytes - 4096}) {
                CHECK(hipMemcpy(h.data(), (char *)ios[0] + off, 4096, hipMemcpyDeviceToHost));
                for (int i = 0; i < 1024; ++i)
                    if (h[i] != a + b) { printf("MISMATCH %s at %ld: %g\n", vars[v].name, off / 4 + i, h[i]); return 1; }
            }
        }
        printf("sum variants correct\n");
    }
    for (int r = 0; r < rounds; ++r) {
        for (int v = 0; v < NV; ++v) {
            long blocks = vars[v].grid > 0 ? vars[v].grid : vars[v].grid < 0 ? nvec / (64L * vars[v].U) : (nvec + 256L * vars[v].U - 1) / (256L * vars[v].U);
            const int bs = vars[v].grid < 0 ? 64 : 256;
            for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(vars[v].f, dim3(blocks), dim3(bs), 0, 0, ins[w % NB], ios[w % NB], nvec);
            CHECK(hipEventRecord(e0, 0));
            for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(vars[v].f, dim3(blocks), dim3(bs), 0, 0, ins[i % NB], ios[i % NB], nvec);
            CHECK(hipEventRecord(e1, 0));
            CHECK(hipEventSynchronize(e1));
            float ms;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            t[v].push_back(ms / reps);
        }
        fprintf(stderr, "round %d done\n", r);
    }
    printf("%-28s %9s %9s %8s %6s\n", "variant", "med_us", "min_us", "TB/s", "of8");
    for (int v = 0; v < NV; ++v) {
        auto x = t[v];
        std::sort(x.begin(), x.end());
        float med = x[x.size() / 2], mn = x[0];
        double tbs = vars[v].moved * (double)nbytes / (med * 1e-3) / 1e12;
        printf("%-28s %9.1f %9.1f %8.3f %6.3f\n", vars[v].name, med * 1e3, mn * 1e3, tbs, tbs / 8.0);
    }
    return 0;
}
