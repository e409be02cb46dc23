// write_gran.hip -- HBM cost of partial-line streams on this GPU: the same
// 128 MiB written (or read) as runs of RUN bytes out of every PERIOD bytes,
// one 16-byte non-temporal access per lane, against the contiguous stream.
// Answers whether a stream that touches 64 of every 128 bytes (the unit
// kernel's unpack of vector(64,16,32,FLOAT)) costs its own
// bytes or whole 128-byte lines.  Measurement probe only.
//   ./write_gran > out.jsonl   (one JSON line per (op, RUN, PERIOD))
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int RUN, int PERIOD>
__global__ void __launch_bounds__(256) k_wrun(f32x4 *__restrict__ b)
{
    const long v = (long)blockIdx.x * 256 + threadIdx.x;       // 16-byte vector of the written data
    constexpr int R = RUN / 16;
    const long at = (v / R) * (PERIOD / 16) + v % R;
    const f32x4 x = {1.f, 2.f, 3.f, (float)blockIdx.x};
    __builtin_nontemporal_store(x, b + at);
}

template <int RUN, int PERIOD>
__global__ void __launch_bounds__(256) k_rrun(const f32x4 *__restrict__ a, f32x4 *__restrict__ sink)
{
    const long v = (long)blockIdx.x * 256 + threadIdx.x;
    constexpr int R = RUN / 16;
    const long at = (v / R) * (PERIOD / 16) + v % R;
    const f32x4 x = __builtin_nontemporal_load(a + at);
    if (x.x == 1234.5f && x.y == -1234.5f) sink[threadIdx.x] = x;
}

#define CHECK(x) do { if ((x) != hipSuccess) { fprintf(stderr, "HIP error %s line %d\n", #x, __LINE__); return 1; } } while (0)

template <int RUN, int PERIOD>
static int run(void *buf, size_t data, hipStream_t st, hipEvent_t e0, hipEvent_t e1)
{
    const unsigned blocks = (unsigned)(data / 16 / 256);
    for (int op = 0; op < 2; ++op) {
        float best = 1e30f, sum = 0;
        const int reps = 20;
        for (int r = -2; r < reps; ++r) {
            CHECK(hipEventRecord(e0, st));
            if (op == 0) hipLaunchKernelGGL((k_wrun<RUN, PERIOD>), dim3(blocks), dim3(256), 0, st, (f32x4 *)buf);
            else hipLaunchKernelGGL((k_rrun<RUN, PERIOD>), dim3(blocks), dim3(256), 0, st, (const f32x4 *)buf,
                                    (f32x4 *)buf);
            CHECK(hipEventRecord(e1, st));
            CHECK(hipEventSynchronize(e1));
            float ms;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            if (r >= 0) { sum += ms; if (ms < best) best = ms; }
        }
        const double us = 1e3 * sum / reps;
        printf("{\"op\": \"%s\", \"run\": %d, \"period\": %d, \"bytes\": %zu, \"span\": %zu, \"us_mean\": %.2f, "
               "\"us_min\": %.2f, \"GBs_of_bytes\": %.1f, \"GBs_of_span\": %.1f}\n",
               op ? "read" : "write", RUN, PERIOD, data, data / RUN * PERIOD, us, 1e3 * best, data / us / 1e3,
               (double)(data / RUN * PERIOD) / us / 1e3);
        fflush(stdout);
    }
    return 0;
}

int main()
{
    const size_t data = 128ul << 20;           // bytes touched per launch
    void *buf;
    hipStream_t st;
    hipEvent_t e0, e1;
    CHECK(hipMalloc(&buf, data * 4));           // PERIOD / RUN <= 4
    CHECK(hipMemset(buf, 0, data * 4));
    CHECK(hipStreamCreate(&st));
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    if (run<16, 16>(buf, data, st, e0, e1) || run<64, 128>(buf, data, st, e0, e1) ||
        run<128, 256>(buf, data, st, e0, e1) || run<256, 512>(buf, data, st, e0, e1) ||
        run<32, 64>(buf, data, st, e0, e1) || run<64, 256>(buf, data, st, e0, e1) ||
        run<16, 32>(buf, data, st, e0, e1) || run<128, 512>(buf, data, st, e0, e1))
        return 1;
    CHECK(hipFree(buf));
    return 0;
}
