// TEST INFRASTRUCTURE: the ops of tests/user_ops.c as MVX_Device_functions
// (include/mvx_coll.h, mvx_op_create_device): each enqueues
// inout[i] = in[i] op inout[i] on the caller's stream, with the same bits as
// the host function (integer math; fsum is one IEEE add, no contraction).
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace {

struct Mix {
    typedef uint32_t T;
    __device__ static T f(T x, T y) { return x * 31u + (y ^ (y >> 3)) * 7u + 1u; }
};
struct Affine {
    typedef uint64_t T;
    __device__ static T f(T a, T b)
    {
        const uint32_t a1 = (uint32_t)a, b1 = (uint32_t)(a >> 32);
        const uint32_t a2 = (uint32_t)b, b2 = (uint32_t)(b >> 32);
        return (uint64_t)(a1 * a2) | ((uint64_t)(a2 * b1 + b2) << 32);
    }
};
struct Fsum {
    typedef float T;
    __device__ static T f(T a, T b) { return a + b; }
};
struct Addem {
    typedef int32_t T;
    __device__ static T f(T a, T b) { return (T)((uint32_t)a + (uint32_t)b); }
};

template <typename Op>
__global__ void __launch_bounds__(256) k_uop(const typename Op::T *in, typename Op::T *inout, size_t n)
{
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
        inout[i] = Op::f(in[i], inout[i]);
}

template <typename Op>
int launch(const void *in, void *inout, size_t len, void *stream)
{
    if (len == 0) return 0;
    size_t blocks = (len + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    hipLaunchKernelGGL(k_uop<Op>, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream,
                       (const typename Op::T *)in, (typename Op::T *)inout, len);
    return hipGetLastError() == hipSuccess ? 0 : 1;
}

struct IdPair { int a; int hole; double b; };

__global__ void __launch_bounds__(256) k_idsum(const IdPair *x, IdPair *y, size_t n)
{
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        y[i].a = (int)((unsigned)x[i].a + (unsigned)y[i].a);
        y[i].b = x[i].b + y[i].b;
    }
}

}  // namespace

extern "C" int duop_idsum(const void *in, void *inout, size_t len, int dt, void *s)
{
    (void)dt;
    if (len == 0) return 0;
    size_t blocks = (len + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    hipLaunchKernelGGL(k_idsum, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)s, (const IdPair *)in,
                       (IdPair *)inout, len);
    return hipGetLastError() == hipSuccess ? 0 : 1;
}

extern "C" int duop_mix(const void *in, void *inout, size_t len, int dt, void *s) { (void)dt; return launch<Mix>(in, inout, len, s); }
extern "C" int duop_affine(const void *in, void *inout, size_t len, int dt, void *s) { (void)dt; return launch<Affine>(in, inout, len, s); }
extern "C" int duop_fsum(const void *in, void *inout, size_t len, int dt, void *s) { (void)dt; return launch<Fsum>(in, inout, len, s); }
extern "C" int duop_addem(const void *in, void *inout, size_t len, int dt, void *s) { (void)dt; return launch<Addem>(in, inout, len, s); }
