// zc_attr.hip -- which device address reaches a page-locked host byte?
// For hipHostMalloc'd memory and for malloc'd memory hipHostRegister'ed
// after the fact, at the base and at an interior offset: what
// hipPointerGetAttributes reports (devicePointer / hostPointer) and what
// hipHostGetDevicePointer returns, then a kernel adds 1 to 1 MiB through the
// reported device address and the host checks the bytes.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

__global__ void k_inc(float *p, long n)
{
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) p[i] += 1.f;
}

static int probe(const char *what, char *base, size_t bytes)
{
    const size_t offs[2] = {0, 12345 * 16};
    for (int k = 0; k < 2; ++k) {
        char *p = base + offs[k];
        hipPointerAttribute_t a;
        void *gd = NULL;
        CHECK(hipPointerGetAttributes(&a, p));
        hipError_t e = hipHostGetDevicePointer(&gd, p, 0);
        (void)hipGetLastError();
        printf("{\"memory\": \"%s\", \"offset\": %zu, \"type\": %d, \"host\": \"%p\", \"attr_dev\": \"%p\", "
               "\"attr_host\": \"%p\", \"get_dev\": \"%p\", \"get_dev_rc\": %d, \"dev_eq_host\": %d}\n",
               what, offs[k], (int)a.type, (void *)p, a.devicePointer, a.hostPointer, gd, (int)e,
               a.devicePointer == (void *)p);
        if (a.type != hipMemoryTypeHost || !a.devicePointer) { printf("not device-accessible\n"); return 1; }
        const long n = (1 << 20) / 4;
        float *h = (float *)p;
        for (long i = 0; i < n; ++i) h[i] = (float)(i % 100);
        hipLaunchKernelGGL(k_inc, dim3(256), dim3(256), 0, 0, (float *)a.devicePointer, n);
        CHECK(hipDeviceSynchronize());
        for (long i = 0; i < n; ++i)
            if (h[i] != (float)(i % 100) + 1.f) { printf("MISMATCH %s at %ld\n", what, i); return 1; }
    }
    (void)bytes;
    return 0;
}

int main()
{
    const size_t bytes = 8 << 20;
    char *hm, *rg;
    CHECK(hipHostMalloc((void **)&hm, bytes, hipHostMallocDefault));
    if (probe("hipHostMalloc", hm, bytes)) return 1;
    rg = (char *)aligned_alloc(4096, bytes);
    memset(rg, 0, bytes);
    CHECK(hipHostRegister(rg, bytes, hipHostRegisterDefault));
    if (probe("hipHostRegister(malloc)", rg, bytes)) return 1;
    CHECK(hipHostUnregister(rg));
    free(rg);
    CHECK(hipHostFree(hm));
    printf("zc_attr ok\n");
    return 0;
}
