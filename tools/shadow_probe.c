/* shadow_probe.c -- what HIP does with a pageable buffer whose first page
 * lies inside another buffer's hipHostRegister'ed range (two heap blocks
 * sharing a page, the first registered page-widened, as the registration
 * cache does): hipMemcpy H2D from the second block and D2H into it, checked
 * byte for byte.  Prints one JSON line. */
#define _GNU_SOURCE 1
#include <malloc.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <hip/hip_runtime_api.h>

int main(void)
{
    const size_t n = 8u << 20;
    char *x, *y, *d;
    uintptr_t base, end;
    hipError_t e1, e2, e3;
    size_t i, bad_in = 0, bad_out = 0;
    mallopt(M_MMAP_THRESHOLD, 512 << 20);
    mallopt(M_TRIM_THRESHOLD, 1024 << 20);
    x = malloc(n);
    y = malloc(n);
    for (i = 0; i < n; i++) { x[i] = (char)(i * 7); y[i] = (char)(i * 13 + 1); }
    base = (uintptr_t)x & ~4095UL;
    end = ((uintptr_t)x + n + 4095) & ~4095UL;
    e1 = hipHostRegister((void *)base, end - base, hipHostRegisterDefault);
    if (hipMalloc((void **)&d, n) != hipSuccess) return 1;
    e2 = hipMemcpy(d, y, n, hipMemcpyHostToDevice);
    {
        char *back = malloc(n);
        hipMemcpy(back, d, n, hipMemcpyDeviceToHost);
        for (i = 0; i < n; i++) bad_in += back[i] != y[i];
        for (i = 0; i < n; i++) back[i] = (char)(i * 5 + 3);
        hipMemcpy(d, back, n, hipMemcpyHostToDevice);
        e3 = hipMemcpy(y, d, n, hipMemcpyDeviceToHost);
        for (i = 0; i < n; i++) bad_out += y[i] != back[i];
        free(back);
    }
    printf("{\"y_first_page_in_x_registration\": %d, \"register\": %d, \"h2d\": %d, \"d2h\": %d, "
           "\"bad_in\": %zu, \"bad_out\": %zu}\n",
           (uintptr_t)y < end, (int)e1, (int)e2, (int)e3, bad_in, bad_out);
    return 0;
}
