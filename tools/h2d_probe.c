/* Host<->device staging strategies for 256 MiB (test-infrastructure probe). */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>
#include <time.h>
#include <hip/hip_runtime_api.h>

static double now(void) { struct timespec t; clock_gettime(CLOCK_MONOTONIC, &t); return t.tv_sec + t.tv_nsec * 1e-9; }
#define MB (1 << 20)
typedef struct { char *d; const char *s; size_t n; } cp_t;
static void *cp_fn(void *a) { cp_t *c = a; memcpy(c->d, c->s, c->n); return NULL; }
static void par_memcpy(char *d, const char *s, size_t n, int nt)
{
    pthread_t th[64]; cp_t c[64]; size_t per = (n + nt - 1) / nt; int i;
    for (i = 0; i < nt; i++) { size_t lo = i * per, hi = lo + per > n ? n : lo + per; c[i].d = d + lo; c[i].s = s + lo; c[i].n = hi > lo ? hi - lo : 0; pthread_create(&th[i], NULL, cp_fn, &c[i]); }
    for (i = 0; i < nt; i++) pthread_join(th[i], NULL);
}

int main(void)
{
    const size_t N = 256UL * MB;
    char *h = malloc(N), *dev, *pin;
    memset(h, 1, N);
    hipMalloc((void **)&dev, N);
    hipHostMalloc((void **)&pin, N, 0);
    memset(pin, 1, N);
    hipStream_t st; hipStreamCreate(&st);
    double t;
    for (int rep = 0; rep < 2; rep++) {
        t = now(); hipMemcpy(dev, h, N, hipMemcpyHostToDevice); printf("pageable hipMemcpy H2D   %6.1f GB/s\n", N / (now() - t) / 1e9);
        t = now(); hipMemcpy(h, dev, N, hipMemcpyDeviceToHost); printf("pageable hipMemcpy D2H   %6.1f GB/s\n", N / (now() - t) / 1e9);
        t = now(); hipMemcpy(dev, pin, N, hipMemcpyHostToDevice); printf("pinned hipMemcpy H2D     %6.1f GB/s\n", N / (now() - t) / 1e9);
        t = now(); hipMemcpy(pin, dev, N, hipMemcpyDeviceToHost); printf("pinned hipMemcpy D2H     %6.1f GB/s\n", N / (now() - t) / 1e9);
        t = now(); hipHostRegister(h, N, 0); double tr = now() - t;
        t = now(); hipMemcpy(dev, h, N, hipMemcpyHostToDevice); double tc = now() - t;
        t = now(); hipHostUnregister(h); double tu = now() - t;
        printf("register %.2f ms, copy %.1f GB/s, unregister %.2f ms -> %.1f GB/s end-to-end\n", tr * 1e3, N / tc / 1e9, tu * 1e3, N / (tr + tc + tu) / 1e9);
        for (int nt = 1; nt <= 16; nt *= 2) {
            t = now(); par_memcpy(pin, h, N, nt); printf("host memcpy %2d threads    %6.1f GB/s\n", nt, N / (now() - t) / 1e9);
        }
        /* chunked bounce pipeline: 4 x 16 MiB pinned slots, 8-thread memcpy */
        const size_t CH = 16 * MB; hipEvent_t ev[4]; for (int i = 0; i < 4; i++) { hipEventCreate(&ev[i]); hipEventRecord(ev[i], st); }
        t = now();
        for (size_t off = 0, i = 0; off < N; off += CH, i++) {
            int sl = i % 4; hipEventSynchronize(ev[sl]);
            par_memcpy(pin + sl * CH, h + off, CH, 8);
            hipMemcpyAsync(dev + off, pin + sl * CH, CH, hipMemcpyHostToDevice, st);
            hipEventRecord(ev[sl], st);
        }
        hipStreamSynchronize(st);
        printf("bounce pipeline H2D (8 thr) %6.1f GB/s\n", N / (now() - t) / 1e9);
        t = now();
        for (size_t off = 0, i = 0; off < N; off += CH, i++) {
            int sl = i % 4;
            hipMemcpyAsync(pin + sl * CH, dev + off, CH, hipMemcpyDeviceToHost, st);
            hipEventRecord(ev[sl], st);
            if (i >= 3) { size_t po = off - 3 * CH; int ps = (i - 3) % 4; hipEventSynchronize(ev[ps]); par_memcpy(h + po, pin + ps * CH, CH, 8); }
        }
        for (size_t k = (N / CH >= 3 ? N / CH - 3 : 0); k < N / CH; k++) { int ps = k % 4; hipEventSynchronize(ev[ps]); par_memcpy(h + k * CH, pin + ps * CH, CH, 8); }
        printf("bounce pipeline D2H (8 thr) %6.1f GB/s\n", N / (now() - t) / 1e9);
    }
    return 0;
}
