/* copy_probe.c -- host copy rates behind the pageable-buffer pipeline
 * (csrc/mvx_host.c mvx_pcopy): T threads each copy one part of a B-byte
 * slice, as the copy pool does, with
 *   libc      glibc memcpy (what mvx_pcopy calls)
 *   nt        AVX2 loads + non-temporal 32-byte stores (no read-for-ownership
 *             of the destination, no cache pollution), sfence at the end
 * over a 1 GiB source / destination pair walked slice by slice (so nothing
 * is cache-resident), for slices of 8 .. 64 MiB and T = 1 .. 16.
 * One JSON line per (method, slice, threads): GB/s of bytes copied.
 *   gcc -O2 -mavx2 -pthread tools/copy_probe.c -o tools/copy_probe */
#define _GNU_SOURCE 1
#include <immintrin.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

static void copy_nt(char *d, const char *s, size_t n)
{
    size_t i = 0;
    /* head to a 32-byte aligned destination */
    while (i < n && ((uintptr_t)(d + i) & 31)) { d[i] = s[i]; i++; }
    for (; i + 128 <= n; i += 128) {
        __m256i a = _mm256_loadu_si256((const __m256i *)(s + i));
        __m256i b = _mm256_loadu_si256((const __m256i *)(s + i + 32));
        __m256i c = _mm256_loadu_si256((const __m256i *)(s + i + 64));
        __m256i e = _mm256_loadu_si256((const __m256i *)(s + i + 96));
        _mm256_stream_si256((__m256i *)(d + i), a);
        _mm256_stream_si256((__m256i *)(d + i + 32), b);
        _mm256_stream_si256((__m256i *)(d + i + 64), c);
        _mm256_stream_si256((__m256i *)(d + i + 96), e);
    }
    for (; i < n; i++) d[i] = s[i];
    _mm_sfence();
}

typedef struct { char *d; const char *s; size_t n; int nt; } part_t;

static void *run_part(void *arg)
{
    part_t *p = (part_t *)arg;
    if (p->nt) copy_nt(p->d, p->s, p->n);
    else memcpy(p->d, p->s, p->n);
    return NULL;
}

static double now(void)
{
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + t.tv_nsec * 1e-9;
}

int main(int argc, char **argv)
{
    const size_t total = (size_t)1 << 30;
    const int reps = argc > 1 ? atoi(argv[1]) : 3;
    char *src = malloc(total), *dst = malloc(total);
    const size_t slices[] = {8u << 20, 32u << 20, 64u << 20};
    const int threads[] = {1, 4, 8, 16};
    int si, ti, nt, r;
    if (!src || !dst) return 1;
    memset(src, 1, total);
    memset(dst, 2, total);
    for (si = 0; si < 3; si++)
        for (ti = 0; ti < 4; ti++)
            for (nt = 0; nt < 2; nt++) {
                const size_t sl = slices[si];
                const int T = threads[ti];
                double best = 0;
                for (r = 0; r < reps; r++) {
                    double t0 = now(), dt;
                    size_t off;
                    for (off = 0; off + sl <= total; off += sl) {
                        pthread_t th[16];
                        part_t pt[16];
                        const size_t per = ((sl + T - 1) / T + 4095) & ~(size_t)4095;
                        int i;
                        for (i = 0; i < T; i++) {
                            size_t lo = per * i, hi = lo + per;
                            if (lo > sl) lo = sl;
                            if (hi > sl) hi = sl;
                            pt[i].d = dst + off + lo; pt[i].s = src + off + lo; pt[i].n = hi - lo; pt[i].nt = nt;
                            if (i) pthread_create(&th[i], NULL, run_part, &pt[i]);
                        }
                        run_part(&pt[0]);
                        for (i = 1; i < T; i++) pthread_join(th[i], NULL);
                    }
                    dt = now() - t0;
                    if (total / dt / 1e9 > best) best = total / dt / 1e9;
                }
                printf("{\"method\": \"%s\", \"slice_mib\": %zu, \"threads\": %d, \"GBps\": %.2f}\n",
                       nt ? "nt" : "libc", sl >> 20, T, best);
                fflush(stdout);
            }
    return 0;
}
