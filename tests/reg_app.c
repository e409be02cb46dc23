/* reg_app.c -- TEST HELPER: the registration cache's release hooks
 * (csrc/mvx_host.c; the reference's mem_hooks.c:97-132 -> dreg.c:1063
 * find_and_free_dregs_inside) in a program linked with -lmvx, so libmvx.so's
 * free / realloc / munmap / mremap / madvise / sbrk are the process's.
 *
 *   reg_app dry   (MVX_HOST_REGISTER_DRY=1, no GPU): register ranges with
 *                 mvx_host_register, release them every way, and check the
 *                 entries are gone -- and that unrelated releases keep them
 *   reg_app gpu   a pageable 96 MiB pair reduced on the device (MPIR_SUM),
 *                 freed with no mvx_host_unregister, allocated again at the
 *                 same size (the same address in practice) and reduced again:
 *                 bit-exact.  The entries are checked to be gone before the
 *                 second DMA; if they were not, the program stops there.
 *                 The same for mmap'd memory unmapped and mapped again.
 *   reg_app stress (dry, no GPU): 8 threads at once, each registering and
 *                 freeing its own mmap'd blocks while others churn small
 *                 malloc / free and unrelated mmap / munmap: every
 *                 registration is dropped by its own block's free, exactly
 *                 once, nothing is left, no thread waits on another for good.
 * Prints "reg_app ok" and one JSON line of what it saw. */
#define _GNU_SOURCE 1
#include <malloc.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <unistd.h>

#include "mvx_coll.h"

#define MIB (1UL << 20)

static long entries(void)
{
    long n = -1;
    mvx_host_register_stats(&n, NULL, NULL, NULL);
    return n;
}

#define CHECK(cond, what)                                                          \
    do {                                                                           \
        if (!(cond)) {                                                             \
            printf("FAIL %s (line %d): entries %ld\n", what, __LINE__, entries()); \
            return 1;                                                              \
        }                                                                          \
    } while (0)

static void *map(size_t n)
{
    void *p = mmap(NULL, n, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    return p == MAP_FAILED ? NULL : p;
}

static int dry(void)
{
    char *a, *b, *h, *m;
    long inv0 = mvx_host_register_invalidations();

    /* malloc'd (mmap'd at this size) then free */
    a = malloc(8 * MIB);
    memset(a, 1, 8 * MIB);
    CHECK(mvx_host_register(a, 8 * MIB) == 0 && entries() == 1, "register malloc");
    free(a);
    CHECK(entries() == 0, "free drops");

    /* an unrelated block's free keeps the entry */
    a = malloc(8 * MIB);
    b = malloc(8 * MIB);
    CHECK(mvx_host_register(a, 8 * MIB) == 0 && entries() == 1, "register a");
    free(b);
    CHECK(entries() == 1, "unrelated free keeps");
    a = realloc(a, 24 * MIB);
    CHECK(entries() == 0, "realloc drops");
    free(a);

    /* mmap'd: munmap, partial munmap, madvise, mremap */
    m = map(4 * MIB);
    CHECK(m && mvx_host_register(m, 4 * MIB) == 0, "register map");
    CHECK(munmap(m, 4 * MIB) == 0 && entries() == 0, "munmap drops");
    m = map(4 * MIB);
    CHECK(m && mvx_host_register(m, 4 * MIB) == 0, "register map 2");
    CHECK(munmap(m + 3 * MIB, MIB) == 0 && entries() == 0, "partial munmap drops");
    munmap(m, 3 * MIB);
    m = map(4 * MIB);
    CHECK(m && mvx_host_register(m, 4 * MIB) == 0, "register map 3");
    CHECK(madvise(m, MIB, MADV_WILLNEED) == 0 && entries() == 1, "madvise WILLNEED keeps");
    CHECK(madvise(m, MIB, MADV_DONTNEED) == 0 && entries() == 0, "madvise DONTNEED drops");
    CHECK(mvx_host_register(m, 4 * MIB) == 0, "register map 4");
    m = mremap(m, 4 * MIB, 2 * MIB, 0);
    CHECK(m != MAP_FAILED && entries() == 0, "mremap drops");
    munmap(m, 2 * MIB);

    /* the break: sbrk up, register, sbrk back down */
    h = sbrk(0);
    h = (char *)(((uintptr_t)h + 4095) & ~(uintptr_t)4095);
    CHECK(brk(h) == 0 && sbrk(2 * MIB) != (void *)-1, "sbrk up");
    memset(h, 2, 2 * MIB);
    CHECK(mvx_host_register(h, 2 * MIB) == 0 && entries() == 1, "register break");
    CHECK(sbrk(-(intptr_t)(2 * MIB)) != (void *)-1 && entries() == 0, "negative sbrk drops");

    printf("{\"mode\": \"dry\", \"invalidations\": %ld}\n", mvx_host_register_invalidations() - inv0);
    return 0;
}

#define ST_THREADS 8
#define ST_ITERS 400
static long st_registered[ST_THREADS], st_failed[ST_THREADS];

static void *st_worker(void *arg)
{
    const long t = (long)arg;
    unsigned seed = 12345u + (unsigned)t;
    int i, j;
    for (i = 0; i < ST_ITERS; i++) {
        size_t n;
        char *p, *small[8];
        seed = seed * 1103515245u + 12345u;
        n = (size_t)(1 + (seed >> 16) % 4) * MIB;          /* 1-4 MiB: mmap'd chunks */
        p = malloc(n);
        if (!p) { st_failed[t]++; continue; }
        p[0] = 1;
        if (mvx_host_register(p + 64, n - 128) == 0) st_registered[t]++;
        else st_failed[t]++;
        for (j = 0; j < 8; j++) small[j] = malloc(32 + 64 * j);   /* the hooks' fast path */
        if (t % 2) {                                        /* an unrelated mapping */
            char *m = mmap(NULL, 64 * 1024, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
            if (m != MAP_FAILED) munmap(m, 64 * 1024);
        }
        for (j = 0; j < 8; j++) free(small[j]);
        free(p);
    }
    return NULL;
}

static int stress(void)
{
    pthread_t th[ST_THREADS];
    long t, reg = 0, failed = 0, inv0 = mvx_host_register_invalidations(), inv;
    mallopt(M_MMAP_THRESHOLD, 512 * 1024);      /* fixed: blocks never share pages */
    for (t = 0; t < ST_THREADS; t++) CHECK(pthread_create(&th[t], NULL, st_worker, (void *)t) == 0, "thread");
    for (t = 0; t < ST_THREADS; t++) pthread_join(th[t], NULL);
    for (t = 0; t < ST_THREADS; t++) { reg += st_registered[t]; failed += st_failed[t]; }
    inv = mvx_host_register_invalidations() - inv0;
    printf("{\"mode\": \"stress\", \"threads\": %d, \"registered\": %ld, \"failed\": %ld, \"invalidations\": %ld}\n",
           ST_THREADS, reg, failed, inv);
    CHECK(failed == 0, "every registration taken");
    CHECK(entries() == 0, "nothing left");
    CHECK(inv == reg, "each registration dropped exactly once, by its own free");
    return 0;
}

static void fill(float *x, size_t n, unsigned seed)
{
    size_t i;
    for (i = 0; i < n; i++) {
        seed = seed * 1103515245u + 12345u;
        x[i] = (float)((int)((seed >> 16) & 15) - 8);      /* small integers: sums exact */
    }
}

/* y = x + y on the device through the host-buffer path of MPIR_SUM; 0 if
 * every element equals the CPU sum */
static int sum_check(float *x, float *y, size_t n, unsigned seed)
{
    int len = (int)n, bad = 0;
    MPI_Datatype t = MPI_FLOAT;
    float *want = malloc(n * sizeof(float));
    size_t i;
    fill(x, n, seed);
    fill(y, n, seed + 1);
    for (i = 0; i < n; i++) want[i] = x[i] + y[i];
    MPIR_SUM(x, y, &len, &t);
    if (mvx_op_errno() != 0) bad = 1;
    for (i = 0; i < n && !bad; i++) bad = y[i] != want[i];
    free(want);
    return bad;
}

static int gpu(void)
{
    const size_t nb = 96 * MIB, n = nb / sizeof(float);
    float *x, *y, *x2, *y2;
    char *m1, *m2;
    long hits0, hits1;
    int same_x, same_y, same_m;

    x = malloc(nb);
    y = malloc(nb);
    CHECK(x && y, "malloc");
    CHECK(sum_check(x, y, n, 1) == 0, "first call");
    CHECK(entries() == 2, "both operands registered");
    free(x);
    free(y);
    CHECK(entries() == 0, "free dropped both registrations");   /* before any further DMA */
    x2 = malloc(nb);
    y2 = malloc(nb);
    same_x = x2 == x;
    same_y = y2 == y;
    CHECK(sum_check(x2, y2, n, 7) == 0, "same-size reallocation reduces its new contents");
    mvx_host_register_stats(NULL, NULL, &hits0, NULL);
    CHECK(sum_check(x2, y2, n, 9) == 0, "third call");
    mvx_host_register_stats(NULL, NULL, &hits1, NULL);
    CHECK(hits1 - hits0 == 2, "third call hits the new registrations");
    free(x2);
    free(y2);
    CHECK(entries() == 0, "free dropped the new registrations");

    /* mmap'd memory unmapped and mapped again at the same address */
    m1 = map(2 * nb);
    CHECK(m1 && sum_check((float *)m1, (float *)(m1 + nb), n, 11) == 0, "mmap call");
    CHECK(entries() == 2, "mmap operands registered");
    CHECK(munmap(m1, 2 * nb) == 0 && entries() == 0, "munmap dropped them");
    m2 = mmap(m1, 2 * nb, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_FIXED_NOREPLACE, -1, 0);
    if (m2 == MAP_FAILED) m2 = map(2 * nb);
    same_m = m2 == m1;
    CHECK(m2 && sum_check((float *)m2, (float *)(m2 + nb), n, 13) == 0, "remapped call");
    munmap(m2, 2 * nb);
    CHECK(entries() == 0, "final munmap dropped them");
    printf("{\"mode\": \"gpu\", \"same_address\": {\"malloc_x\": %d, \"malloc_y\": %d, \"mmap\": %d}, "
           "\"invalidations\": %ld}\n", same_x, same_y, same_m, mvx_host_register_invalidations());
    return 0;
}

int main(int argc, char **argv)
{
    int rc;
    if (argc < 2) return 2;
    if (!mvx_host_hooks_active()) {
        printf("FAIL hooks not in effect\n");
        return 1;
    }
    if (mvx_host_register_enable(1, 0) != 0) {
        printf("FAIL enable\n");
        return 1;
    }
    rc = !strcmp(argv[1], "dry") ? dry() : !strcmp(argv[1], "gpu") ? gpu() : !strcmp(argv[1], "stress") ? stress() : 2;
    mvx_host_register_enable(0, 0);
    if (rc == 0) printf("reg_app ok\n");
    return rc;
}
