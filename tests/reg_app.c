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
 *   reg_app stub  (built with -DREG_STUB, no GPU): hipHostRegister /
 *                 hipHostUnregister / hipPointerGetAttributes are counting
 *                 stubs defined here, so libmvx.so's real (non-dry) cache
 *                 runs against them: a free of a registered buffer makes no
 *                 HIP call at all inside the hook -- the registration leaves
 *                 the cache and waits on the deferred list -- and the next
 *                 libmvx entry unregisters it (dreg.c:1063-1080, 678-767).
 *   reg_app neighbour (GPU) a 64 MiB heap buffer pair (not mmap'd: they
 *                 share their boundary pages with small neighbour blocks)
 *                 reduced on the device (MPIR_SUM through the registered
 *                 pages) over and over while a second thread frees and
 *                 reallocates the neighbour blocks: the registrations stay
 *                 (no invalidation), every result is bit-exact, no fault.
 *                 Then the second thread reports a release of the operand
 *                 itself (mvx_host_invalidate) while a call holds it: the
 *                 registration is deferred, not unpinned under the DMA, and
 *                 unregistered once the call is done.
 *   reg_app shadow (GPU) buffers that share pages with a registration:
 *                 (a) two adjacent 8 MiB heap buffers reduced together: the
 *                 second's registration merges with the first's (which this
 *                 same call holds) into one; (b) a thread reduces a 64 MiB
 *                 heap buffer A over and over (the op holds A's
 *                 registration) while the main thread runs a 2-rank
 *                 Allreduce on a virtual communicator whose sendbuf starts
 *                 in A's last page: when A is held that buffer is copied by
 *                 the CPU (HIP refuses a copy that starts inside a
 *                 registration and runs past it), else the two merge.  Every
 *                 result bit-exact.
 * Prints "reg_app ok" and one JSON line of what it saw. */
#define _GNU_SOURCE 1
#include <malloc.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <time.h>
#include <unistd.h>

#include "mvx_coll.h"

#define MIB (1UL << 20)

#ifdef REG_STUB
/* counting stubs in place of the HIP runtime's (the executable's
 * definitions come first in the lookup; no GPU needed) */
#include <hip/hip_runtime_api.h>
static long n_reg, n_unreg, n_attr;
static __thread int in_hook_probe;     /* set while a release is in progress on this thread */
static long hip_in_release;            /* HIP calls made while it was set */
hipError_t hipHostRegister(void *p, size_t n, unsigned int f)
{
    (void)p; (void)n; (void)f;
    __atomic_add_fetch(&n_reg, 1, __ATOMIC_RELAXED);
    if (in_hook_probe) __atomic_add_fetch(&hip_in_release, 1, __ATOMIC_RELAXED);
    return hipSuccess;
}
hipError_t hipHostUnregister(void *p)
{
    (void)p;
    __atomic_add_fetch(&n_unreg, 1, __ATOMIC_RELAXED);
    if (in_hook_probe) __atomic_add_fetch(&hip_in_release, 1, __ATOMIC_RELAXED);
    return hipSuccess;
}
hipError_t hipGetLastError(void) { return hipSuccess; }
hipError_t hipPointerGetAttributes(hipPointerAttribute_t *a, const void *p)
{
    (void)a; (void)p;
    __atomic_add_fetch(&n_attr, 1, __ATOMIC_RELAXED);
    if (in_hook_probe) __atomic_add_fetch(&hip_in_release, 1, __ATOMIC_RELAXED);
    return hipErrorInvalidValue;       /* not HIP memory: pageable */
}
#endif

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

/* a heap block of `n` bytes and a small block right after it that shares
 * its last page (retried past the rare layouts where it does not) */
static int heap_pair(char **a, char **b, size_t n)
{
    int t;
    for (t = 0; t < 8; t++) {
        *a = malloc(n);
        *b = malloc(64);
        if (*a && *b && ((uintptr_t)(*a + n - 1) & ~4095UL) == ((uintptr_t)*b & ~4095UL)) return 0;
        if (!malloc(48)) return 1;                  /* shift the next pair (kept) */
    }
    return 1;
}

/* blocks of n1 and n2 bytes, the second starting in the first's last page */
static int heap_adjacent(char **a, char **b, size_t n1, size_t n2)
{
    int t;
    for (t = 0; t < 8; t++) {
        *a = malloc(n1);
        *b = malloc(n2);
        if (*a && *b && ((uintptr_t)(*a + n1 - 1) & ~4095UL) == ((uintptr_t)*b & ~4095UL)) return 0;
        if (!malloc(48)) return 1;                  /* shift the next pair (kept) */
    }
    return 1;
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

    /* heap blocks sharing a page: freeing the neighbour keeps the entry,
     * freeing the buffer itself drops it */
    mallopt(M_MMAP_THRESHOLD, 256 * MIB);
    mallopt(M_TRIM_THRESHOLD, 512 * MIB);
    CHECK(heap_pair(&a, &b, 4 * MIB) == 0, "neighbour shares a page");
    CHECK(mvx_host_register(a, 4 * MIB) == 0 && entries() == 1, "register heap block");
    free(b);
    CHECK(entries() == 1, "neighbour free keeps");
    b = malloc(64);
    free(a);
    CHECK(entries() == 0, "own free drops");
    free(b);

    printf("{\"mode\": \"dry\", \"invalidations\": %ld}\n", mvx_host_register_invalidations() - inv0);
    return 0;
}

#ifdef REG_STUB
static long deferred(void)
{
    long d = -1;
    mvx_host_register_deferred(&d, NULL, NULL, NULL);
    return d;
}

static int stub(void)
{
    char *a, *m;
    long reg0, unreg0, u0, u1;
    a = malloc(8 * MIB);
    memset(a, 1, 8 * MIB);
    reg0 = n_reg;
    CHECK(mvx_host_register(a, 8 * MIB) == 0 && entries() == 1 && n_reg == reg0 + 1, "register through the stub");
    unreg0 = n_unreg;
    mvx_host_register_deferred(NULL, NULL, &u0, NULL);
    in_hook_probe = 1;
    free(a);                                        /* the hook: no HIP call */
    in_hook_probe = 0;
    CHECK(hip_in_release == 0, "no HIP call inside free()");
    CHECK(entries() == 0 && deferred() == 1 && n_unreg == unreg0, "free only defers");
    m = mmap(NULL, 4 * MIB, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    CHECK(m != MAP_FAILED && mvx_host_register(m, 4 * MIB) == 0, "register map");   /* a libmvx entry: flushes */
    CHECK(n_unreg == unreg0 + 1 && deferred() == 0, "the next entry unregisters the deferred one");
    in_hook_probe = 1;
    munmap(m, 4 * MIB);
    mvx_host_invalidate(m, 4 * MIB);                /* a host MPI's hook: nothing left to drop */
    in_hook_probe = 0;
    CHECK(hip_in_release == 0 && deferred() == 1 && n_unreg == unreg0 + 1, "munmap only defers");
    mvx_host_register_deferred(NULL, NULL, &u1, NULL);
    CHECK(u1 == u0 + 1, "counter agrees");
    mvx_host_register_enable(0, 0);                 /* off: flushes */
    CHECK(n_unreg == unreg0 + 2 && deferred() == 0, "off unregisters the rest");
    printf("{\"mode\": \"stub\", \"registers\": %ld, \"unregisters\": %ld, \"hip_in_release\": %ld}\n",
           n_reg, n_unreg, hip_in_release);
    return 0;
}
#endif

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

/* ---- neighbour frees and a release under a held registration (GPU) ---- */
static volatile int nb_stop, nb_go;
static char *volatile nb_a, *volatile nb_b;
static long nb_frees;
static float *nb_inval;
static size_t nb_bytes;
static volatile long nb_held_seen = -1;

static void *nb_worker(void *arg)
{
    (void)arg;
    while (!nb_stop) {
        char *a = nb_a, *b = nb_b;
        nb_a = NULL; nb_b = NULL;
        free(a);
        free(b);
        nb_a = malloc(64);
        nb_b = malloc(64);
        nb_frees += 2;
    }
    return NULL;
}

static void *inval_worker(void *arg)
{
    long held = 0;
    int i;
    (void)arg;
    struct timespec t0, t;
    while (!nb_go) ;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (i = 0; held < 1; i++) {
        mvx_host_register_deferred(NULL, &held, NULL, NULL);
        clock_gettime(CLOCK_MONOTONIC, &t);
        if (t.tv_sec - t0.tv_sec > 20) break;
    }
    nb_held_seen = held;
    mvx_host_invalidate(nb_inval, nb_bytes);       /* as a host MPI's hook would */
    return NULL;
}

static int neighbour(void)
{
    const size_t nb = 64 * MIB, n = nb / sizeof(float);
    float *x, *y;
    char *after_x, *after_y;
    long inv0, hits0, hits1, d0, d1, u0, u1, held_after;
    int rep, share_x, share_y;
    pthread_t th;
    mallopt(M_MMAP_THRESHOLD, 512 * MIB);          /* 64 MiB from the heap, beside other blocks */
    mallopt(M_TRIM_THRESHOLD, 1024 * MIB);
    {
        char *cx, *cy;
        share_x = heap_pair(&cx, &after_x, nb) == 0;
        if (!malloc(3 * 4096)) return 1;            /* y's pages apart from x's (else one union entry) */
        share_y = heap_pair(&cy, &after_y, nb) == 0;
        x = (float *)cx;
        y = (float *)cy;
    }
    CHECK(share_x && share_y, "the neighbours share the operands' boundary pages");
    CHECK(sum_check(x, y, n, 3) == 0, "first call");
    CHECK(entries() == 2, "both operands registered");
    inv0 = mvx_host_register_invalidations();
    mvx_host_register_stats(NULL, NULL, &hits0, NULL);
    nb_a = after_x;
    nb_b = after_y;
    CHECK(pthread_create(&th, NULL, nb_worker, NULL) == 0, "thread");
    for (rep = 0; rep < 24; rep++)
        CHECK(sum_check(x, y, n, 100 + (unsigned)rep) == 0, "bit-exact while the neighbours churn");
    nb_stop = 1;
    pthread_join(th, NULL);
    mvx_host_register_stats(NULL, NULL, &hits1, NULL);
    CHECK(mvx_host_register_invalidations() == inv0, "no neighbour free dropped a registration");
    CHECK(entries() == 2 && hits1 - hits0 == 48, "every call found both registrations");

    /* a release of x itself reported while a call holds it */
    mvx_host_register_deferred(&d0, NULL, &u0, NULL);
    nb_inval = x;
    nb_bytes = nb;
    CHECK(pthread_create(&th, NULL, inval_worker, NULL) == 0, "thread 2");
    nb_go = 1;
    CHECK(sum_check(x, y, n, 999) == 0, "bit-exact with the release deferred under it");
    pthread_join(th, NULL);
    mvx_host_register_deferred(&d1, &held_after, &u1, NULL);
    CHECK(nb_held_seen >= 1, "the release came while the call held the registration");
    CHECK(d1 == 0 && held_after == 0 && u1 >= u0 + 1, "unregistered once the call was done");
    CHECK(entries() == 1, "y stays registered");
    CHECK(sum_check(x, y, n, 1234) == 0, "the next call registers x again");
    printf("{\"mode\": \"neighbour\", \"neighbour_frees\": %ld, \"calls\": %d, \"held_seen\": %ld, "
           "\"unregistered\": %ld}\n", nb_frees, rep, (long)nb_held_seen, u1 - u0);
    free(nb_a);
    free(nb_b);
    free(x);
    free(y);
    CHECK(entries() == 0, "frees dropped the registrations");
    return 0;
}

/* ---- buffers under a neighbour's registration (GPU) ------------------- */
static volatile int sh_stop;
static float *sh_a, *sh_c;
static size_t sh_n;
static long sh_iters, sh_bad;

static void *sh_worker(void *arg)
{
    int len = (int)sh_n;
    MPI_Datatype t = MPI_FLOAT;
    (void)arg;
    while (!sh_stop) {
        MPIR_SUM(sh_a, sh_c, &len, &t);          /* c += a: holds A's registration while it runs */
        if (mvx_op_errno() != 0) sh_bad++;
        sh_iters++;
    }
    return NULL;
}

static int shadow(void)
{
    const size_t nb8 = 8 * MIB, n8 = nb8 / sizeof(float), nb = 64 * MIB, n = nb / sizeof(float);
    float *x, *y, *c0, *b2, *r1, *r2;
    char *pa, *pb;
    long bounced0, bounced1, calls = 0;
    MPI_Comm comm;
    pthread_t th;
    size_t i;
    int rep;
    mallopt(M_MMAP_THRESHOLD, 512 * MIB);
    mallopt(M_TRIM_THRESHOLD, 1024 * MIB);

    /* (a) the call's own operands sharing a page */
    CHECK(heap_adjacent(&pa, &pb, nb8, nb8) == 0, "adjacent pair");
    x = (float *)pa;
    y = (float *)pb;
    CHECK(((uintptr_t)((char *)x + nb8 - 1) & ~4095UL) == ((uintptr_t)y & ~4095UL), "x and y share a page");
    CHECK(sum_check(x, y, n8, 21) == 0, "adjacent operands, one call");
    CHECK(entries() == 1, "their registrations merged into one");
    CHECK(sum_check(x, y, n8, 22) == 0, "again, on the merged registration");
    free(x);
    free(y);
    CHECK(entries() == 0, "freed");

    /* (b) a neighbour of a registration another call holds */
    CHECK(heap_adjacent(&pa, &pb, nb, nb8) == 0, "B starts in A's last page");
    if (!malloc(3 * 4096)) return 1;
    sh_a = (float *)pa;
    sh_n = n;
    sh_c = malloc(nb);
    c0 = malloc(nb);
    b2 = malloc(nb8 + 3 * 4096);
    r1 = malloc(nb8 + 3 * 4096);
    r2 = malloc(nb8 + 3 * 4096);
    CHECK(sh_c && c0 && b2 && r1 && r2, "malloc");
    fill(sh_a, n, 31);
    fill(c0, n, 32);
    memcpy(sh_c, c0, nb);
    fill((float *)pb, n8, 33);
    fill(b2, n8, 34);
    CHECK(mvx_comm_init_local(&comm, 2, 0) == 0, "virtual communicator");
    mvx_host_register_deferred(NULL, NULL, NULL, &bounced0);
    CHECK(pthread_create(&th, NULL, sh_worker, NULL) == 0, "thread");
    for (rep = 0; rep < 40; rep++) {
        void *s[2] = {pb, b2}, *r[2] = {r1, r2};
        int rcs[2] = {-1, -1};
        memset(r1, 0, nb8);
        memset(r2, 0, nb8);
        CHECK(mvx_allreduce_multi(s, r, (int)n8, MPI_FLOAT, MPI_SUM, comm, rcs, NULL) == 0 && rcs[0] == 0 &&
              rcs[1] == 0, "allreduce");
        for (i = 0; i < n8; i++)
            if (r1[i] != ((float *)pb)[i] + b2[i] || r2[i] != r1[i]) break;
        CHECK(i == n8, "bit-exact beside a held registration");
        calls++;
    }
    sh_stop = 1;
    pthread_join(th, NULL);
    mvx_host_register_deferred(NULL, NULL, NULL, &bounced1);
    CHECK(sh_bad == 0, "the op thread's calls");
    for (i = 0; i < n; i++)
        if (sh_c[i] != c0[i] + (float)sh_iters * sh_a[i]) break;
    CHECK(i == n, "the op thread's result");
    printf("{\"mode\": \"shadow\", \"allreduce_calls\": %ld, \"op_calls\": %ld, \"bounced\": %ld}\n", calls,
           sh_iters, bounced1 - bounced0);
    mvx_comm_free(&comm);
    free(pa); free(pb); free(sh_c); free(c0); free(b2); free(r1); free(r2);
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
    rc = !strcmp(argv[1], "dry") ? dry() : !strcmp(argv[1], "gpu") ? gpu() : !strcmp(argv[1], "stress") ? stress()
       : !strcmp(argv[1], "neighbour") ? neighbour() : !strcmp(argv[1], "shadow") ? shadow()
#ifdef REG_STUB
       : !strcmp(argv[1], "stub") ? stub()
#endif
       : 2;
    mvx_host_register_enable(0, 0);
    if (rc == 0) printf("reg_app ok\n");
    return rc;
}
