/*
 * mvx_host.c -- host-memory side of the reduction path: MPI user buffers
 * live in the caller's address space (the reference's collectives read and
 * write them directly, src/coll/allreduce.c:57-92), so a host-buffer call
 * streams them through HBM.
 *
 *   mvx_host_pinned(p)   page-locked memory (hipHostMalloc / hipHostRegister):
 *                        DMA engines read and write it directly, async.
 *   mvx_pcopy(d, s, n)   memcpy split over a small persistent worker pool:
 *                        pageable user memory is copied into / out of pinned
 *                        bounce slots by host cores while the DMA engines
 *                        move the previous / next slice over PCIe.
 *
 * Why bounce buffers and not a registration cache: a cached hipHostRegister
 * of a user buffer goes stale when the user frees the buffer and malloc
 * hands the same range out again (MVAPICH's dreg needs malloc hooks for
 * that); registering per call costs about as much as the copy itself
 * (tools/h2d_probe.c: 4.6 ms per 256 MiB).  Callers that keep a buffer for
 * long can pin it themselves and get the zero-copy DMA path.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <hip/hip_runtime_api.h>

#include "mvx_internal.h"

int mvx_buf_kind(const void *p)
{
    hipPointerAttribute_t a;
    if (!p) return MVX_BUF_PAGEABLE;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return MVX_BUF_PAGEABLE;
    }
    if (a.type == hipMemoryTypeDevice || a.isManaged) return MVX_BUF_DEVICE;
    return a.type == hipMemoryTypeHost ? MVX_BUF_PINNED : MVX_BUF_PAGEABLE;
}

int mvx_host_pinned(const void *p)
{
    hipPointerAttribute_t a;
    if (!p) return 0;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    return a.type == hipMemoryTypeHost;
}

/* ---- parallel memcpy ---------------------------------------------------- */

#define PC_MAX_WORKERS 31
#define PC_MIN_SPLIT (1L << 20)    /* below this one thread copies */

/* one split copy at a time: `job` is held from publishing a copy until its
 * last part is done, so callers on several threads (MPIR_* op functions,
 * two communicators) queue whole jobs and no worker skips a generation */
static pthread_mutex_t g_pc_job = PTHREAD_MUTEX_INITIALIZER;

static struct {
    pthread_mutex_t mu;
    pthread_cond_t go, done;
    int nworkers;
    unsigned gen;
    int pending;
    char *dst;
    const char *src;
    size_t bytes;
} g_pc = { PTHREAD_MUTEX_INITIALIZER, PTHREAD_COND_INITIALIZER, PTHREAD_COND_INITIALIZER,
           -1, 0, 0, NULL, NULL, 0 };

/* part `i` of `n` of a copy, split at 4 KiB (parts are ceil(bytes / n)
 * rounded up, so the n parts cover every byte) */
static void pc_part(int i, int n, char *dst, const char *src, size_t bytes)
{
    const size_t per = ((bytes + (size_t)n - 1) / (size_t)n + 4095) & ~(size_t)4095;
    const size_t lo = per * (size_t)i;
    size_t hi = lo + per;
    if (lo >= bytes) return;
    if (hi > bytes) hi = bytes;
    memcpy(dst + lo, src + lo, hi - lo);
}

static void *pc_worker(void *arg)
{
    const int id = (int)(intptr_t)arg;
    unsigned seen = 0;
    for (;;) {
        char *d;
        const char *s;
        size_t b;
        int n;
        pthread_mutex_lock(&g_pc.mu);
        while (g_pc.gen == seen) pthread_cond_wait(&g_pc.go, &g_pc.mu);
        seen = g_pc.gen;
        d = g_pc.dst; s = g_pc.src; b = g_pc.bytes; n = g_pc.nworkers + 1;
        pthread_mutex_unlock(&g_pc.mu);
        pc_part(id, n, d, s, b);
        pthread_mutex_lock(&g_pc.mu);
        if (--g_pc.pending == 0) pthread_cond_signal(&g_pc.done);
        pthread_mutex_unlock(&g_pc.mu);
    }
    return NULL;
}

/* MVX_COPY_THREADS host threads copy (default 8, the caller included) */
static void pc_start(void)
{
    const char *e = getenv("MVX_COPY_THREADS");
    int n = e ? atoi(e) : 8, i, ok = 0;
    long ncpu = sysconf(_SC_NPROCESSORS_ONLN);
    if (n < 1) n = 1;
    if (ncpu > 0 && n > ncpu) n = (int)ncpu;
    if (n - 1 > PC_MAX_WORKERS) n = PC_MAX_WORKERS + 1;
    for (i = 1; i < n; i++) {
        pthread_t t;
        pthread_attr_t at;
        pthread_attr_init(&at);
        pthread_attr_setdetachstate(&at, PTHREAD_CREATE_DETACHED);
        if (pthread_create(&t, &at, pc_worker, (void *)(intptr_t)i) == 0) ok++;
        pthread_attr_destroy(&at);
        if (ok != i) break;
    }
    g_pc.nworkers = ok;
}

void mvx_pcopy(void *dst, const void *src, size_t bytes)
{
    int n;
    if (!bytes) return;
    pthread_mutex_lock(&g_pc.mu);
    if (g_pc.nworkers < 0) pc_start();
    n = g_pc.nworkers;
    if (n == 0 || (long)bytes < PC_MIN_SPLIT) {
        pthread_mutex_unlock(&g_pc.mu);
        memcpy(dst, src, bytes);
        return;
    }
    pthread_mutex_unlock(&g_pc.mu);
    pthread_mutex_lock(&g_pc_job);
    pthread_mutex_lock(&g_pc.mu);
    g_pc.dst = (char *)dst; g_pc.src = (const char *)src; g_pc.bytes = bytes;
    g_pc.pending = n;
    g_pc.gen++;
    pthread_cond_broadcast(&g_pc.go);
    pthread_mutex_unlock(&g_pc.mu);
    pc_part(0, n + 1, (char *)dst, (const char *)src, bytes);
    pthread_mutex_lock(&g_pc.mu);
    while (g_pc.pending) pthread_cond_wait(&g_pc.done, &g_pc.mu);
    pthread_mutex_unlock(&g_pc.mu);
    pthread_mutex_unlock(&g_pc_job);
}

int mvx_copy_threads(void)
{
    int n;
    pthread_mutex_lock(&g_pc.mu);
    if (g_pc.nworkers < 0) pc_start();
    n = g_pc.nworkers + 1;
    pthread_mutex_unlock(&g_pc.mu);
    return n;
}
