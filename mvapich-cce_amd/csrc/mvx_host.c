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
 * Registration cache (opt-in: MVX_HOST_REGISTER=1, or
 * mvx_host_register_enable).  MVAPICH pins a user buffer once and reuses
 * the registration (mpid/ch_gen2/dreg.c:774-832, dreg_register / dreg_find);
 * here a pageable range a call uses is hipHostRegister'ed on first use and
 * kept, so later calls on it DMA directly instead of copying through the
 * bounce slots.  Entries are page-aligned [base, end) ranges, evicted least
 * recently used past MVX_HOST_REGISTER_MAX_MIB (default 16384); ranges under
 * MVX_HOST_REGISTER_MIN_KIB (default 1024) are never registered.  The
 * reference learns of freed memory through malloc hooks (mem_hooks.c); here
 * the contract is mvx_host_unregister(addr) before the memory is freed.
 * The contract is not optional: on MI355X a registered range that is freed
 * (unmapped) and handed out again by malloc at the same address, with no
 * mvx_host_unregister in between, left the GPU in the memory-access-fault
 * state at its next DMA (round 4).  No CPU-side check
 * sees the free, and a probing DMA would fault the same way; that is why
 * the cache is off unless the application asks for it and keeps the
 * contract.
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

/* ---- the registration cache ------------------------------------------------ */

#define REG_MAX 64
#define PAGE 4096UL
typedef struct { uintptr_t base, end; unsigned long stamp; } reg_t;
static struct {
    pthread_mutex_t mu;
    int init, on;
    size_t min_bytes, max_bytes, total;
    unsigned long clock, hits, misses, evictions, failures;
    int n;
    reg_t e[REG_MAX];
} g_reg = { PTHREAD_MUTEX_INITIALIZER, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, {{0, 0, 0}} };

static void reg_env(void)
{
    const char *v;
    if (g_reg.init) return;
    g_reg.init = 1;
    v = getenv("MVX_HOST_REGISTER");
    g_reg.on = v && atoi(v) == 1;
    v = getenv("MVX_HOST_REGISTER_MIN_KIB");
    g_reg.min_bytes = (size_t)(v ? atol(v) : 1024) << 10;
    v = getenv("MVX_HOST_REGISTER_MAX_MIB");
    g_reg.max_bytes = (size_t)(v ? atol(v) : 16384) << 20;
}

static void reg_drop(int i)
{
    (void)hipHostUnregister((void *)g_reg.e[i].base);
    (void)hipGetLastError();
    g_reg.total -= g_reg.e[i].end - g_reg.e[i].base;
    g_reg.e[i] = g_reg.e[--g_reg.n];
}

static void reg_drop_all(void)
{
    while (g_reg.n) reg_drop(g_reg.n - 1);
}

int mvx_host_register_enable(int on, size_t max_bytes)
{
    pthread_mutex_lock(&g_reg.mu);
    reg_env();
    g_reg.on = on ? 1 : 0;
    if (max_bytes) g_reg.max_bytes = max_bytes;
    if (!g_reg.on) reg_drop_all();
    pthread_mutex_unlock(&g_reg.mu);
    return 0;
}

int mvx_host_unregister(const void *addr)
{
    const uintptr_t a = (uintptr_t)addr;
    int i, found = 0;
    pthread_mutex_lock(&g_reg.mu);
    for (i = g_reg.n - 1; i >= 0; i--)
        if (g_reg.e[i].base <= a && a < g_reg.e[i].end) { reg_drop(i); found = 1; }
    pthread_mutex_unlock(&g_reg.mu);
    return found ? 0 : MPI_ERR_ARG;
}

int mvx_host_register_stats(long *entries, size_t *bytes, long *hits, long *misses)
{
    pthread_mutex_lock(&g_reg.mu);
    reg_env();
    if (entries) *entries = g_reg.n;
    if (bytes) *bytes = g_reg.total;
    if (hits) *hits = (long)g_reg.hits;
    if (misses) *misses = (long)g_reg.misses;
    pthread_mutex_unlock(&g_reg.mu);
    return 0;
}

int mvxi_buf_kind_range(const void *p, size_t bytes)
{
    const int k = mvx_buf_kind(p);
    uintptr_t base, end;
    int i, cover = -1, overlap = 0;
    if (k == MVX_BUF_DEVICE || !p || !bytes) return k;
    pthread_mutex_lock(&g_reg.mu);
    reg_env();
    if (!g_reg.on && !g_reg.n) { pthread_mutex_unlock(&g_reg.mu); return k; }
    base = (uintptr_t)p & ~(PAGE - 1);
    end = ((uintptr_t)p + bytes + PAGE - 1) & ~(PAGE - 1);
    for (i = 0; i < g_reg.n; i++) {
        if (g_reg.e[i].base <= base && end <= g_reg.e[i].end) cover = i;
        else if (g_reg.e[i].base < end && base < g_reg.e[i].end) overlap = 1;
    }
    if (cover >= 0) {                                   /* dreg_find */
        g_reg.e[cover].stamp = ++g_reg.clock;
        g_reg.hits++;
        pthread_mutex_unlock(&g_reg.mu);
        return MVX_BUF_PINNED;
    }
    if (k == MVX_BUF_PINNED && !overlap) {              /* the caller's own page-locked memory */
        pthread_mutex_unlock(&g_reg.mu);
        return k;
    }
    /* a range that runs past a registration of ours: the union replaces it
     * (a DMA must never read past the pinned pages) */
    for (i = g_reg.n - 1; i >= 0; i--)
        if (g_reg.e[i].base < end && base < g_reg.e[i].end) {
            if (g_reg.e[i].base < base) base = g_reg.e[i].base;
            if (g_reg.e[i].end > end) end = g_reg.e[i].end;
            reg_drop(i);
        }
    if (!g_reg.on || end - base < g_reg.min_bytes || end - base > g_reg.max_bytes) {
        pthread_mutex_unlock(&g_reg.mu);
        return mvx_buf_kind(p);
    }
    while (g_reg.n && (g_reg.n == REG_MAX || g_reg.total + (end - base) > g_reg.max_bytes)) {
        int lru = 0;                                    /* evict the least recently used */
        for (i = 1; i < g_reg.n; i++)
            if (g_reg.e[i].stamp < g_reg.e[lru].stamp) lru = i;
        reg_drop(lru);
        g_reg.evictions++;
    }
    g_reg.misses++;
    if (hipHostRegister((void *)base, end - base, hipHostRegisterDefault) != hipSuccess) {   /* dreg_register */
        (void)hipGetLastError();
        g_reg.failures++;
        pthread_mutex_unlock(&g_reg.mu);
        return mvx_buf_kind(p);
    }
    g_reg.e[g_reg.n].base = base;
    g_reg.e[g_reg.n].end = end;
    g_reg.e[g_reg.n].stamp = ++g_reg.clock;
    g_reg.n++;
    g_reg.total += end - base;
    pthread_mutex_unlock(&g_reg.mu);
    return MVX_BUF_PINNED;
}


/* A stream for work that must run beside the caller's stream.  HIP spreads
 * streams over GPU_MAX_HW_QUEUES hardware queues, and two streams that share
 * a queue run in submission order whatever their events say.  Mode (env
 * `env`, else `dflt`): "priority" -- the greatest stream priority, whose
 * streams HIP takes from a queue pool of their own; "cumask" -- every CU in
 * the stream's mask, which HIP gives a queue of its own; "plain". */
hipError_t mvxi_queue_stream(hipStream_t *s, const char *env, const char *dflt)
{
    const char *e = getenv(env);
    int least = 0, greatest = 0;
    if (!e) e = dflt;
    /* each flavour falls back to the next one if the runtime refuses it */
    if (!strcmp(e, "cumask")) {
        uint32_t mask[16];
        memset(mask, 0xff, sizeof mask);        /* 512 CUs: more than any part has */
        if (hipExtStreamCreateWithCUMask(s, 16, mask) == hipSuccess) return hipSuccess;
        (void)hipGetLastError();
        e = "priority";
    }
    if (!strcmp(e, "priority")) {
        if (hipDeviceGetStreamPriorityRange(&least, &greatest) == hipSuccess &&
            hipStreamCreateWithPriority(s, hipStreamNonBlocking, greatest) == hipSuccess)
            return hipSuccess;
        (void)hipGetLastError();
    }
    return hipStreamCreateWithFlags(s, hipStreamNonBlocking);
}
