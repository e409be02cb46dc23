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
 * MVX_HOST_REGISTER_MIN_KIB (default 1024) are never registered.
 * A registration must not outlive its memory: on MI355X a registered range
 * that was freed (unmapped) and handed out again by malloc at the same
 * address left the GPU in the memory-access-fault state at its next DMA
 * (round 4), and no CPU-side check can see the free
 * afterwards.  So, as the reference learns of released memory through its
 * hooks (mem_hooks.c), libmvx.so interposes the calls that release memory
 * (free, realloc, munmap, mremap, madvise, sbrk; below) and unlinks every
 * registration a release hits before the release; the unregistration itself
 * is deferred to the next libmvx entry and waits for the calls still using
 * the registration (dreg.c's deferred, refcounted scheme).  Mode 1 of the cache needs
 * those hooks in effect; mode 2 is for callers that report releases
 * themselves (mvx_host_unregister / mvx_host_invalidate: a dlopen'ed
 * library, or a host MPI whose own hooks call mvx_host_invalidate).
 */
#define _GNU_SOURCE 1   /* RTLD_NEXT, MREMAP_FIXED, malloc_usable_size */
#include <pthread.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <hip/hip_runtime_api.h>

#include "mvx_internal.h"

static void reg_flush(void);

/* (the registration cache's deferred releases are unregistered first: a
 * stale registration would make HIP report pages it no longer maps as
 * page-locked) */
int mvx_buf_kind(const void *p)
{
    hipPointerAttribute_t a;
    reg_flush();
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

/* How many slices / chunks behind the one just issued a host pipeline drains
 * its bounced result (MVX_HOST_DRAIN_LAG, 1 or 2; default 2).  Lag 1 (rounds
 * 1-4) made the host wait for the D2H of the chunk it had just queued the
 * H2D behind, and the DMA engines idled while it then copied the next chunk
 * in (tools/drain_lag_ab.sh: pageable 256 MiB op 11.3-13.5 ms against
 * 12.3-14.2 at lag 1, 64 MiB 3.2-3.3 against 3.5-4.0). */
int mvxi_host_drain_lag(void)
{
    static int lag = 0;
    if (!lag) {
        const char *v = getenv("MVX_HOST_DRAIN_LAG");
        int l = v ? atoi(v) : 2;
        lag = l < 1 ? 1 : l > STAGE_LAG_MAX ? STAGE_LAG_MAX : l;
    }
    return lag;
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

/* ---- the registration cache ------------------------------------------------
 * Entries are page-aligned [base, end) ranges -- the pages hipHostRegister
 * locked -- with the span [ulo, uhi) of the buffers the calls asked for.
 * The rules follow MVAPICH's dreg (mpid/ch_gen2/dreg.c):
 *   - no HIP call is made while the table's mutex is held;
 *   - a release never calls into HIP where it is reported (the hooks run
 *     inside free(), on any thread, HIP's own included): it only unlinks the
 *     entries the released memory overlaps, so that no later call finds
 *     them, and moves them to a deferred list (find_and_free_dregs_inside,
 *     dreg.c:1063-1080).  Deferred entries are unregistered at the next
 *     libmvx entry (reg_flush: every buffer-kind query, every registration,
 *     the end of every call that held one; flush_dereg_mrs_external,
 *     dreg.c:678-767);
 *   - an entry a call is using is never unregistered: a call takes a hold
 *     when it finds or makes the registration (mvxi_buf_kind_hold) and drops
 *     it after its last DMA (mvxi_buf_release); a deferred entry that is
 *     still held waits for its last hold (dreg.c:725-733, "still being
 *     referenced by other pending MPI operations"), and eviction and merging
 *     pass held entries by;
 *   - a release reported on a thread that is inside our own registration
 *     calls (HIP freeing its own memory inside hipHostRegister /
 *     hipHostUnregister) records nothing, as have_dereg() / have_dreg() make
 *     the reference's hook return (dreg.c:1066).
 * Which releases drop an entry: one that releases pages (munmap, mremap,
 * madvise, negative sbrk, mvx_host_invalidate) drops every entry whose
 * pages it overlaps; free / realloc of a heap block drops the entries whose
 * buffer span the block overlaps.  A block beside a registered buffer that
 * only shares its boundary page keeps the registration: no allocator gives
 * back a page that still holds a live buffer, so those pages stay mapped
 * (and pinned) for as long as the buffer lives. */

#define REG_MAX 64
/* new entries are refused while REG_MAX are deferred (checked at the insert
 * itself), so the table and the deferred list never hold more than
 * 2 * REG_MAX - 1 between them: every deferral moves a table entry */
#define REG_DEFER (2 * REG_MAX)
#define REG_FLY 8                  /* registrations in progress (hipHostRegister outside the lock) */
#define PAGE 4096UL
typedef struct { uintptr_t base, end, ulo, uhi; unsigned long stamp, id; int hold; } reg_t;
typedef struct { uintptr_t base, end, ulo, uhi; int used, stale; } reg_fly_t;
static struct {
    pthread_mutex_t mu;
    int init, on, dry;
    size_t min_bytes, max_bytes, total;
    unsigned long clock, next_id, hits, misses, evictions, failures, invalidations, bounced;
    int n, nd;
    reg_t e[REG_MAX];              /* the table: registered, findable */
    reg_t d[REG_DEFER];            /* deferred: released, still registered until unheld and flushed */
    reg_fly_t fly[REG_FLY];
} g_reg = { PTHREAD_MUTEX_INITIALIZER };

/* read without the lock: entries or registrations in progress exist, and the
 * span [lo, hi) covering all of them (a superset while they change); the
 * deferred count (reg_flush's fast path); HIP unregister calls made (or, dry,
 * that would have been) */
static volatile int g_reg_live, g_reg_nd;
static volatile uintptr_t g_reg_lo, g_reg_hi;
static volatile long g_reg_unregisters;

/* > 0 while this thread is inside our own hipHostRegister / Unregister */
static __thread int t_in_reg;

static void reg_env(void)
{
    const char *v;
    if (g_reg.init) return;
    g_reg.init = 1;
    v = getenv("MVX_HOST_REGISTER");
    g_reg.on = v ? atoi(v) : 0;
    if (g_reg.on == 1 && !mvx_host_hooks_active()) g_reg.on = 0;   /* nothing would see a release */
    if (g_reg.on != 1 && g_reg.on != 2) g_reg.on = 0;
    v = getenv("MVX_HOST_REGISTER_DRY");        /* tests: track ranges, no page-locking */
    g_reg.dry = v && atoi(v) == 1;
    v = getenv("MVX_HOST_REGISTER_MIN_KIB");
    g_reg.min_bytes = (size_t)(v ? atol(v) : 1024) << 10;
    v = getenv("MVX_HOST_REGISTER_MAX_MIB");
    g_reg.max_bytes = (size_t)(v ? atol(v) : 16384) << 20;
}

static void reg_span_locked(void)
{
    uintptr_t lo = UINTPTR_MAX, hi = 0;
    int i, live = g_reg.n;
    for (i = 0; i < g_reg.n; i++) {
        if (g_reg.e[i].base < lo) lo = g_reg.e[i].base;
        if (g_reg.e[i].end > hi) hi = g_reg.e[i].end;
    }
    for (i = 0; i < REG_FLY; i++)
        if (g_reg.fly[i].used) {
            live++;
            if (g_reg.fly[i].base < lo) lo = g_reg.fly[i].base;
            if (g_reg.fly[i].end > hi) hi = g_reg.fly[i].end;
        }
    __atomic_store_n(&g_reg_lo, live ? lo : UINTPTR_MAX, __ATOMIC_RELAXED);
    __atomic_store_n(&g_reg_hi, live ? hi : 0, __ATOMIC_RELAXED);
    __atomic_store_n(&g_reg_nd, g_reg.nd, __ATOMIC_RELEASE);
    __atomic_store_n(&g_reg_live, live, __ATOMIC_RELEASE);
}

/* entries leaving the table now, unregistered once the lock is dropped */
typedef struct { int n; uintptr_t base[REG_DEFER + REG_MAX]; } reg_out_t;

static void reg_take_locked(int i, reg_out_t *out)
{
    out->base[out->n++] = g_reg.e[i].base;
    g_reg.total -= g_reg.e[i].end - g_reg.e[i].base;
    g_reg.e[i] = g_reg.e[--g_reg.n];
}

/* entry i leaves the table for the deferred list (no HIP call) */
static void reg_defer_locked(int i)
{
    g_reg.d[g_reg.nd++] = g_reg.e[i];
    g_reg.total -= g_reg.e[i].end - g_reg.e[i].base;
    g_reg.e[i] = g_reg.e[--g_reg.n];
}

static void reg_unregister(uintptr_t base, int dry)
{
    __atomic_add_fetch(&g_reg_unregisters, 1, __ATOMIC_RELAXED);
    if (dry) return;
    t_in_reg++;
    (void)hipHostUnregister((void *)base);
    (void)hipGetLastError();
    t_in_reg--;
}

static void reg_release(const reg_out_t *out, int dry)
{
    int i;
    for (i = 0; i < out->n; i++) reg_unregister(out->base[i], dry);
}

/* unregister every deferred entry no call holds any more */
static void reg_flush(void)
{
    reg_out_t out;
    int i, dry;
    if (!__atomic_load_n(&g_reg_nd, __ATOMIC_ACQUIRE)) return;
    out.n = 0;
    pthread_mutex_lock(&g_reg.mu);
    for (i = g_reg.nd - 1; i >= 0; i--)
        if (g_reg.d[i].hold == 0) {
            out.base[out.n++] = g_reg.d[i].base;
            g_reg.d[i] = g_reg.d[--g_reg.nd];
        }
    reg_span_locked();
    dry = g_reg.dry;
    pthread_mutex_unlock(&g_reg.mu);
    reg_release(&out, dry);
}

static int overlaps(uintptr_t a0, uintptr_t a1, uintptr_t b0, uintptr_t b1) { return a0 < b1 && b0 < a1; }

/* A release of [lo, hi): unlink what it hits (reg_t rules above), mark the
 * registrations in progress it hits stale.  `block`: a heap block (free /
 * realloc), tested against the buffer spans; else pages.  No HIP call. */
static int reg_unlink(uintptr_t lo, uintptr_t hi, int block)
{
    int i, n = 0;
    if (!block) {
        lo &= ~(PAGE - 1);
        hi = (hi + PAGE - 1) & ~(PAGE - 1);
    }
    pthread_mutex_lock(&g_reg.mu);
    for (i = g_reg.n - 1; i >= 0; i--) {
        const reg_t *e = &g_reg.e[i];
        if (block ? overlaps(e->ulo, e->uhi, lo, hi) : overlaps(e->base, e->end, lo, hi)) {
            reg_defer_locked(i);
            n++;
        }
    }
    for (i = 0; i < REG_FLY; i++) {
        reg_fly_t *f = &g_reg.fly[i];
        if (f->used && (block ? overlaps(f->ulo, f->uhi, lo, hi) : overlaps(f->base, f->end, lo, hi))) f->stale = 1;
    }
    g_reg.invalidations += (unsigned long)n;
    reg_span_locked();
    pthread_mutex_unlock(&g_reg.mu);
    return n;
}

/* the host MPI's hooks report a release (mem_hooks.c -> dreg.c:1063): they
 * run inside the release, so the entries are only unlinked here and
 * unregistered at the next libmvx entry */
int mvx_host_invalidate(const void *addr, size_t bytes)
{
    const uintptr_t a = (uintptr_t)addr;
    if (!bytes || !__atomic_load_n(&g_reg_live, __ATOMIC_ACQUIRE)) return 0;
    return reg_unlink(a, a + bytes, 0);
}

int mvx_host_register_enable(int on, size_t max_bytes)
{
    if (on < 0 || on > 2) return MPI_ERR_ARG;
    if (on == 1 && !mvx_host_hooks_active()) return MPI_ERR_OTHER;
    pthread_mutex_lock(&g_reg.mu);
    reg_env();
    g_reg.on = on;
    if (max_bytes) g_reg.max_bytes = max_bytes;
    if (!g_reg.on)
        while (g_reg.n) reg_defer_locked(g_reg.n - 1);
    reg_span_locked();
    pthread_mutex_unlock(&g_reg.mu);
    reg_flush();
    return 0;
}

int mvx_host_unregister(const void *addr)
{
    const uintptr_t a = (uintptr_t)addr;
    int i, n = 0;
    pthread_mutex_lock(&g_reg.mu);
    for (i = g_reg.n - 1; i >= 0; i--)
        if (g_reg.e[i].base <= a && a < g_reg.e[i].end) {
            reg_defer_locked(i);          /* unregistered once no call holds it */
            n++;
        }
    reg_span_locked();
    pthread_mutex_unlock(&g_reg.mu);
    reg_flush();
    return n ? 0 : MPI_ERR_ARG;
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

long mvx_host_register_invalidations(void)
{
    long n;
    pthread_mutex_lock(&g_reg.mu);
    n = (long)g_reg.invalidations;
    pthread_mutex_unlock(&g_reg.mu);
    return n;
}

int mvx_host_register_deferred(long *deferred, long *held, long *unregisters, long *bounced)
{
    int i;
    long h = 0;
    pthread_mutex_lock(&g_reg.mu);
    for (i = 0; i < g_reg.n; i++) h += g_reg.e[i].hold > 0;
    for (i = 0; i < g_reg.nd; i++) h += g_reg.d[i].hold > 0;
    if (deferred) *deferred = g_reg.nd;
    if (held) *held = h;
    if (bounced) *bounced = (long)g_reg.bounced;
    pthread_mutex_unlock(&g_reg.mu);
    if (unregisters) *unregisters = __atomic_load_n(&g_reg_unregisters, __ATOMIC_RELAXED);
    return 0;
}

/* how many of the caller's holds (mine[]) are on entry id */
static int mine_on(unsigned long id, unsigned long *const *mine, int nmine)
{
    int i, n = 0;
    for (i = 0; i < nmine; i++) n += *mine[i] == id;
    return n;
}

/* Register [p, p + bytes) (page-widened) in the cache; MVX_BUF_PINNED when
 * the range is (now) registered, MVX_BUF_BOUNCE when its pages are partly
 * under a registration the cache cannot merge it with (held by another
 * call, deferred, or being registered by another thread), else what
 * mvx_buf_kind says.  `k` is p's kind as mvx_buf_kind reported it (after a
 * flush).  With `id`, a call's hold is taken on the entry and its id stored
 * (0: none); mine[0..nmine) are the call's earlier holds (mvxi_buf_kind_hold). */
static int reg_range(const void *p, size_t bytes, int k, unsigned long *id, unsigned long *const *mine, int nmine)
{
    const uintptr_t ulo = (uintptr_t)p, uhi = (uintptr_t)p + bytes;
    uintptr_t base, end;
    reg_out_t out;
    int i, cover = -1, overlap = 0, dry, ok, f = -1, conflict, carried = 0;
    unsigned long merged[REG_MAX];
    int nmerged = 0;
    hipError_t hr = hipSuccess;
    if (id) *id = 0;
    pthread_mutex_lock(&g_reg.mu);
    reg_env();
    if (!g_reg.on && !g_reg.n && !g_reg.nd) { pthread_mutex_unlock(&g_reg.mu); return k; }
    base = ulo & ~(PAGE - 1);
    end = (uhi + PAGE - 1) & ~(PAGE - 1);
    for (i = 0; i < g_reg.n; i++) {
        if (g_reg.e[i].base <= base && end <= g_reg.e[i].end) cover = i;
        else if (overlaps(g_reg.e[i].base, g_reg.e[i].end, base, end)) overlap = 1;
    }
    if (cover >= 0) {                                   /* dreg_find */
        reg_t *e = &g_reg.e[cover];
        e->stamp = ++g_reg.clock;
        if (ulo < e->ulo) e->ulo = ulo;
        if (uhi > e->uhi) e->uhi = uhi;
        g_reg.hits++;
        if (id) { e->hold++; *id = e->id; }
        pthread_mutex_unlock(&g_reg.mu);
        return MVX_BUF_PINNED;
    }
    for (i = 0; i < g_reg.nd; i++)                       /* released pages still pinned for a call */
        if (overlaps(g_reg.d[i].base, g_reg.d[i].end, base, end)) {
            g_reg.bounced++;
            pthread_mutex_unlock(&g_reg.mu);
            return MVX_BUF_BOUNCE;
        }
    for (i = 0; i < REG_FLY; i++)
        if (g_reg.fly[i].used && overlaps(g_reg.fly[i].base, g_reg.fly[i].end, base, end)) {
            g_reg.bounced++;
            pthread_mutex_unlock(&g_reg.mu);
            return MVX_BUF_BOUNCE;
        }
    if (k == MVX_BUF_PINNED && !overlap) {              /* the caller's own page-locked memory */
        pthread_mutex_unlock(&g_reg.mu);
        return k;
    }
    /* a range that runs past a registration of ours: the union replaces it
     * (a DMA must never read past the pinned pages) -- unless another call
     * is using that registration.  This call's own holds (its other
     * operands, no DMA issued yet) move to the union. */
    for (i = 0; i < g_reg.n; i++)
        if (g_reg.e[i].hold && overlaps(g_reg.e[i].base, g_reg.e[i].end, base, end) &&
            g_reg.e[i].hold != mine_on(g_reg.e[i].id, mine, nmine)) {
            g_reg.bounced++;
            pthread_mutex_unlock(&g_reg.mu);
            return MVX_BUF_BOUNCE;
        }
    out.n = 0;
    {
        uintptr_t u0 = ulo, u1 = uhi;
        for (i = g_reg.n - 1; i >= 0; i--)
            if (overlaps(g_reg.e[i].base, g_reg.e[i].end, base, end)) {
                if (g_reg.e[i].base < base) base = g_reg.e[i].base;
                if (g_reg.e[i].end > end) end = g_reg.e[i].end;
                if (g_reg.e[i].ulo < u0) u0 = g_reg.e[i].ulo;
                if (g_reg.e[i].uhi > u1) u1 = g_reg.e[i].uhi;
                if (g_reg.e[i].hold) { merged[nmerged++] = g_reg.e[i].id; carried += g_reg.e[i].hold; }
                reg_take_locked(i, &out);
            }
        ok = g_reg.on && end - base >= g_reg.min_bytes && end - base <= g_reg.max_bytes && g_reg.nd < REG_MAX;
        while (ok && g_reg.n && (g_reg.n == REG_MAX || g_reg.total + (end - base) > g_reg.max_bytes)) {
            int lru = -1;                               /* evict the least recently used unheld entry */
            for (i = 0; i < g_reg.n; i++)
                if (!g_reg.e[i].hold && (lru < 0 || g_reg.e[i].stamp < g_reg.e[lru].stamp)) lru = i;
            if (lru < 0) { ok = 0; break; }
            reg_take_locked(lru, &out);
            g_reg.evictions++;
        }
        for (i = 0; ok && i < REG_FLY; i++)
            if (!g_reg.fly[i].used) { f = i; break; }
        if (f < 0) ok = 0;
        if (ok) {
            g_reg.misses++;
            g_reg.fly[f].base = base; g_reg.fly[f].end = end;
            g_reg.fly[f].ulo = u0; g_reg.fly[f].uhi = u1;
            g_reg.fly[f].used = 1; g_reg.fly[f].stale = 0;
        }
    }
    /* this call's holds on the registrations just taken out: dropped here
     * (their ranges are unregistered below); if the union is registered
     * they move to it, else those operands read as unregistered -- the
     * caller re-reads their kinds (mvxi_buf_kind_hold returns the union's
     * verdict for them through `mine`) */
    for (i = 0; i < nmine; i++) {
        int m;
        for (m = 0; m < nmerged; m++)
            if (*mine[i] == merged[m]) *mine[i] = ~0UL;   /* moved: resolved below */
    }
    reg_span_locked();
    dry = g_reg.dry;
    pthread_mutex_unlock(&g_reg.mu);
    reg_release(&out, dry);
    if (!ok) {
        for (i = 0; i < nmine; i++)
            if (*mine[i] == ~0UL) *mine[i] = 0;           /* the operand lost its registration */
        return mvx_buf_kind(p);
    }
    if (!dry) {                                          /* dreg_register */
        t_in_reg++;
        hr = hipHostRegister((void *)base, end - base, hipHostRegisterDefault);
        t_in_reg--;
        if (hr != hipSuccess) (void)hipGetLastError();
    }
    pthread_mutex_lock(&g_reg.mu);
    {
        reg_fly_t *fl = &g_reg.fly[f];
        /* meanwhile: a release of these pages (stale), another entry over
         * them, or the table / the byte budget filled */
        conflict = fl->stale || g_reg.n == REG_MAX || g_reg.nd >= REG_MAX ||
                   g_reg.total + (end - base) > g_reg.max_bytes;
        for (i = 0; !conflict && i < g_reg.n; i++) conflict = overlaps(g_reg.e[i].base, g_reg.e[i].end, base, end);
        fl->used = 0;
        if (hr != hipSuccess) {
            g_reg.failures++;
        } else if (!conflict) {
            reg_t *e = &g_reg.e[g_reg.n++];
            e->base = base; e->end = end; e->ulo = fl->ulo; e->uhi = fl->uhi;
            e->stamp = ++g_reg.clock;
            e->id = ++g_reg.next_id;
            e->hold = (id ? 1 : 0) + carried;
            if (id) *id = e->id;
            for (i = 0; i < nmine; i++)
                if (*mine[i] == ~0UL) *mine[i] = e->id;   /* the operands merged in hold the union */
            g_reg.total += end - base;
        }
    }
    reg_span_locked();
    pthread_mutex_unlock(&g_reg.mu);
    if (hr != hipSuccess || conflict) {
        for (i = 0; i < nmine; i++)
            if (*mine[i] == ~0UL) *mine[i] = 0;
    }
    if (hr != hipSuccess) return mvx_buf_kind(p);
    if (conflict) {
        reg_unregister(base, dry);
        pthread_mutex_lock(&g_reg.mu);
        g_reg.bounced++;
        pthread_mutex_unlock(&g_reg.mu);
        return MVX_BUF_BOUNCE;
    }
    return MVX_BUF_PINNED;
}

int mvxi_buf_kind_hold(const void *p, size_t bytes, unsigned long *hold, unsigned long *const *mine, int nmine)
{
    const int k = mvx_buf_kind(p);                      /* flushes the deferred entries first */
    if (hold) *hold = 0;
    if (k == MVX_BUF_DEVICE || !p || !bytes) return k;
    return reg_range(p, bytes, k, hold, mine, nmine);
}

int mvxi_buf_kind_range(const void *p, size_t bytes)
{
    return mvxi_buf_kind_hold(p, bytes, NULL, NULL, 0);
}

/* a call's last DMA on the entry is done */
void mvxi_buf_release(unsigned long hold)
{
    int i, done = 0;
    if (!hold) return;
    pthread_mutex_lock(&g_reg.mu);
    for (i = 0; i < g_reg.n && !done; i++)
        if (g_reg.e[i].id == hold) { g_reg.e[i].hold--; done = 1; }
    for (i = 0; i < g_reg.nd && !done; i++)
        if (g_reg.d[i].id == hold) { g_reg.d[i].hold--; done = 1; }
    pthread_mutex_unlock(&g_reg.mu);
    reg_flush();
}

/* explicit registration (dreg_register without a transfer) */
int mvx_host_register(const void *addr, size_t bytes)
{
    int on;
    if (!addr || !bytes) return MPI_ERR_ARG;
    reg_flush();
    pthread_mutex_lock(&g_reg.mu);
    reg_env();
    on = g_reg.on;
    pthread_mutex_unlock(&g_reg.mu);
    if (!on) return MPI_ERR_OTHER;
    return reg_range(addr, bytes, g_reg.dry ? MVX_BUF_PAGEABLE : mvx_buf_kind(addr), NULL, NULL, 0) == MVX_BUF_PINNED
               ? MPI_SUCCESS : MPI_ERR_OTHER;
}

/* ---- release hooks (mpid/ch_gen2/mem_hooks.c:97-132) ------------------------
 * MVAPICH interposes munmap and its own malloc's negative sbrk and records
 * every registration inside a released range before the release
 * (find_and_free_dregs_inside, dreg.c:1063).  With glibc's malloc the
 * releases happen inside free() / realloc() (which unmap or trim through
 * libc-internal calls no munmap interposer sees), so libmvx.so interposes
 * those too: free / realloc unlink the registrations whose buffers overlap
 * the block [p, p + malloc_usable_size(p)), munmap / mremap / madvise
 * (DONTNEED, FREE, REMOVE) / negative sbrk those whose pages overlap the
 * range they release.  No hook calls into HIP: the unlinked registrations
 * are unregistered at the next libmvx entry, once no call holds them (the
 * cache's rules above).  Then the real call runs
 * (the next definition in the lookup order: glibc's, or an allocator
 * interposed after this library).  The hooks take effect when libmvx.so is
 * in the program's global scope ahead of libc -- a program linked with
 * -lmvx (mvx_host_hooks_active reports it); a library dlopen'ed without
 * that (ctypes) runs the cache under the unregister contract instead.
 * libmvx_embed.so has no hooks: the host MPI's own (mem_hooks.c) call
 * mvx_host_invalidate. */
#ifndef MVX_NO_MEMHOOKS
#include <dlfcn.h>
#include <malloc.h>
#include <sys/mman.h>
#include <sys/syscall.h>

extern void __libc_free(void *);
extern void *__libc_realloc(void *, size_t);

static void (*real_free)(void *);
static void *(*real_realloc)(void *, size_t);
static int (*real_munmap)(void *, size_t);
static void *(*real_mremap)(void *, size_t, size_t, int, ...);
static int (*real_madvise)(void *, size_t, int);
static void *(*real_sbrk)(intptr_t);

__attribute__((constructor)) static void hooks_resolve(void)
{
    real_free = (void (*)(void *))dlsym(RTLD_NEXT, "free");
    real_realloc = (void *(*)(void *, size_t))dlsym(RTLD_NEXT, "realloc");
    real_munmap = (int (*)(void *, size_t))dlsym(RTLD_NEXT, "munmap");
    real_mremap = (void *(*)(void *, size_t, size_t, int, ...))dlsym(RTLD_NEXT, "mremap");
    real_madvise = (int (*)(void *, size_t, int))dlsym(RTLD_NEXT, "madvise");
    real_sbrk = (void *(*)(intptr_t))dlsym(RTLD_NEXT, "sbrk");
}

/* cheap test first: no entries, or [lo, hi) outside every entry's span;
 * nothing while this thread is inside our own (de)registration (dreg.c:1066) */
static void hook_release(uintptr_t lo, uintptr_t hi, int block)
{
    if (!__atomic_load_n(&g_reg_live, __ATOMIC_ACQUIRE) || hi <= lo || t_in_reg) return;
    if (hi <= __atomic_load_n(&g_reg_lo, __ATOMIC_RELAXED) || lo >= __atomic_load_n(&g_reg_hi, __ATOMIC_RELAXED))
        return;
    reg_unlink(lo, hi, block);
}

static void hook_block(void *p)
{
    if (p && __atomic_load_n(&g_reg_live, __ATOMIC_ACQUIRE))
        hook_release((uintptr_t)p, (uintptr_t)p + malloc_usable_size(p), 1);
}

/* the definitions, named so their own addresses can be compared with what
 * the program's lookup finds (a reference to `free` here would go through
 * the PLT to whichever free is the process's) */
static void hook_free(void *p)
{
    hook_block(p);
    if (real_free) real_free(p);
    else __libc_free(p);
}
void free(void *p) __attribute__((alias("hook_free")));

void *realloc(void *p, size_t n)
{
    hook_block(p);
    return real_realloc ? real_realloc(p, n) : __libc_realloc(p, n);
}

static int hook_munmap(void *addr, size_t len)
{
    hook_release((uintptr_t)addr, (uintptr_t)addr + len, 0);
    if (real_munmap) return real_munmap(addr, len);
    return (int)syscall(SYS_munmap, addr, len);
}
int munmap(void *addr, size_t len) __attribute__((alias("hook_munmap")));

void *mremap(void *old, size_t old_len, size_t new_len, int flags, ...)
{
    void *target = NULL;
    va_list ap;
    hook_release((uintptr_t)old, (uintptr_t)old + old_len, 0);
    if (flags & MREMAP_FIXED) {
        va_start(ap, flags);
        target = va_arg(ap, void *);
        va_end(ap);
        hook_release((uintptr_t)target, (uintptr_t)target + new_len, 0);   /* replaced by the move */
    }
    if (real_mremap) return real_mremap(old, old_len, new_len, flags, target);
    return (void *)syscall(SYS_mremap, old, old_len, new_len, flags, target);
}

int madvise(void *addr, size_t len, int advice)
{
    if (advice == MADV_DONTNEED || advice == MADV_FREE || advice == MADV_REMOVE)
        hook_release((uintptr_t)addr, (uintptr_t)addr + len, 0);
    if (real_madvise) return real_madvise(addr, len, advice);
    return (int)syscall(SYS_madvise, addr, len, advice);
}

void *sbrk(intptr_t delta)
{
    extern void *__sbrk(intptr_t);
    if (delta < 0) {                                   /* mvapich_sbrk */
        const uintptr_t cur = (uintptr_t)(real_sbrk ? real_sbrk(0) : __sbrk(0));
        hook_release(cur + (uintptr_t)delta, cur, 0);
    }
    return real_sbrk ? real_sbrk(delta) : __sbrk(delta);
}

int mvx_host_hooks_active(void)
{
    return dlsym(RTLD_DEFAULT, "free") == (void *)hook_free && dlsym(RTLD_DEFAULT, "munmap") == (void *)hook_munmap;
}
#else
int mvx_host_hooks_active(void) { return 0; }
#endif


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
