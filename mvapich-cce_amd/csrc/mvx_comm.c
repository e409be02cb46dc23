/*
 * mvx_comm.c -- communicators of libmvx.so: creation (RCCL, virtual,
 * caller-supplied transport), teardown, per-communicator knobs, per-phase
 * timing and RCCL's own view.  Every table a call works in hangs off its
 * communicator (mvx_comm_t.w, mvx_internal.h).
 *
 * Error codes keep the reference's form (mpi_error.h, nerrmsg.c:181:
 * code = class | kind << 6 | ring_id << 13 for messages created through
 * MPIR_Err_setmsg).
 */
#include <stdlib.h>
#include <string.h>

#include "mvx_internal.h"

/* ---------------------------------------------------------------------- */
/* error codes                                                            */

static int g_err_ring = 1;   /* error_big_ring_pos, nerrmsg.c:75 */

int mvxi_setmsg_code(int cls, int kind)
{
    int id = g_err_ring++;
    if (g_err_ring > 8192) g_err_ring = 1;
    return cls | (kind << MVX_ERR_CLASS_BITS) | (id << 13);
}

int MPI_Error_class(int errorcode, int *errorclass)
{
    if (errorclass) *errorclass = errorcode & ((1 << MVX_ERR_CLASS_BITS) - 1);
    return MPI_SUCCESS;
}

/* ---------------------------------------------------------------------- */
/* the communicator table                                                 */

#define MAX_COMMS 32
#define COMM_HANDLE_BASE 1000

static mvx_comm_t g_comms[MAX_COMMS];
static int g_have_world = 0;

mvx_comm_t *mvxi_get_comm(MPI_Comm h)
{
    int i;
    for (i = 0; i < MAX_COMMS; i++)
        if (g_comms[i].used && g_comms[i].handle == h) return &g_comms[i];
    return NULL;
}

mvx_work *mvxi_work(mvx_comm_t *c)
{
    if (!c->w) c->w = (mvx_work *)calloc(1, sizeof *c->w);
    return c->w;
}

/* The first communicator that finishes initialising becomes
 * MPI_COMM_WORLD (a failed init leaves the handle free for the retry). */
static void publish_comm(mvx_comm_t *c, MPI_Comm *out)
{
    if (!g_have_world) { c->handle = MPI_COMM_WORLD; g_have_world = 1; }
    *out = c->handle;
}

static mvx_comm_t *new_comm(MPI_Comm *out)
{
    int i;
    mvx_comm_reap();
    for (i = 0; i < MAX_COMMS; i++) {
        if (!g_comms[i].used) {
            memset(&g_comms[i], 0, sizeof g_comms[i]);
            g_comms[i].used = 1;
            g_comms[i].handle = COMM_HANDLE_BASE + i;
            *out = g_comms[i].handle;
            return &g_comms[i];
        }
    }
    return NULL;
}

/* ---- device flavour (mvx_tuning) --------------------------------------- */

static int env_int(const char *name, int *out)
{
    const char *v = getenv(name);
    if (!v) return 0;
    *out = atoi(v);
    return 1;
}

/* MPIR_Init's knob parsing for the _SMP_ devices, initutil.c:230-293 */
int mvx_tuning_from_env(mvx_tuning *t, int smp)
{
    int v, max_msg = 1 << 16;   /* shmem_coll_max_msg_size, mpid/ch_gen2/shmem_coll.c:47 */
    if (!t) return MPI_ERR_ARG;
    memset(t, 0, sizeof *t);
    t->shmem_coll_reduce_threshold = 1 << 10;      /* intra_fns_new.c:70-71 */
    t->shmem_coll_allreduce_threshold = 1 << 15;
    t->smp = smp ? 1 : 0;
    if (!t->smp) return MPI_SUCCESS;
    t->enable_shmem_collectives = 1;               /* initutil.c:146 */
    t->shmem_coll_ok = 1;
    if (env_int("VIADEV_USE_SHMEM_REDUCE", &v)) t->disable_shmem_reduce = !v;
    if (env_int("VIADEV_USE_SHMEM_ALLREDUCE", &v)) t->disable_shmem_allreduce = !v;
    if (env_int("VIADEV_USE_BLOCKING", &v) && v == 1) t->enable_shmem_collectives = 0;
    if (env_int("VIADEV_USE_SHMEM_COLL", &v) && v == 0) t->enable_shmem_collectives = 0;
    if (env_int("VIADEV_USE_SHARED_MEM", &v) && v == 0) t->enable_shmem_collectives = 0;
    if (env_int("MV_USE_SHARED_MEM", &v) && v == 0) t->enable_shmem_collectives = 0;
    env_int("VIADEV_SHMEM_COLL_MAX_MSG_SIZE", &max_msg);
    env_int("VIADEV_SHMEM_COLL_REDUCE_THRESHOLD", &t->shmem_coll_reduce_threshold);
    env_int("VIADEV_SHMEM_COLL_ALLREDUCE_THRESHOLD", &t->shmem_coll_allreduce_threshold);
    /* the reference prints "Shmem_coll_max_msg_size should be greater than
     * the thresholds" and exits (289-293); here the init call fails */
    if (max_msg < t->shmem_coll_reduce_threshold || max_msg < t->shmem_coll_allreduce_threshold)
        return MPI_ERR_OTHER;
    if (!t->enable_shmem_collectives) t->shmem_coll_ok = 0;
    return MPI_SUCCESS;
}

/* shmem collective blocks: every _SMP_ communicator's leader takes the first
 * free one of shmem_coll_blocks (create_2level_comm.c:199-225; 16 by default,
 * VIADEV_MAX_SHMEM_COLL_COMM, initutil.c:260-266) and frees it with the comm
 * (free_2level_comm, :96-100). */
#define MAX_SHMEM_BLOCKS 1024
static unsigned char g_shmem_taken[MAX_SHMEM_BLOCKS];

static int claim_shmem_block(void)
{
    int n = 16, i;
    env_int("VIADEV_MAX_SHMEM_COLL_COMM", &n);
    if (n > MAX_SHMEM_BLOCKS) n = MAX_SHMEM_BLOCKS;
    for (i = 0; i < n; i++)
        if (!g_shmem_taken[i]) { g_shmem_taken[i] = 1; return i; }
    return -1;
}

/* MVX_EXCHANGE = p2p | pipe[:slices] | coll (default p2p);
 * MVX_HOST_PIPELINE = 1: host buffers at p > 1 take the sliced pipeline;
 * MVX_GRAPH = 1: device calls are captured and replayed as HIP graphs */
static void exchange_from_env(mvx_comm_t *c)
{
    const char *e = getenv("MVX_EXCHANGE");
    int v;
    c->exch = MVX_EXCH_P2P;
    c->exch_slices = 4;
    c->host_sliced = env_int("MVX_HOST_PIPELINE", &v) && v == 1;
    c->graphs = env_int("MVX_GRAPH", &v) && v == 1;
    c->graph_cap = GRAPH_CACHE;
    if (env_int("MVX_GRAPH_CACHE", &v) && v >= 1 && v <= GRAPH_CACHE) c->graph_cap = v;
    c->graph_evict = mvxi_graph_evict_default();
    if (env_int("MVX_GRAPH_EVICT", &v) && v >= MVX_GRAPH_EVICT_NONE && v <= MVX_GRAPH_EVICT_ALL) c->graph_evict = v;
    if (!e) return;
    if (!strncmp(e, "pipe", 4)) {
        c->exch = MVX_EXCH_PIPE;
        if (e[4] == ':' && atoi(e + 5) > 0) c->exch_slices = atoi(e + 5);
    } else if (!strcmp(e, "coll")) {
        c->exch = MVX_EXCH_COLL;
    }
}

/* Which captured graphs may be destroyed mid-life on this HIP runtime.
 * HIP 7.0 (70051831, the runtime torch 2.10+rocm7.0 bundles) crashes in
 * hipGraphLaunch once execs of graphs with parallel branches (a fork / join
 * across streams) have been destroyed -- with no RCCL and no libmvx in the
 * process, while the same graphs kept alive, and single-branch graphs
 * destroyed, run clean (tools/graph_probe2.c churn_*);
 * HIP 7.2 (70226015, the image's /opt/rocm) runs all of it clean.  So from
 * 7.2 any graph may be destroyed; before it, only single-branch ones.
 * MVX_GRAPH_EVICT = 0 | 1 | 2 overrides (none / single-branch / all). */
int mvxi_graph_evict_default(void)
{
    int v = 0;
    if (hipRuntimeGetVersion(&v) != hipSuccess) { (void)hipGetLastError(); return MVX_GRAPH_EVICT_SERIAL; }
    return v >= 70200000 ? MVX_GRAPH_EVICT_ALL : MVX_GRAPH_EVICT_SERIAL;
}

/* a new communicator's flavour: MVX_DEVICE names the reference device */
static int comm_flavour(mvx_comm_t *c)
{
    const char *d = getenv("MVX_DEVICE");
    const int smp = d && (!strcmp(d, "ch_gen2") || !strcmp(d, "ch_smp") || !strcmp(d, "ch_gen2_ud"));
    int rc = mvx_tuning_from_env(&c->tune, smp);
    c->shmem_block = -1;
    exchange_from_env(c);
    if (rc) return rc;
    if (c->tune.smp && c->tune.enable_shmem_collectives) {
        c->shmem_block = claim_shmem_block();
        c->tune.shmem_coll_ok = c->shmem_block >= 0;
    }
    return MPI_SUCCESS;
}

static void release_shmem_block(mvx_comm_t *c)
{
    if (c->shmem_block >= 0) g_shmem_taken[c->shmem_block] = 0;
    c->shmem_block = -1;
}

int mvx_get_unique_id(void *id_out)
{
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess) return MPI_ERR_OTHER;
    memcpy(id_out, &id, MVX_UNIQUE_ID_BYTES);
    return MPI_SUCCESS;
}

/* ---- the caller's current device -----------------------------------------
 * Communicator creation and every call that works on a communicator switch
 * to its device for their duration and switch back: a C application driving
 * two devices from one thread keeps the device it had selected. */
int mvxi_dev_enter(int device)
{
    int prev = -1;
    if (hipGetDevice(&prev) != hipSuccess) { (void)hipGetLastError(); prev = -1; }
    if (prev != device && hipSetDevice(device) != hipSuccess) {
        (void)hipGetLastError();
        return MVXI_DEV_FAILED;
    }
    return prev;
}

void mvxi_dev_leave(int device, int prev)
{
    if (prev >= 0 && prev != device) (void)hipSetDevice(prev);
}

/* 0 if `device` can be selected and holds a context (a communicator can be
 * created on it); MPI_ERR_OTHER otherwise.  The current device is kept. */
int mvx_device_check(int device)
{
    int n = mvx_device_count(), prev, rc = MPI_SUCCESS;
    if (device < 0 || device >= n) return MPI_ERR_OTHER;
    prev = mvxi_dev_enter(device);
    if (prev == MVXI_DEV_FAILED) return MPI_ERR_OTHER;
    if (hipFree(NULL) != hipSuccess) { (void)hipGetLastError(); rc = MPI_ERR_OTHER; }
    mvxi_dev_leave(device, prev);
    return rc;
}

static int comm_init_rccl(MPI_Comm *comm, int rank, int size, int device, const void *unique_id)
{
    ncclUniqueId id;
    mvx_comm_t *c = new_comm(comm);
    if (!c) return MPI_ERR_INTERN;
    c->rank = rank; c->size = size; c->device = device; c->local = 0;
    if (comm_flavour(c)) { c->used = 0; return MPI_ERR_OTHER; }
    memcpy(&id, unique_id, MVX_UNIQUE_ID_BYTES);
    if (ncclCommInitRank(&c->nccl, size, id, rank) != ncclSuccess) {
        release_shmem_block(c);
        c->used = 0;
        return MPI_ERR_OTHER;
    }
    publish_comm(c, comm);
    return MPI_SUCCESS;
}

int mvx_comm_init(MPI_Comm *comm, int rank, int size, int device,
                  const void *unique_id)
{
    int prev, rc;
    if (!comm || size < 1 || size > MVX_MAXP || rank < 0 || rank >= size)
        return MPI_ERR_ARG;
    if ((prev = mvxi_dev_enter(device)) == MVXI_DEV_FAILED) return MPI_ERR_OTHER;
    rc = comm_init_rccl(comm, rank, size, device, unique_id);
    mvxi_dev_leave(device, prev);
    return rc;
}

int mvx_comm_init_local(MPI_Comm *comm, int size, int device)
{
    mvx_comm_t *c;
    int prev;
    if (!comm || size < 1 || size > MVX_MAXP) return MPI_ERR_ARG;
    if ((prev = mvxi_dev_enter(device)) == MVXI_DEV_FAILED) return MPI_ERR_OTHER;
    mvxi_dev_leave(device, prev);
    c = new_comm(comm);
    if (!c) return MPI_ERR_INTERN;
    c->rank = 0; c->size = size; c->device = device; c->local = 1;
    if (comm_flavour(c)) { c->used = 0; return MPI_ERR_OTHER; }
    publish_comm(c, comm);
    return MPI_SUCCESS;
}

/* The transport table is read up to `bytes` (the caller's sizeof): a table
 * from a header without the collective hooks is taken as having none, so
 * its COLL calls run as P2P instead of jumping through bytes it never set. */
int mvx_comm_init_transport_ex(MPI_Comm *comm, int rank, int size, int device,
                               const mvx_transport *transport, size_t bytes)
{
    mvx_comm_t *c;
    mvx_transport t;
    int prev;
    if (!comm || !transport || bytes < MVX_TRANSPORT_BASE_BYTES || size < 1 || size > MVX_MAXP ||
        rank < 0 || rank >= size)
        return MPI_ERR_ARG;
    memset(&t, 0, sizeof t);
    memcpy(&t, transport, bytes < sizeof t ? bytes : sizeof t);
    if (!t.start || !t.send || !t.recv || !t.end) return MPI_ERR_ARG;
    if (!t.alltoall || !t.allgather) t.alltoall = NULL, t.allgather = NULL;
    if ((prev = mvxi_dev_enter(device)) == MVXI_DEV_FAILED) return MPI_ERR_OTHER;
    mvxi_dev_leave(device, prev);
    c = new_comm(comm);
    if (!c) return MPI_ERR_INTERN;
    c->rank = rank; c->size = size; c->device = device; c->local = 0;
    if (comm_flavour(c)) { c->used = 0; return MPI_ERR_OTHER; }
    c->has_ops = 1;
    c->ops = t;
    publish_comm(c, comm);
    return MPI_SUCCESS;
}

int mvx_comm_init_transport(MPI_Comm *comm, int rank, int size, int device,
                            const mvx_transport *transport)
{
    return mvx_comm_init_transport_ex(comm, rank, size, device, transport, MVX_TRANSPORT_BASE_BYTES);
}

int mvx_copy(void *dst, const void *src, size_t bytes)
{
    return hipMemcpy(dst, src, bytes, hipMemcpyDefault) == hipSuccess ? MPI_SUCCESS : MPI_ERR_OTHER;
}

int mvx_stream_synchronize(void *stream)
{
    return hipStreamSynchronize((hipStream_t)stream) == hipSuccess ? MPI_SUCCESS : MPI_ERR_OTHER;
}

int mvx_device_count(void)
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) { (void)hipGetLastError(); return 0; }
    return n;
}

/* ---- teardown ------------------------------------------------------------
 * An aborted communicator's staging may still be read by work queued behind
 * the aborted transfers (a combine waiting on its stream).  Its allocations
 * go to a deferred list with an event recorded behind that work on every
 * stream the communicator used; mvx_comm_reap frees an entry once all its
 * events have completed (it runs at every communicator creation and
 * reserve, and may be called directly). */
#define MAX_ZOMBIES 64
#define Z_DEV 4
#define Z_PIN (1 + 2 * STAGE_NB)
#define Z_EV 4
typedef struct {
    int used, device;
    char *dev[Z_DEV];
    char *pin[Z_PIN];
    hipEvent_t ev[Z_EV];
    int nev;
    hipStream_t streams[3];   /* the communicator's own streams, destroyed at reap */
} zombie_t;
static zombie_t g_zombies[MAX_ZOMBIES];

static int zombie_ready(zombie_t *z)
{
    int i;
    for (i = 0; i < z->nev; i++) {
        hipError_t e = hipEventQuery(z->ev[i]);
        if (e == hipErrorNotReady) return 0;
        if (e != hipSuccess) (void)hipGetLastError();   /* a failed stream is drained too */
    }
    return 1;
}

int mvx_comm_reap(void)
{
    int i, j, left = 0, dev = -1;
    (void)hipGetDevice(&dev);
    for (i = 0; i < MAX_ZOMBIES; i++) {
        zombie_t *z = &g_zombies[i];
        if (!z->used) continue;
        if (!zombie_ready(z)) { left++; continue; }
        if (z->device != dev) (void)hipSetDevice(z->device);
        for (j = 0; j < Z_DEV; j++) if (z->dev[j]) hipFree(z->dev[j]);
        for (j = 0; j < Z_PIN; j++) if (z->pin[j]) hipHostFree(z->pin[j]);
        for (j = 0; j < z->nev; j++) hipEventDestroy(z->ev[j]);
        for (j = 0; j < 3; j++) if (z->streams[j]) hipStreamDestroy(z->streams[j]);
        if (z->device != dev && dev >= 0) (void)hipSetDevice(dev);
        memset(z, 0, sizeof *z);
    }
    return left;
}

/* park an aborted communicator's memory; 1 if parked, 0 if it must leak */
static int park(mvx_comm_t *c)
{
    hipStream_t watch[4];
    int i, n = 0;
    zombie_t *z = NULL;
    for (i = 0; i < MAX_ZOMBIES && !z; i++)
        if (!g_zombies[i].used) z = &g_zombies[i];
    if (!z) return 0;
    memset(z, 0, sizeof *z);
    z->used = 1;
    z->device = c->device;
    z->dev[0] = c->pool; z->dev[1] = c->hpool; z->dev[2] = c->upool; z->dev[3] = c->xpool;
    z->pin[0] = c->uhost;
    watch[n++] = c->last_st;
    if (c->cstream) watch[n++] = c->cstream;
    if (c->w && c->w->stage.ready) {
        stage_res_t *S = &c->w->stage;
        for (i = 0; i < STAGE_NB; i++) { z->pin[1 + 2 * i] = S->bin[i]; z->pin[2 + 2 * i] = S->bout[i]; }
        watch[n++] = S->sh;
        watch[n++] = S->sd;
        z->streams[1] = S->sh;
        z->streams[2] = S->sd;
        for (i = 0; i < STAGE_NB; i++) {
            hipEventDestroy(S->ein[i]);
            hipEventDestroy(S->eout[i]);
            hipEventDestroy(S->ex[i]);
        }
        memset(S, 0, sizeof *S);
    }
    z->streams[0] = c->cstream;
    for (i = 0; i < n && i < Z_EV; i++) {
        if (hipEventCreateWithFlags(&z->ev[z->nev], hipEventDisableTiming) != hipSuccess) continue;
        if (hipEventRecord(z->ev[z->nev], watch[i]) != hipSuccess) {
            hipEventDestroy(z->ev[z->nev]);
            (void)hipGetLastError();
            continue;
        }
        z->nev++;
    }
    return 1;
}

static int comm_release(MPI_Comm *comm, int abort)
{
    mvx_comm_t *c = comm ? mvxi_get_comm(*comm) : NULL;
    int i, device, prev;
    if (!c) return ERR_COMM_NULL_CODE;
    device = c->device;
    prev = mvxi_dev_enter(device);
    /* the graphs first: a captured RCCL group holds a reference on its
     * communicator, and ncclCommDestroy waits for every such reference to go
     * (measured: destroying the communicator first never returned).  An
     * aborted communicator's graphs may still be running: left to the
     * process, like any work queued behind its transfers. */
    if (!abort) {
        if (c->last_st || c->gstream) hipDeviceSynchronize();
        mvxi_graphs_clear(c);
    }
    if (c->nccl) {
        if (abort) ncclCommAbort(c->nccl);
        else ncclCommDestroy(c->nccl);
    }
    if (abort && park(c)) {
        c->cstream = NULL;     /* the parked entry owns it */
    } else if (!abort) {
        if (c->pool) hipFree(c->pool);
        if (c->hpool) hipFree(c->hpool);
        if (c->upool) hipFree(c->upool);
        if (c->uhost) hipHostFree(c->uhost);
        if (c->xpool) hipFree(c->xpool);
        if (c->w) mvxi_stage_release(&c->w->stage);
    }
    if (c->gstream) {
        hipStreamDestroy(c->gstream);
        hipEventDestroy(c->gev[0]);
        hipEventDestroy(c->gev[1]);
    }
    if (c->cstream) hipStreamDestroy(c->cstream);
    if (c->pev[0])
        for (i = 0; i < 4; i++) hipEventDestroy(c->pev[i]);
    if (c->tev_ready)
        for (i = 0; i < 4; i++) hipEventDestroy(c->tev[i]);
    free(c->w);
    release_shmem_block(c);
    if (c->handle == MPI_COMM_WORLD) g_have_world = 0;
    memset(c, 0, sizeof *c);
    *comm = 0;
    mvxi_dev_leave(device, prev);
    return MPI_SUCCESS;
}

int mvx_comm_free(MPI_Comm *comm) { return comm_release(comm, 0); }

/* ncclCommAbort stops the communicator's kernels without waiting for their
 * peers; the staging memory is parked until its streams drain (see park) */
int mvx_comm_abort(MPI_Comm *comm) { return comm_release(comm, 1); }

int MPI_Comm_size(MPI_Comm comm, int *size)
{
    mvx_comm_t *c = mvxi_get_comm(comm);
    if (!c) return ERR_COMM_NULL_CODE;
    *size = c->size;
    return MPI_SUCCESS;
}

int MPI_Comm_rank(MPI_Comm comm, int *rank)
{
    mvx_comm_t *c = mvxi_get_comm(comm);
    if (!c) return ERR_COMM_NULL_CODE;
    *rank = c->rank;
    return MPI_SUCCESS;
}

int mvx_comm_get_tuning(MPI_Comm comm, mvx_tuning *t)
{
    mvx_comm_t *c = mvxi_get_comm(comm);
    if (!c) return ERR_COMM_NULL_CODE;
    if (!t) return MPI_ERR_ARG;
    *t = c->tune;
    return MPI_SUCCESS;
}

/* Replaces the communicator's flavour and knobs as given (the shmem block
 * accounting stays with the communicator's creation-time claim). */
int mvx_comm_set_tuning(MPI_Comm comm, const mvx_tuning *t)
{
    mvx_comm_t *c = mvxi_get_comm(comm);
    if (!c) return ERR_COMM_NULL_CODE;
    if (!t) return MPI_ERR_ARG;
    c->tune = *t;
    return MPI_SUCCESS;
}

int mvx_comm_set_exchange(MPI_Comm comm, int mode, int slices)
{
    mvx_comm_t *c = mvxi_get_comm(comm);
    if (!c) return ERR_COMM_NULL_CODE;
    if (mode < MVX_EXCH_P2P || mode > MVX_EXCH_COLL || slices < 0) return MPI_ERR_ARG;
    c->exch = mode;
    if (slices > 0) c->exch_slices = slices;
    return MPI_SUCCESS;
}

int mvx_comm_get_exchange(MPI_Comm comm, int *mode, int *slices)
{
    mvx_comm_t *c = mvxi_get_comm(comm);
    if (!c) return ERR_COMM_NULL_CODE;
    if (mode) *mode = c->exch;
    if (slices) *slices = c->exch_slices;
    return MPI_SUCCESS;
}

int mvx_comm_set_host_pipeline(MPI_Comm comm, int on)
{
    mvx_comm_t *c = mvxi_get_comm(comm);
    if (!c) return ERR_COMM_NULL_CODE;
    c->host_sliced = on ? 1 : 0;
    return MPI_SUCCESS;
}

int mvx_comm_set_call_kinds(MPI_Comm comm, int kinds)
{
    mvx_comm_t *c = mvxi_get_comm(comm);
    if (!c) return ERR_COMM_NULL_CODE;
    if (kinds < MVX_KINDS_UNKNOWN || kinds > MVX_KINDS_HOST) return MPI_ERR_ARG;
    c->call_kinds = kinds;
    return MPI_SUCCESS;
}

int mvx_comm_set_graphs(MPI_Comm comm, int on)
{
    mvx_comm_t *c = mvxi_get_comm(comm);
    if (!c) return ERR_COMM_NULL_CODE;
    /* turning graphs off keeps what was captured (destroyed with the
     * communicator, mvx_exec.c); on again, they replay */
    c->graphs = on ? 1 : 0;
    c->graph_error = 0;
    return MPI_SUCCESS;
}

int mvx_comm_last_graph(MPI_Comm comm, int *state, int *error)
{
    mvx_comm_t *c = mvxi_get_comm(comm);
    if (!c) return ERR_COMM_NULL_CODE;
    if (state) *state = c->last_graph;
    if (error) *error = c->graph_error;
    return MPI_SUCCESS;
}

int mvx_comm_last_exchange(MPI_Comm comm, int *mode)
{
    mvx_comm_t *c = mvxi_get_comm(comm);
    if (!c) return ERR_COMM_NULL_CODE;
    if (!mode) return MPI_ERR_ARG;
    *mode = c->ran_exch;
    return MPI_SUCCESS;
}

/* RCCL's own reduction on this communicator's RCCL handle, for the
 * ablation SURVEY.md 8(e) keeps beside the path: ncclAllReduce /
 * ncclReduceScatter with ncclSum, RCCL's ring / tree order -- not the
 * reference's, so not bit-exact for floats, and no BAND / MAXLOC.  The MPI
 * entry points never call it; bench.py times it after its line. */
int mvx_comm_rccl_native(MPI_Comm comm, int coll, const void *sendbuf, void *recvbuf, size_t count,
                         MPI_Datatype dt, void *stream)
{
    hipStream_t st = (hipStream_t)stream;
    mvx_comm_t *c = mvxi_get_comm(comm);
    ncclDataType_t t;
    ncclResult_t r;
    int prev;
    if (!c) return ERR_COMM_NULL_CODE;
    if (c->local || c->has_ops || !c->nccl) return MPI_ERR_COMM;
    if (dt == MPI_FLOAT) t = ncclFloat32;
    else if (dt == MPI_DOUBLE) t = ncclFloat64;
    else if (dt == MPI_INT) t = ncclInt32;
    else if (dt == MPI_LONG || dt == MPI_LONG_LONG_INT) t = ncclInt64;
    else return MPI_ERR_TYPE;
    c->last_st = st;
    if (coll != MVX_COLL_ALLREDUCE && coll != MVX_COLL_REDUCE_SCATTER) return MPI_ERR_ARG;
    if ((prev = mvxi_dev_enter(c->device)) == MVXI_DEV_FAILED) return MPI_ERR_OTHER;
    if (coll == MVX_COLL_ALLREDUCE) r = ncclAllReduce(sendbuf, recvbuf, count, t, ncclSum, c->nccl, st);
    else r = ncclReduceScatter(sendbuf, recvbuf, count, t, ncclSum, c->nccl, st);
    mvxi_dev_leave(c->device, prev);
    return r == ncclSuccess ? MPI_SUCCESS : MPI_ERR_OTHER;
}

/* What RCCL itself reports for the communicator: its rank count
 * (ncclCommCount), the device it drives for this rank (ncclCommCuDevice)
 * and its version (ncclGetVersion) -- bench.py puts every rank's answer in
 * its line so "did RCCL see N ranks on N GPUs" is read off RCCL, not off
 * the launcher's environment.  MPI_ERR_COMM without an RCCL handle. */
int mvx_comm_rccl_info(MPI_Comm comm, int *nranks, int *device, int *version)
{
    mvx_comm_t *c = mvxi_get_comm(comm);
    if (!c) return ERR_COMM_NULL_CODE;
    if (c->local || c->has_ops || !c->nccl) return MPI_ERR_COMM;
    if (nranks && ncclCommCount(c->nccl, nranks) != ncclSuccess) return MPI_ERR_OTHER;
    if (device && ncclCommCuDevice(c->nccl, device) != ncclSuccess) return MPI_ERR_OTHER;
    if (version && ncclGetVersion(version) != ncclSuccess) return MPI_ERR_OTHER;
    return MPI_SUCCESS;
}

/* ---- per-phase timing of device calls -----------------------------------
 * With timing on, every device-buffer call records four events on its
 * stream: before phase A, after A, after B, after C (the pipelined variant,
 * whose phases overlap, records only the first and the last). */
int mvx_comm_set_phase_timing(MPI_Comm comm, int on)
{
    mvx_comm_t *c = mvxi_get_comm(comm);
    int i;
    if (!c) return ERR_COMM_NULL_CODE;
    if (on && !c->tev_ready) {
        const int prev = mvxi_dev_enter(c->device);
        int rc = prev == MVXI_DEV_FAILED ? MPI_ERR_OTHER : MPI_SUCCESS;
        for (i = 0; i < 4 && !rc; i++)
            if (hipEventCreate(&c->tev[i]) != hipSuccess) rc = MPI_ERR_OTHER;
        if (prev != MVXI_DEV_FAILED) mvxi_dev_leave(c->device, prev);
        if (rc) return rc;
        c->tev_ready = 1;
    }
    c->timing = on ? 1 : 0;
    c->tev_kind = TEV_NONE;
    return MPI_SUCCESS;
}

int mvx_comm_phase_times(MPI_Comm comm, float *ms)
{
    mvx_comm_t *c = mvxi_get_comm(comm);
    int i;
    if (!c) return ERR_COMM_NULL_CODE;
    if (!ms) return MPI_ERR_ARG;
    if (c->tev_kind == TEV_NONE) return MPI_ERR_OTHER;
    if (hipEventSynchronize(c->tev[3]) != hipSuccess) return MPI_ERR_OTHER;
    for (i = 0; i < 3; i++) {
        ms[i] = -1.0f;
        if (c->tev_kind == TEV_PHASES && hipEventElapsedTime(&ms[i], c->tev[i], c->tev[i + 1]) != hipSuccess)
            return MPI_ERR_OTHER;
    }
    return hipEventElapsedTime(&ms[3], c->tev[0], c->tev[3]) == hipSuccess ? MPI_SUCCESS : MPI_ERR_OTHER;
}

int mvxi_tev(mvx_comm_t *c, int i, hipStream_t st)
{
    if (!c->timing) return MPI_SUCCESS;
    return hipEventRecord(c->tev[i], st) == hipSuccess ? MPI_SUCCESS : MPI_ERR_OTHER;
}

int mvx_comm_set_stream(MPI_Comm comm, void *stream)
{
    mvx_comm_t *c = mvxi_get_comm(comm);
    if (!c) return ERR_COMM_NULL_CODE;
    c->stream = (hipStream_t)stream;
    return MPI_SUCCESS;
}

/* ---- staging pools --------------------------------------------------------- */

__thread int mvxi_capturing;

int mvxi_grow(char **buf, size_t *have, size_t need)
{
    if (need <= *have) return MPI_SUCCESS;
    if (mvxi_capturing) return MPI_ERR_OTHER;   /* no reallocation inside a graph capture */
    if (*buf) { hipDeviceSynchronize(); hipFree(*buf); *buf = NULL; *have = 0; }
    need = (need + (1 << 20) - 1) & ~(size_t)((1 << 20) - 1);
    if (hipMalloc((void **)buf, need) != hipSuccess) { *buf = NULL; return MPI_ERR_OTHER; }
    *have = need;
    return MPI_SUCCESS;
}

int mvxi_grow_host(char **buf, size_t *have, size_t need)
{
    if (need <= *have) return MPI_SUCCESS;
    if (mvxi_capturing) return MPI_ERR_OTHER;
    if (*buf) { hipHostFree(*buf); *buf = NULL; *have = 0; }
    need = (need + (1 << 20) - 1) & ~(size_t)((1 << 20) - 1);
    if (hipHostMalloc((void **)buf, need, hipHostMallocDefault) != hipSuccess) { *buf = NULL; return MPI_ERR_OTHER; }
    *have = need;
    return MPI_SUCCESS;
}

int mvx_comm_reserve(MPI_Comm comm, size_t bytes)
{
    mvx_comm_t *c = mvxi_get_comm(comm);
    int prev, rc;
    if (!c) return ERR_COMM_NULL_CODE;
    mvx_comm_reap();
    if ((prev = mvxi_dev_enter(c->device)) == MVXI_DEV_FAILED) return MPI_ERR_OTHER;
    rc = mvxi_grow_pool(c, bytes);
    mvxi_dev_leave(c->device, prev);
    return rc;
}
