/*
 * mvx_coll.c -- libmvx.so: the MPI reduction API of the reference, run on
 * MI355X.  Host code in C; device work goes through the C-ABI of
 * libmvx_hip.so (include/mvx_hip.h) and RCCL (one process per GPU, xGMI).
 *
 * Reference call stacks replaced:
 *   MPI_Allreduce (allreduce.c:57-92) -> collops->Allreduce -> intra_Allreduce
 *   MPI_Reduce    (reduce.c:62-96)    -> collops->Reduce    -> intra_Reduce
 *   MPI_Reduce_scatter (red_scat.c:60-90) -> intra_Reduce_scatter
 * Argument checks keep the reference's order and codes (mpi_error.h,
 * nerrmsg.c:181: code = class | kind << 6 | ring_id << 13 for messages
 * created through MPIR_Err_setmsg).  The collective itself runs the plan of
 * mvx_plan.c: RCCL grouped send/recv for the exchanges, one combine kernel
 * in the reference's order for the arithmetic.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include "mvx_coll.h"
#include "mvx_hip.h"
#include "mvx_internal.h"

/* ---------------------------------------------------------------------- */
/* error codes                                                            */

#define ERR_KIND_DEFAULT 1      /* MPIR_ERR_DEFAULT, mpi_error.h:119 */
#define ERR_KIND_ALIAS 7        /* MPIR_ERR_BUFFER_ALIAS, mpi_error.h:127 */
#define ERR_KIND_ROOT_TOOBIG 3  /* mpi_error.h:169 */
#define ERR_TYPE_NULL_CODE MVX_ERRCLASS_TO_CODE(MPI_ERR_TYPE, 5)  /* 323 */
#define ERR_COMM_NULL_CODE MVX_ERRCLASS_TO_CODE(MPI_ERR_COMM, 3)  /* 197 */

static int g_err_ring = 1;   /* error_big_ring_pos, nerrmsg.c:75 */

/* MPIR_Err_setmsg's return value (nerrmsg.c:111-182) */
static int setmsg_code(int cls, int kind)
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
/* communicators                                                          */

#define MAX_COMMS 32
#define COMM_HANDLE_BASE 1000

typedef struct {
    int used, rank, size, device, local;
    MPI_Comm handle;
    ncclComm_t nccl;
    hipStream_t stream;
    char *pool;          /* plan staging (received shards, temporaries) */
    size_t pool_bytes;
    char *hpool;         /* host-buffer staging */
    size_t hpool_bytes;
    char *upool;         /* user-op scratch: device (device functions) */
    size_t upool_bytes;
    char *uhost;         /* user-op scratch: pinned host (MPI_User_functions) */
    size_t uhost_bytes;
    char *xpool;         /* extent-layout scratch of packed (holey) datatypes */
    size_t xpool_bytes;
    mvx_tuning tune;     /* device flavour + knobs (mvx_coll.h) */
    int shmem_block;     /* claimed shmem collective block, -1 = none */
    int exch, exch_slices;      /* exchange variant, MVX_EXCH_* (mvx_coll.h) */
    int has_ops;                /* caller-supplied transport instead of RCCL */
    mvx_transport ops;
    hipStream_t cstream;        /* combine stream of the pipelined exchange */
    hipEvent_t pev[4];          /* its exchange-done / combine-done events */
    int timing;                 /* mvx_comm_set_phase_timing: events around phases A / B / C */
    int tev_ready, tev_kind;    /* events created; what the last timed call recorded (TEV_*) */
    hipEvent_t tev[4];          /* start, after A, after B, after C */
    int keep;                   /* this call's (op, type) is undefined: every combine keeps its inout */
    int ran_exch;               /* the variant the last call ran (mvx_comm_last_exchange), -1 none */
} mvx_comm_t;

static mvx_comm_t g_comms[MAX_COMMS];
static int g_have_world = 0;

static mvx_comm_t *get_comm(MPI_Comm h)
{
    int i;
    for (i = 0; i < MAX_COMMS; i++)
        if (g_comms[i].used && g_comms[i].handle == h) return &g_comms[i];
    return NULL;
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

/* MVX_EXCHANGE = p2p | pipe[:slices] | coll (default p2p) */
static void exchange_from_env(mvx_comm_t *c)
{
    const char *e = getenv("MVX_EXCHANGE");
    c->exch = MVX_EXCH_P2P;
    c->exch_slices = 4;
    if (!e) return;
    if (!strncmp(e, "pipe", 4)) {
        c->exch = MVX_EXCH_PIPE;
        if (e[4] == ':' && atoi(e + 5) > 0) c->exch_slices = atoi(e + 5);
    } else if (!strcmp(e, "coll")) {
        c->exch = MVX_EXCH_COLL;
    }
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

int mvx_comm_init(MPI_Comm *comm, int rank, int size, int device,
                  const void *unique_id)
{
    ncclUniqueId id;
    mvx_comm_t *c;
    if (!comm || size < 1 || size > MVX_MAXP || rank < 0 || rank >= size)
        return MPI_ERR_ARG;
    if (hipSetDevice(device) != hipSuccess) return MPI_ERR_OTHER;
    c = new_comm(comm);
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

int mvx_comm_init_local(MPI_Comm *comm, int size, int device)
{
    mvx_comm_t *c;
    if (!comm || size < 1 || size > MVX_MAXP) return MPI_ERR_ARG;
    if (hipSetDevice(device) != hipSuccess) return MPI_ERR_OTHER;
    c = new_comm(comm);
    if (!c) return MPI_ERR_INTERN;
    c->rank = 0; c->size = size; c->device = device; c->local = 1;
    if (comm_flavour(c)) { c->used = 0; return MPI_ERR_OTHER; }
    publish_comm(c, comm);
    return MPI_SUCCESS;
}

int mvx_comm_init_transport(MPI_Comm *comm, int rank, int size, int device,
                            const mvx_transport *transport)
{
    mvx_comm_t *c;
    if (!comm || !transport || !transport->start || !transport->send || !transport->recv ||
        !transport->end || size < 1 || size > MVX_MAXP || rank < 0 || rank >= size)
        return MPI_ERR_ARG;
    if (hipSetDevice(device) != hipSuccess) return MPI_ERR_OTHER;
    c = new_comm(comm);
    if (!c) return MPI_ERR_INTERN;
    c->rank = rank; c->size = size; c->device = device; c->local = 0;
    if (comm_flavour(c)) { c->used = 0; return MPI_ERR_OTHER; }
    c->has_ops = 1;
    c->ops = *transport;
    publish_comm(c, comm);
    return MPI_SUCCESS;
}

int mvx_copy(void *dst, const void *src, size_t bytes)
{
    return hipMemcpy(dst, src, bytes, hipMemcpyDefault) == hipSuccess ? MPI_SUCCESS : MPI_ERR_OTHER;
}

int mvx_stream_synchronize(void *stream)
{
    return hipStreamSynchronize((hipStream_t)stream) == hipSuccess ? MPI_SUCCESS : MPI_ERR_OTHER;
}

static int comm_release(MPI_Comm *comm, int abort)
{
    mvx_comm_t *c = comm ? get_comm(*comm) : NULL;
    if (!c) return ERR_COMM_NULL_CODE;
    if (c->nccl) {
        if (abort) ncclCommAbort(c->nccl);
        else ncclCommDestroy(c->nccl);
    }
    /* an aborted communicator's staging may still be read by work queued
     * behind the aborted transfers (a combine waiting on its stream): those
     * allocations are left to the process rather than freed under it */
    if (!abort) {
        if (c->pool) hipFree(c->pool);
        if (c->hpool) hipFree(c->hpool);
        if (c->upool) hipFree(c->upool);
        if (c->uhost) hipHostFree(c->uhost);
        if (c->xpool) hipFree(c->xpool);
    }
    if (c->cstream) {
        int i;
        hipStreamDestroy(c->cstream);
        for (i = 0; i < 4; i++) hipEventDestroy(c->pev[i]);
    }
    if (c->tev_ready) {
        int i;
        for (i = 0; i < 4; i++) hipEventDestroy(c->tev[i]);
    }
    release_shmem_block(c);
    if (c->handle == MPI_COMM_WORLD) g_have_world = 0;
    memset(c, 0, sizeof *c);
    *comm = 0;
    return MPI_SUCCESS;
}

int mvx_comm_free(MPI_Comm *comm) { return comm_release(comm, 0); }

/* ncclCommAbort stops the communicator's kernels without waiting for their
 * peers; the staging memory is not freed (see comm_release) */
int mvx_comm_abort(MPI_Comm *comm) { return comm_release(comm, 1); }

int MPI_Comm_size(MPI_Comm comm, int *size)
{
    mvx_comm_t *c = get_comm(comm);
    if (!c) return ERR_COMM_NULL_CODE;
    *size = c->size;
    return MPI_SUCCESS;
}

int MPI_Comm_rank(MPI_Comm comm, int *rank)
{
    mvx_comm_t *c = get_comm(comm);
    if (!c) return ERR_COMM_NULL_CODE;
    *rank = c->rank;
    return MPI_SUCCESS;
}

int mvx_comm_get_tuning(MPI_Comm comm, mvx_tuning *t)
{
    mvx_comm_t *c = get_comm(comm);
    if (!c) return ERR_COMM_NULL_CODE;
    if (!t) return MPI_ERR_ARG;
    *t = c->tune;
    return MPI_SUCCESS;
}

/* Replaces the communicator's flavour and knobs as given (the shmem block
 * accounting stays with the communicator's creation-time claim). */
int mvx_comm_set_tuning(MPI_Comm comm, const mvx_tuning *t)
{
    mvx_comm_t *c = get_comm(comm);
    if (!c) return ERR_COMM_NULL_CODE;
    if (!t) return MPI_ERR_ARG;
    c->tune = *t;
    return MPI_SUCCESS;
}

int mvx_comm_set_exchange(MPI_Comm comm, int mode, int slices)
{
    mvx_comm_t *c = get_comm(comm);
    if (!c) return ERR_COMM_NULL_CODE;
    if (mode < MVX_EXCH_P2P || mode > MVX_EXCH_COLL || slices < 0) return MPI_ERR_ARG;
    c->exch = mode;
    if (slices > 0) c->exch_slices = slices;
    return MPI_SUCCESS;
}

int mvx_comm_get_exchange(MPI_Comm comm, int *mode, int *slices)
{
    mvx_comm_t *c = get_comm(comm);
    if (!c) return ERR_COMM_NULL_CODE;
    if (mode) *mode = c->exch;
    if (slices) *slices = c->exch_slices;
    return MPI_SUCCESS;
}

int mvx_comm_last_exchange(MPI_Comm comm, int *mode)
{
    mvx_comm_t *c = get_comm(comm);
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
    mvx_comm_t *c = get_comm(comm);
    ncclDataType_t t;
    ncclResult_t r;
    if (!c) return ERR_COMM_NULL_CODE;
    if (c->local || c->has_ops || !c->nccl) return MPI_ERR_COMM;
    if (dt == MPI_FLOAT) t = ncclFloat32;
    else if (dt == MPI_DOUBLE) t = ncclFloat64;
    else if (dt == MPI_INT) t = ncclInt32;
    else if (dt == MPI_LONG || dt == MPI_LONG_LONG_INT) t = ncclInt64;
    else return MPI_ERR_TYPE;
    if (coll == MVX_COLL_ALLREDUCE) r = ncclAllReduce(sendbuf, recvbuf, count, t, ncclSum, c->nccl, st);
    else if (coll == MVX_COLL_REDUCE_SCATTER) r = ncclReduceScatter(sendbuf, recvbuf, count, t, ncclSum, c->nccl, st);
    else return MPI_ERR_ARG;
    return r == ncclSuccess ? MPI_SUCCESS : MPI_ERR_OTHER;
}

/* What RCCL itself reports for the communicator: its rank count
 * (ncclCommCount), the device it drives for this rank (ncclCommCuDevice)
 * and its version (ncclGetVersion) -- bench.py puts every rank's answer in
 * its line so "did RCCL see N ranks on N GPUs" is read off RCCL, not off
 * the launcher's environment.  MPI_ERR_COMM without an RCCL handle. */
int mvx_comm_rccl_info(MPI_Comm comm, int *nranks, int *device, int *version)
{
    mvx_comm_t *c = get_comm(comm);
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
#define TEV_NONE 0
#define TEV_PHASES 1
#define TEV_TOTAL 2

int mvx_comm_set_phase_timing(MPI_Comm comm, int on)
{
    mvx_comm_t *c = get_comm(comm);
    int i;
    if (!c) return ERR_COMM_NULL_CODE;
    if (on && !c->tev_ready) {
        if (hipSetDevice(c->device) != hipSuccess) return MPI_ERR_OTHER;
        for (i = 0; i < 4; i++)
            if (hipEventCreate(&c->tev[i]) != hipSuccess) return MPI_ERR_OTHER;
        c->tev_ready = 1;
    }
    c->timing = on ? 1 : 0;
    c->tev_kind = TEV_NONE;
    return MPI_SUCCESS;
}

int mvx_comm_phase_times(MPI_Comm comm, float *ms)
{
    mvx_comm_t *c = get_comm(comm);
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

/* event i of a timed call (no-op when timing is off) */
static int tev(mvx_comm_t *c, int i, hipStream_t st)
{
    if (!c->timing) return MPI_SUCCESS;
    return hipEventRecord(c->tev[i], st) == hipSuccess ? MPI_SUCCESS : MPI_ERR_OTHER;
}

int mvx_comm_set_stream(MPI_Comm comm, void *stream)
{
    mvx_comm_t *c = get_comm(comm);
    if (!c) return ERR_COMM_NULL_CODE;
    c->stream = (hipStream_t)stream;
    return MPI_SUCCESS;
}

static int grow(char **buf, size_t *have, size_t need)
{
    if (need <= *have) return MPI_SUCCESS;
    if (*buf) { hipDeviceSynchronize(); hipFree(*buf); *buf = NULL; *have = 0; }
    need = (need + (1 << 20) - 1) & ~(size_t)((1 << 20) - 1);
    if (hipMalloc((void **)buf, need) != hipSuccess) { *buf = NULL; return MPI_ERR_OTHER; }
    *have = need;
    return MPI_SUCCESS;
}

static int grow_host(char **buf, size_t *have, size_t need)
{
    if (need <= *have) return MPI_SUCCESS;
    if (*buf) { hipHostFree(*buf); *buf = NULL; *have = 0; }
    need = (need + (1 << 20) - 1) & ~(size_t)((1 << 20) - 1);
    if (hipHostMalloc((void **)buf, need, hipHostMallocDefault) != hipSuccess) { *buf = NULL; return MPI_ERR_OTHER; }
    *have = need;
    return MPI_SUCCESS;
}

int mvx_comm_reserve(MPI_Comm comm, size_t bytes)
{
    mvx_comm_t *c = get_comm(comm);
    if (!c) return ERR_COMM_NULL_CODE;
    return grow(&c->pool, &c->pool_bytes, bytes);
}

/* ---------------------------------------------------------------------- */
/* ops                                                                    */

#define MAX_USER_OPS 64
#define USER_OP_BASE 200
typedef struct {           /* struct MPIR_OP, include/mpiops.h:1-11 */
    MPI_User_function *op;     /* host function (MPI_Op_create) */
    MVX_Device_function *dop;  /* stream-ordered device function */
    unsigned cookie;
    int commute, permanent;
} mvx_op_t;
static mvx_op_t g_user_ops[MAX_USER_OPS];
#define OP_COOKIE 0xca01beafu

static int predefined(MPI_Op op) { return op >= MPI_MAX && op <= MPI_MAXLOC; }

static mvx_op_t *user_op(MPI_Op op)
{
    int i = op - USER_OP_BASE;
    if (i < 0 || i >= MAX_USER_OPS || g_user_ops[i].cookie != OP_COOKIE) return NULL;
    return &g_user_ops[i];
}

static int op_register(MPI_User_function *fn, MVX_Device_function *dfn, int commute, MPI_Op *op)
{
    int i;
    if (!op) return MPI_ERR_ARG;
    for (i = 0; i < MAX_USER_OPS; i++) {
        if (g_user_ops[i].cookie != OP_COOKIE) {
            g_user_ops[i].op = fn;
            g_user_ops[i].dop = dfn;
            g_user_ops[i].cookie = OP_COOKIE;
            g_user_ops[i].commute = commute;
            g_user_ops[i].permanent = 0;
            *op = USER_OP_BASE + i;
            return MPI_SUCCESS;
        }
    }
    return MPI_ERR_INTERN;
}

int MPI_Op_create(MPI_User_function *function, int commute, MPI_Op *op)
{
    return op_register(function, NULL, commute, op);
}

int mvx_op_create(MPI_User_function *function, int commute, MPI_Op *op)
{
    return op_register(function, NULL, commute, op);
}

int mvx_op_create_device(MVX_Device_function *function, int commute, MPI_Op *op)
{
    if (!function) return MPI_ERR_ARG;
    return op_register(NULL, function, commute, op);
}

/* ---- derived datatypes (the table is libmvx_hip.so's) ------------------ */

/* the type engine's codes: a negative value is MVX_SETMSG(class, kind), a
 * code the reference makes with MPIR_Err_setmsg (error ring position added) */
static int type_rc(int rc)
{
    if (rc >= 0) return rc;
    rc = -rc;
    return setmsg_code(rc & ((1 << MVX_ERR_CLASS_BITS) - 1), rc >> MVX_ERR_CLASS_BITS);
}

int MPI_Type_contiguous(int count, MPI_Datatype old, MPI_Datatype *newtype)
{
    return type_rc(mvx_type_contiguous(count, old, newtype));
}

int MPI_Type_vector(int count, int blocklen, int stride, MPI_Datatype old, MPI_Datatype *newtype)
{
    return type_rc(mvx_type_vector(count, blocklen, stride, old, newtype));
}

int MPI_Type_hvector(int count, int blocklen, MPI_Aint stride, MPI_Datatype old, MPI_Datatype *newtype)
{
    return type_rc(mvx_type_hvector(count, blocklen, stride, old, newtype));
}

int MPI_Type_indexed(int count, int *blocklens, int *indices, MPI_Datatype old, MPI_Datatype *newtype)
{
    return type_rc(mvx_type_indexed(count, blocklens, indices, old, newtype));
}

int MPI_Type_hindexed(int count, int *blocklens, MPI_Aint *indices, MPI_Datatype old, MPI_Datatype *newtype)
{
    return type_rc(mvx_type_hindexed(count, blocklens, indices, old, newtype));
}

int MPI_Type_struct(int count, int *blocklens, MPI_Aint *indices, MPI_Datatype *types, MPI_Datatype *newtype)
{
    return type_rc(mvx_type_struct(count, blocklens, indices, types, newtype));
}

int MPI_Type_commit(MPI_Datatype *datatype)   /* type_commit.c:41-143 */
{
    if (!datatype) return MVX_ERR_TYPE_NULL;
    return type_rc(mvx_type_commit(*datatype));
}

int MPI_Type_free(MPI_Datatype *datatype) { return type_rc(mvx_type_free(datatype)); }

int MPI_Type_extent(MPI_Datatype datatype, MPI_Aint *extent)
{
    long e;
    if (mvx_type_describe(datatype, NULL, NULL, &e, NULL)) return MVX_ERR_TYPE_NULL;
    if (!extent) return MPI_ERR_ARG;
    *extent = e;
    return MPI_SUCCESS;
}

int MPI_Type_size(MPI_Datatype datatype, int *size)
{
    long s;
    if (mvx_type_describe(datatype, NULL, NULL, NULL, &s)) return MVX_ERR_TYPE_NULL;
    if (!size) return MPI_ERR_ARG;
    *size = (int)s;
    return MPI_SUCCESS;
}

int MPI_Type_lb(MPI_Datatype datatype, MPI_Aint *displacement)   /* type_lb.c */
{
    long lb;
    if (mvx_type_layout(datatype, NULL, NULL, &lb, NULL, NULL, NULL)) return MVX_ERR_TYPE_NULL;
    if (!displacement) return MPI_ERR_ARG;
    *displacement = lb;
    return MPI_SUCCESS;
}

int MPI_Type_ub(MPI_Datatype datatype, MPI_Aint *displacement)   /* type_ub.c */
{
    long ub;
    if (mvx_type_layout(datatype, NULL, NULL, NULL, &ub, NULL, NULL)) return MVX_ERR_TYPE_NULL;
    if (!displacement) return MPI_ERR_ARG;
    *displacement = ub;
    return MPI_SUCCESS;
}

/* the plan kind of an op handle (an invalid handle plans as predefined and
 * is rejected by op_verdict) */
static int op_kind(MPI_Op op)
{
    const mvx_op_t *o = predefined(op) ? NULL : user_op(op);
    if (!o) return MVX_OPKIND_PREDEFINED;
    return o->commute ? MVX_OPKIND_USER_COMMUTE : MVX_OPKIND_USER_NONCOMMUTE;
}

int mvx_op_free(MPI_Op *op) { return MPI_Op_free(op); }

int mvx_device_count(void)
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) { (void)hipGetLastError(); return 0; }
    return n;
}

int MPI_Op_free(MPI_Op *op)  /* opfree.c:51-82 */
{
    mvx_op_t *o;
    if (!op) return MPI_ERR_ARG;
    if (*op == MPI_OP_NULL) return MVX_ERR_OP_NULL;
    if (predefined(*op)) return MVX_ERR_PERM_OP;
    o = user_op(*op);
    if (!o) return MPI_ERR_OP;
    memset(o, 0, sizeof *o);
    *op = MPI_OP_NULL;
    return MPI_SUCCESS;
}

/* The op's verdict on (op, type) before any data moves: 0, 329 (undefined
 * pair, reported only by ranks that call the op), MPI_ERR_OP (bad handle).
 * A user function accepts every datatype (the reference never checks). */
static int op_verdict(MPI_Op op, MPI_Datatype dt)
{
    if (predefined(op)) return mvx_op_apply(op, dt, NULL, NULL, 0, NULL);
    return user_op(op) ? MPI_SUCCESS : MPI_ERR_OP;
}

/* ---------------------------------------------------------------------- */
/* buffers                                                                */

static int is_device_ptr(const void *p)
{
    hipPointerAttribute_t a;
    if (!p) return 0;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    return a.type == hipMemoryTypeDevice || a.isManaged;
}

/* staging slot base with the same alignment mod 16 as `like`, so the
 * combine kernel keeps its 16-byte vector path */
static size_t slot_at(size_t cur, const void *like)
{
    size_t base = (cur + 255) & ~(size_t)255;
    return base + ((uintptr_t)like & 15);
}

static size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }

/* Consecutive staging slots are 4 KiB apart beyond their size: back-to-back
 * equal-size shards put the same chunk of every leaf at the same DRAM
 * interleave position, and the k-leaf combine then ran 5-6 % slower
 * (tools/tune_combine_layout.py, profiles/r01/tune_combine_layout.jsonl:
 * 53.9 vs 51.2 us for 8 x 32 MiB). */
#define SLOT_STAGGER 4096

/* ---- user ops: the combine program as a sequence of user calls --------
 * The reference hands a user function (*uop)(in, inout, &len, &type) its
 * operands in the roles the plan's program records, a swapped step being
 * uop(in = left, inout = right) whose result becomes the left value.  The
 * program runs over k scratch copies of the leaves (a user function writes
 * its inout operand, and leaves include the caller's send buffer); a swap
 * just renames which scratch buffer holds the left value. */
/* the handle a user function is given for a libmvx type (mvx_embed.h) */
#define MAX_TYPE_ALIASES 256
static struct { int type, handle; } g_alias[MAX_TYPE_ALIASES];
static int g_nalias;

int mvx_type_set_handle(int type, int handle)
{
    int i;
    for (i = 0; i < g_nalias; i++)
        if (g_alias[i].type == type) break;
    if (handle == type) {
        if (i < g_nalias) g_alias[i] = g_alias[--g_nalias];
        return MPI_SUCCESS;
    }
    if (i == g_nalias) {
        if (g_nalias == MAX_TYPE_ALIASES) return MPI_ERR_OTHER;
        g_nalias++;
    }
    g_alias[i].type = type;
    g_alias[i].handle = handle;
    return MPI_SUCCESS;
}

static MPI_Datatype user_handle(MPI_Datatype dt)
{
    int i;
    for (i = 0; i < g_nalias; i++)
        if (g_alias[i].type == dt) return g_alias[i].handle;
    return dt;
}

static int call_host(const mvx_op_t *o, const char *in, char *inout, long n, int esize,
                     MPI_Datatype dt)
{
    const MPI_Datatype uh = user_handle(dt);
    while (n > 0) {   /* the reference's len is an int */
        int len = n > 0x40000000L ? 0x40000000 : (int)n;
        MPI_Datatype t = uh;
        o->op((void *)in, inout, &len, &t);
        in += (long)len * esize;
        inout += (long)len * esize;
        n -= len;
    }
    return MPI_SUCCESS;
}

static int user_step(const mvx_op_t *o, const char *in, char *inout, long n, int esize,
                     MPI_Datatype dt, hipStream_t st)
{
    if (o->dop) return o->dop(in, inout, (size_t)n, user_handle(dt), st) ? MPI_ERR_OTHER : MPI_SUCCESS;
    return call_host(o, in, inout, n, esize, dt);
}

/* segment q's end: the next head after q, or k */
static int seg_end(const mvx_plan *P, int q)
{
    int e = q + 1;
    while (e < P->k && !(P->seg_heads >> e & 1ull)) e++;
    return e;
}

/* The user function sees every operand at its origin (element i at
 * origin + i * extent); the bytes it may touch are [origin + lo,
 * origin + lo + region) -- the whole vector for a contiguous type. */
static int combine_user(mvx_comm_t *c, const mvx_plan *P, const void *const *srcs,
                        const void *const *fold, void *dst, hipStream_t st, long lo, size_t region)
{
    const mvx_op_t *o = user_op(P->op);
    const long n = P->c_cnt, E = P->esize;
    const size_t slot = (region + 255) & ~(size_t)255;
    const int dev = o && o->dop;
    const hipMemcpyKind in_kind = dev ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
    char *y[MVX_MAXK] = {0}, *base;
    int q, l, s, e, rc;
    if (!o) return MPI_ERR_OP;
    if (dev) rc = grow(&c->upool, &c->upool_bytes, slot * (size_t)P->k * 2);
    else rc = grow_host(&c->uhost, &c->uhost_bytes, slot * (size_t)P->k * 2);
    if (rc) return rc;
    base = (dev ? c->upool : c->uhost) - lo;   /* origins of the scratch slots */
    for (q = 0; q < P->k; q++) {
        y[q] = base + slot * (size_t)q;
        if (hipMemcpyAsync(y[q] + lo, (const char *)srcs[q] + lo, region, in_kind, st) != hipSuccess)
            return MPI_ERR_OTHER;
        if (fold[q] && hipMemcpyAsync(base + slot * (size_t)(P->k + q) + lo, (const char *)fold[q] + lo, region,
                                      in_kind, st) != hipSuccess)
            return MPI_ERR_OTHER;
    }
    if (!dev && hipStreamSynchronize(st) != hipSuccess) return MPI_ERR_OTHER;
    for (q = 0; q < P->k; q++)   /* leaf q = op(leaf, fold): fold is `in` */
        if (fold[q] && (rc = user_step(o, base + slot * (size_t)(P->k + q), y[q], n, (int)E, P->dtype, st)))
            return rc;
    /* every segment's tree, then the chain over the segment heads; a swapped
     * step runs uop(in = left, inout = right) and renames the result left */
    for (s = 0; s < P->k; s = e) {
        e = seg_end(P, s);
        for (l = 0; (1 << l) < e - s; l++)
            for (q = s; q + (1 << l) < e; q += 2 << l) {
                char *a = y[q], *b = y[q + (1 << l)];
                if (P->tree_swap) { rc = user_step(o, a, b, n, (int)E, P->dtype, st); y[q] = b; y[q + (1 << l)] = a; }
                else rc = user_step(o, b, a, n, (int)E, P->dtype, st);
                if (rc) return rc;
            }
    }
    for (q = 1; q < P->k; q++) {
        char *a = y[0], *b = y[q];
        if (!(P->seg_heads >> q & 1ull)) continue;
        if (P->chain_swap >> q & 1ull) { rc = user_step(o, a, b, n, (int)E, P->dtype, st); y[0] = b; y[q] = a; }
        else rc = user_step(o, b, a, n, (int)E, P->dtype, st);
        if (rc) return rc;
    }
    if (hipMemcpyAsync((char *)dst + lo, y[0] + lo, region, dev ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice,
                       st) != hipSuccess)
        return MPI_ERR_OTHER;
    /* the pinned scratch is reused by the next call */
    return (!dev && hipStreamSynchronize(st) != hipSuccess) ? MPI_ERR_OTHER : MPI_SUCCESS;
}

/* ---- predefined ops over more than MVX_COMBINE_KMAX leaves --------------
 * A launch takes at most 8 leaves.  A TREE over m > 8 values is evaluated in
 * groups of 8 consecutive values into temporaries, then as the TREE over
 * those: S(8j, 3) is exactly the left operand the higher levels use, and a
 * truncated group tree is the truncated tree's restriction (q + 2^l < m
 * within the last group), so the association is the reference's.  A CHAIN
 * runs in windows of 8 whose result is the next window's first value. */
typedef struct { const void *p, *f; } leafref;
typedef struct { char *base; size_t slot; int used, cap; } scratch_t;

static char *scratch_take(scratch_t *S)
{
    return S->used < S->cap ? S->base + S->slot * (size_t)S->used++ : NULL;
}

static int launch_prog(const mvx_plan *P, const leafref *v, int m, unsigned tmask,
                       unsigned cmask, void *dst, hipStream_t st)
{
    const void *srcs[MVX_COMBINE_KMAX], *fold[MVX_COMBINE_KMAX];
    int q;
    if (!dst) return MPI_ERR_INTERN;
    for (q = 0; q < m; q++) { srcs[q] = v[q].p; fold[q] = v[q].f; }
    return mvx_op_program(P->op, P->dtype, srcs, fold, m, tmask, cmask, dst, (size_t)P->c_cnt, st);
}

static int tree_eval(const mvx_plan *P, leafref *v, int m, void *dst, scratch_t *S, hipStream_t st)
{
    int rc;
    while (m > MVX_COMBINE_KMAX) {
        const int ng = (m + 7) / 8;
        int g;
        for (g = 0; g < ng; g++) {
            const int len = m - 8 * g < 8 ? m - 8 * g : 8;
            char *t;
            if (len == 1 && !v[8 * g].f) { v[g] = v[8 * g]; continue; }
            t = scratch_take(S);
            if ((rc = launch_prog(P, v + 8 * g, len, mvx_tree_mask(len), 0u, t, st))) return rc;
            v[g].p = t; v[g].f = NULL;
        }
        m = ng;
    }
    return launch_prog(P, v, m, mvx_tree_mask(m), 0u, dst, st);
}

static int chain_eval(const mvx_plan *P, leafref *v, int m, void *dst, scratch_t *S, hipStream_t st)
{
    int i = 0, rc;
    while (m - i > MVX_COMBINE_KMAX) {
        char *t = scratch_take(S);
        if ((rc = launch_prog(P, v + i, 8, 0u, mvx_chain_mask(8), t, st))) return rc;
        i += 7;
        v[i].p = t; v[i].f = NULL;
    }
    return launch_prog(P, v + i, m - i, 0u, mvx_chain_mask(m - i), dst, st);
}

/* scratch slots a >8-leaf program can take: per segment its group temps
 * (< len/7 + 1 over all levels) and its value, plus the chain's windows */
static int wide_temps(const mvx_plan *P)
{
    int s, e, need = 0, nseg = 0;
    if (P->k <= MVX_COMBINE_KMAX) return 0;
    for (s = 0; s < P->k; s = e) {
        e = seg_end(P, s);
        need += (e - s) / 7 + 2;
        nseg++;
    }
    return need + nseg / 7 + 2;
}

static int combine_wide(const mvx_plan *P, const void *const *srcs, const void *const *fold,
                        void *dst, scratch_t *S, hipStream_t st)
{
    leafref v[MVX_MAXK], heads[MVX_MAXK];
    int q, s, e, nh = 0, rc;
    for (q = 0; q < P->k; q++) { v[q].p = srcs[q]; v[q].f = fold[q]; }
    if (seg_end(P, 0) == P->k) return tree_eval(P, v, P->k, dst, S, st);
    for (s = 0; s < P->k; s = e) {
        e = seg_end(P, s);
        if (e - s == 1) { heads[nh++] = v[s]; continue; }
        heads[nh].p = scratch_take(S);
        heads[nh].f = NULL;
        if ((rc = tree_eval(P, v + s, e - s, (void *)heads[nh].p, S, st))) return rc;
        nh++;
    }
    return chain_eval(P, heads, nh, dst, S, st);
}

/* ---- datatypes with holes (plan->packed) --------------------------------
 * Leaves arrive packed (type-map bytes only).  The op sees the reference's
 * layout -- count elements at the type's extent, as the (*uop) calls on
 * tmp_buf / recvbuf do (intra_fns_new.c:5505-5512) -- so the combine
 * unpacks every leaf into an extent-layout scratch slot (bytes outside the
 * type map read as zero), runs the program there and packs the result. */
static int combine_packed(mvx_comm_t *c, const mvx_plan *P, const void *const *srcs,
                          const void *const *fold, void *dst, hipStream_t st)
{
    const long n = P->c_cnt;
    const void *usrc[MVX_MAXK], *ufold[MVX_MAXK];
    long ext, lo, hi, a, b;
    size_t slot;
    int q, j = 0, nf = 0, rc, wide = 0;
    mvx_plan Q;
    char *out;
    if (mvx_type_describe(P->dtype, NULL, NULL, &ext, NULL) ||
        mvx_type_layout(P->dtype, NULL, NULL, NULL, NULL, &lo, &hi))
        return MPI_ERR_TYPE;
    Q = *P;
    Q.packed = 0;
    Q.esize = (int)ext;
    if (Q.opkind == MVX_OPKIND_PREDEFINED) {
        /* the kernel reads n C pair structs from each origin: the reference's
         * (*uop) calls on a struct type whose extent is not its first
         * member's pair struct overlap elements, which no reordering of the
         * calls reproduces -- refused */
        if (mvx_op_element_size(P->op, P->dtype) != ext) return MPI_ERR_TYPE;
        wide = wide_temps(&Q);
    }
    /* a slot covers the type map of n elements and the op's n * extent */
    a = lo < 0 ? lo : 0;
    b = (n - 1) * ext + hi;
    if (b < n * ext) b = n * ext;
    slot = al256((size_t)(b - a) + SLOT_STAGGER);
    for (q = 0; q < P->k; q++) nf += fold[q] != NULL;
    if ((rc = grow(&c->xpool, &c->xpool_bytes, slot * (size_t)(P->k + nf + 1 + wide)))) return rc;
    if (hipMemsetAsync(c->xpool, 0, slot * (size_t)(P->k + nf + 1), st) != hipSuccess) return MPI_ERR_OTHER;
    for (q = 0; q < P->k; q++) {
        usrc[q] = c->xpool + slot * (size_t)j++ - a;
        if ((rc = mvx_type_unpack(P->dtype, srcs[q], (void *)usrc[q], (size_t)n, st))) return rc;
        ufold[q] = NULL;
        if (fold[q]) {
            ufold[q] = c->xpool + slot * (size_t)j++ - a;
            if ((rc = mvx_type_unpack(P->dtype, fold[q], (void *)ufold[q], (size_t)n, st))) return rc;
        }
    }
    out = c->xpool + slot * (size_t)j++ - a;
    if (Q.opkind != MVX_OPKIND_PREDEFINED) {
        rc = combine_user(c, &Q, usrc, ufold, out, st, a, (size_t)(b - a));
    } else if (Q.k > MVX_COMBINE_KMAX) {
        scratch_t S;
        S.base = c->xpool + slot * (size_t)j - a;
        S.slot = slot; S.used = 0; S.cap = wide;
        rc = combine_wide(&Q, usrc, ufold, out, &S, st);
    } else {
        unsigned tm, cm;
        mvx_plan_masks(&Q, &tm, &cm);
        rc = mvx_op_program(Q.op, Q.dtype, usrc, ufold, Q.k, tm, cm, out, (size_t)n, st);
    }
    if (rc) return rc;
    return mvx_type_pack(P->dtype, out, dst, (size_t)n, st);
}

static int combine(mvx_comm_t *c, const mvx_plan *P, const char *const *leafp, void *dst,
                   scratch_t *S, hipStream_t st)
{
    const void *srcs[MVX_MAXK], *fold[MVX_MAXK];
    unsigned tm, cm;
    int q;
    for (q = 0; q < P->k; q++) {
        srcs[q] = leafp[P->leaf[q]];
        fold[q] = P->leaf_fold[q] >= 0 ? leafp[P->leaf_fold[q]] : NULL;
    }
    if (c->keep) {
        /* an undefined (op, type): the reference's op functions return with
         * inoutvec untouched (global_ops.c, e.g. 401-404), and every step's
         * left operand is the inout one (mvx_plan), so the program's result
         * is leaf 0 as it arrived -- packed or not, the same bytes */
        const size_t nb = (size_t)(P->c_cnt * P->esize);
        if (!nb || srcs[0] == dst) return MPI_SUCCESS;
        return hipMemcpyAsync(dst, srcs[0], nb, hipMemcpyDeviceToDevice, st) == hipSuccess ? MPI_SUCCESS
                                                                                        : MPI_ERR_OTHER;
    }
    if (P->packed) return combine_packed(c, P, srcs, fold, dst, st);
    if (P->opkind != MVX_OPKIND_PREDEFINED)
        return combine_user(c, P, srcs, fold, dst, st, 0, (size_t)(P->c_cnt * P->esize));
    if (P->k > MVX_COMBINE_KMAX) return combine_wide(P, srcs, fold, dst, S, st);
    mvx_plan_masks(P, &tm, &cm);
    return mvx_op_program(P->op, P->dtype, srcs, fold, P->k, tm, cm, dst, (size_t)P->c_cnt, st);
}

/* ---- transports ------------------------------------------------------ */
/* A phase is a group of point-to-point transfers.  RCCL issues them as one
 * ncclGroupStart/End; the loopback transport (virtual communicators) records
 * every rank's sends and receives of a phase and, once all ranks have
 * issued theirs, pairs them and copies device-to-device.  Both run the same
 * per-rank phase code below. */
#define LB_MAX (MVX_MAXP * MVX_MAXP)
typedef struct { int from, to; const void *src; void *dst; size_t bytes; int used; } lb_msg;
typedef struct { lb_msg send[LB_MAX], recv[LB_MAX]; int ns, nr; } loopback_t;

typedef struct mvx_xport {
    int (*start)(struct mvx_xport *);
    int (*end)(struct mvx_xport *);
    int (*send)(struct mvx_xport *, const void *, size_t, int, hipStream_t);
    int (*recv)(struct mvx_xport *, void *, size_t, int, hipStream_t);
    /* whole-communicator exchanges of the COLL variant (NULL: none) */
    int (*alltoall)(struct mvx_xport *, const void *, void *, size_t, hipStream_t);
    int (*allgather)(struct mvx_xport *, void *, size_t, hipStream_t);
    ncclComm_t nccl;
    loopback_t *lb;
    const mvx_transport *ops;   /* caller-supplied transport */
    hipStream_t st;             /* the stream its phases end on */
    int depth;                  /* nesting of start / end (one group) */
    int me;
} mvx_xport;

static int nc_start(mvx_xport *t) { (void)t; return ncclGroupStart() == ncclSuccess ? 0 : MPI_ERR_OTHER; }
static int nc_end(mvx_xport *t) { (void)t; return ncclGroupEnd() == ncclSuccess ? 0 : MPI_ERR_OTHER; }
static int nc_send(mvx_xport *t, const void *b, size_t n, int peer, hipStream_t st)
{ return ncclSend(b, n, ncclUint8, peer, t->nccl, st) == ncclSuccess ? 0 : MPI_ERR_OTHER; }
static int nc_recv(mvx_xport *t, void *b, size_t n, int peer, hipStream_t st)
{ return ncclRecv(b, n, ncclUint8, peer, t->nccl, st) == ncclSuccess ? 0 : MPI_ERR_OTHER; }
static int nc_alltoall(mvx_xport *t, const void *s, void *r, size_t n, hipStream_t st)
{ return ncclAllToAll(s, r, n, ncclUint8, t->nccl, st) == ncclSuccess ? 0 : MPI_ERR_OTHER; }
/* in place: the send operand is this rank's block of the receive buffer */
static int nc_allgather(mvx_xport *t, void *b, size_t n, hipStream_t st)
{ return ncclAllGather((char *)b + (size_t)t->me * n, b, n, ncclUint8, t->nccl, st) == ncclSuccess ? 0 : MPI_ERR_OTHER; }

/* a caller-supplied transport; nested start / end pairs form one group */
static int op_start(mvx_xport *t)
{
    if (t->depth++) return 0;
    return t->ops->start(t->ops->ctx) ? MPI_ERR_OTHER : 0;
}
static int op_end(mvx_xport *t)
{
    if (--t->depth) return 0;
    return t->ops->end(t->ops->ctx, (void *)t->st) ? MPI_ERR_OTHER : 0;
}
static int op_send(mvx_xport *t, const void *b, size_t n, int peer, hipStream_t st)
{ return t->ops->send(t->ops->ctx, b, n, peer, (void *)st) ? MPI_ERR_OTHER : 0; }
static int op_recv(mvx_xport *t, void *b, size_t n, int peer, hipStream_t st)
{ return t->ops->recv(t->ops->ctx, b, n, peer, (void *)st) ? MPI_ERR_OTHER : 0; }
static int op_alltoall(mvx_xport *t, const void *s, void *r, size_t n, hipStream_t st)
{ return t->ops->alltoall(t->ops->ctx, s, r, n, (void *)st) ? MPI_ERR_OTHER : 0; }
static int op_allgather(mvx_xport *t, void *b, size_t n, hipStream_t st)
{ return t->ops->allgather(t->ops->ctx, b, n, (void *)st) ? MPI_ERR_OTHER : 0; }

static int lb_nop(mvx_xport *t) { (void)t; return 0; }
static int lb_send(mvx_xport *t, const void *b, size_t n, int peer, hipStream_t st)
{
    lb_msg *m;
    (void)st;
    if (t->lb->ns >= LB_MAX) return MPI_ERR_INTERN;
    m = &t->lb->send[t->lb->ns++];
    m->from = t->me; m->to = peer; m->src = b; m->dst = NULL; m->bytes = n; m->used = 0;
    return 0;
}
static int lb_recv(mvx_xport *t, void *b, size_t n, int peer, hipStream_t st)
{
    lb_msg *m;
    (void)st;
    if (t->lb->nr >= LB_MAX) return MPI_ERR_INTERN;
    m = &t->lb->recv[t->lb->nr++];
    m->from = peer; m->to = t->me; m->src = NULL; m->dst = b; m->bytes = n; m->used = 0;
    return 0;
}
/* pair every receive with its send (same from/to, issue order) and copy */
static int lb_flush(loopback_t *lb, hipStream_t st)
{
    int i, j, rc = MPI_SUCCESS;
    for (i = 0; i < lb->nr && rc == MPI_SUCCESS; i++) {
        lb_msg *r = &lb->recv[i];
        for (j = 0; j < lb->ns; j++) {
            lb_msg *s = &lb->send[j];
            if (!s->used && s->from == r->from && s->to == r->to) break;
        }
        if (j == lb->ns || lb->send[j].bytes != r->bytes) { rc = MPI_ERR_INTERN; break; }
        lb->send[j].used = 1;
        if (hipMemcpyAsync(r->dst, lb->send[j].src, r->bytes, hipMemcpyDeviceToDevice, st) != hipSuccess)
            rc = MPI_ERR_OTHER;
    }
    for (j = 0; j < lb->ns && rc == MPI_SUCCESS; j++)
        if (!lb->send[j].used) rc = MPI_ERR_INTERN;   /* unmatched send */
    lb->ns = lb->nr = 0;
    return rc;
}

/* ---- one rank's execution of its plan ---------------------------------- */
typedef struct {
    const mvx_plan *P;              /* the plan, or the current slice of it */
    mvx_comm_t *c;
    const char *sendbuf;            /* device */
    char *recvbuf;                  /* device */
    char *pool;                     /* this rank's staging region */
    size_t slot[MVX_MAXP], tmp_off;
    size_t wide_off, wide_slot;     /* scratch of a > 8-leaf combine */
    int wide_n;
} rank_exec_t;

/* staging layout: one slot per received shard, plus the temporary result
 * of a non-root Reduce; returns the bytes this rank needs (slots are
 * SLOT_STAGGER apart beyond their size). */
static size_t exec_layout(rank_exec_t *X)
{
    const mvx_plan *P = X->P;
    const long E = P->esize;
    const char *like = X->sendbuf + P->c_src_off * E;
    size_t need = 0;
    int s;
    for (s = 0; s < P->p; s++) {
        X->slot[s] = 0;
        if (P->a_recv[s].cnt) {
            X->slot[s] = slot_at(need, like);
            need = X->slot[s] + P->a_recv[s].cnt * E + SLOT_STAGGER;
        }
    }
    X->tmp_off = 0;
    if (P->c_dst_tmp) { X->tmp_off = slot_at(need, like); need = X->tmp_off + P->c_cnt * E; }
    X->wide_n = P->has_combine ? wide_temps(P) : 0;
    X->wide_off = X->wide_slot = 0;
    if (X->wide_n) {
        X->wide_off = slot_at(need, like);
        X->wide_slot = ((size_t)(P->c_cnt * E) + SLOT_STAGGER + 255) & ~(size_t)255;
        need = X->wide_off + X->wide_slot * (size_t)X->wide_n;
    }
    return need;
}

static char *exec_out(const rank_exec_t *X)
{
    const mvx_plan *P = X->P;
    return P->c_dst_tmp ? X->pool + X->tmp_off : X->recvbuf + P->c_dst_off * P->esize;
}

/* phase A: shards to the rank that combines them */
static int exec_phase_a(rank_exec_t *X, mvx_xport *t, hipStream_t st)
{
    const mvx_plan *P = X->P;
    const long E = P->esize;
    int s, any = 0, rc = 0, rc2;
    for (s = 0; s < P->p; s++) any |= (P->a_send[s].cnt || P->a_recv[s].cnt);
    if (!any) return MPI_SUCCESS;
    if ((rc = t->start(t))) return rc;
    for (s = 0; s < P->p && !rc; s++) {
        if (P->a_send[s].cnt)
            rc = t->send(t, X->sendbuf + P->a_send[s].off * E, (size_t)(P->a_send[s].cnt * E), s, st);
        if (!rc && P->a_recv[s].cnt)
            rc = t->recv(t, X->pool + X->slot[s], (size_t)(P->a_recv[s].cnt * E), s, st);
    }
    rc2 = t->end(t);
    return rc ? rc : rc2;
}

/* phase B: the reference's whole combine tree for this rank's block */
static int exec_phase_b(rank_exec_t *X, hipStream_t st)
{
    const mvx_plan *P = X->P;
    const long E = P->esize;
    const char *leafp[MVX_MAXP];
    scratch_t S;
    int s;
    if (!P->has_combine || P->c_cnt == 0) return MPI_SUCCESS;
    for (s = 0; s < P->p; s++)
        leafp[s] = (s == P->rank) ? X->sendbuf + P->c_src_off * E : X->pool + X->slot[s];
    S.base = X->pool + X->wide_off;
    S.slot = X->wide_slot;
    S.used = 0;
    S.cap = X->wide_n;
    return combine(X->c, P, leafp, exec_out(X), &S, st);
}

/* phase C: combined blocks to the ranks that need them */
static int exec_phase_c(rank_exec_t *X, mvx_xport *t, hipStream_t st)
{
    const mvx_plan *P = X->P;
    const long E = P->esize;
    int s, any = 0, rc = 0, rc2;
    for (s = 0; s < P->p; s++) any |= (P->b_send[s].cnt || P->b_recv[s].cnt);
    if (!any) return MPI_SUCCESS;
    if ((rc = t->start(t))) return rc;
    for (s = 0; s < P->p && !rc; s++) {
        if (P->b_send[s].cnt)
            rc = t->send(t, exec_out(X), (size_t)(P->b_send[s].cnt * E), s, st);
        if (!rc && P->b_recv[s].cnt)
            rc = t->recv(t, X->recvbuf + P->b_recv[s].off * E, (size_t)(P->b_recv[s].cnt * E), s, st);
    }
    rc2 = t->end(t);
    return rc ? rc : rc2;
}

/* every local rank through phases A, B, C: one rank over RCCL, or all ranks
 * of a virtual communicator over the loopback transport (whose transfers
 * are paired once every rank has issued its phase) */
static int exec_group(rank_exec_t *X, mvx_xport *t, int nr, hipStream_t st, mvx_comm_t *timed)
{
    int r, rc;
    if (timed && (rc = tev(timed, 0, st))) return rc;
    for (r = 0; r < nr; r++)
        if ((rc = exec_phase_a(&X[r], &t[r], st))) return rc;
    if (t[0].lb && (rc = lb_flush(t[0].lb, st))) return rc;
    if (timed && (rc = tev(timed, 1, st))) return rc;
    for (r = 0; r < nr; r++)
        if ((rc = exec_phase_b(&X[r], st))) return rc;
    if (timed && (rc = tev(timed, 2, st))) return rc;
    for (r = 0; r < nr; r++)
        if ((rc = exec_phase_c(&X[r], &t[r], st))) return rc;
    if (t[0].lb && (rc = lb_flush(t[0].lb, st))) return rc;
    if (timed && (rc = tev(timed, 3, st))) return rc;
    if (timed && timed->timing) timed->tev_kind = TEV_PHASES;
    return MPI_SUCCESS;
}

/* ---- slices ------------------------------------------------------------
 * Slice i of a plan restricts every range to [i*cs, (i+1)*cs) relative to
 * its own start.  Matched send / receive ranges have equal counts on both
 * sides, so their slices stay matched; the combine range, its staging slots
 * and the combined block slice together.  Block boundaries (the
 * cnts[i] = n/pof2 of intra_fns_new.c:5645-5651) are untouched, so every
 * element keeps its leaves, order and operand roles: slicing changes when a
 * byte moves, never what is computed. */
static void slice_range(mvx_range *r, long lo, long cs)
{
    long c = r->cnt - lo;
    if (c > cs) c = cs;
    if (c <= 0) { r->off = 0; r->cnt = 0; }
    else r->off += lo;
    if (c > 0) r->cnt = c;
}

static void plan_slice(const mvx_plan *P, long i, long cs, mvx_plan *Q)
{
    const long lo = i * cs;
    long c = P->c_cnt - lo;
    int s;
    *Q = *P;
    for (s = 0; s < P->p; s++) {
        slice_range(&Q->a_send[s], lo, cs);
        slice_range(&Q->a_recv[s], lo, cs);
        slice_range(&Q->b_send[s], lo, cs);
        slice_range(&Q->b_recv[s], lo, cs);
    }
    if (c > cs) c = cs;
    if (c < 0) c = 0;
    Q->c_cnt = c;
    Q->c_src_off = P->c_src_off + lo;
    Q->c_dst_off = P->c_dst_off + lo;
}

/* the longest range of a plan (slices needed = ceil(span / cs)) */
static long plan_span(const mvx_plan *P)
{
    long m = P->has_combine ? P->c_cnt : 0;
    int s;
    for (s = 0; s < P->p; s++) {
        if (P->a_send[s].cnt > m) m = P->a_send[s].cnt;
        if (P->a_recv[s].cnt > m) m = P->a_recv[s].cnt;
        if (P->b_send[s].cnt > m) m = P->b_send[s].cnt;
        if (P->b_recv[s].cnt > m) m = P->b_recv[s].cnt;
    }
    return m;
}

/* ranges of sendbuf a plan reads and of recvbuf it writes, without repeats */
static void add_range(mvx_range *v, int *n, long off, long cnt)
{
    int i;
    if (cnt <= 0) return;
    for (i = 0; i < *n; i++)
        if (v[i].off == off && v[i].cnt == cnt) return;
    v[*n].off = off;
    v[*n].cnt = cnt;
    (*n)++;
}

static int send_ranges(const mvx_plan *Q, mvx_range *v)
{
    int n = 0, s;
    for (s = 0; s < Q->p; s++) add_range(v, &n, Q->a_send[s].off, Q->a_send[s].cnt);
    if (Q->has_combine) add_range(v, &n, Q->c_src_off, Q->c_cnt);
    return n;
}

static int recv_ranges(const mvx_plan *Q, mvx_range *v)
{
    int n = 0, s;
    if (Q->has_combine && !Q->c_dst_tmp) add_range(v, &n, Q->c_dst_off, Q->c_cnt);
    for (s = 0; s < Q->p; s++) add_range(v, &n, Q->b_recv[s].off, Q->b_recv[s].cnt);
    return n;
}

/* ---- a job: this process's ranks of one collective call ---------------- */
typedef struct {
    int nr;                          /* local ranks: 1 (RCCL) or p (virtual) */
    const mvx_plan *P;               /* nr plans */
    const char *send[MVX_MAXP];      /* the caller's buffers */
    char *recv[MVX_MAXP];
    long nsend[MVX_MAXP], nrecv[MVX_MAXP];   /* elements */
    mvx_xport *t;                    /* nr transports */
    int kinds;                       /* 1: skind / rkind are filled (job_kinds) */
    int skind[MVX_MAXP], rkind[MVX_MAXP];   /* MVX_BUF_* of send / recv (empty: DEVICE) */
} job_t;

/* the buffers' kinds, one pointer query each; returns 1 if any is host memory */
static int job_kinds(job_t *J)
{
    int r, host = 0;
    if (!J->kinds) {
        for (r = 0; r < J->nr; r++) {
            J->skind[r] = J->nsend[r] > 0 ? mvx_buf_kind(J->send[r]) : MVX_BUF_DEVICE;
            J->rkind[r] = J->nrecv[r] > 0 ? mvx_buf_kind(J->recv[r]) : MVX_BUF_DEVICE;
        }
        J->kinds = 1;
    }
    for (r = 0; r < J->nr; r++) host |= J->skind[r] != MVX_BUF_DEVICE || J->rkind[r] != MVX_BUF_DEVICE;
    return host;
}


/* every local rank's staging region for plans Q: X[r].P / c set, per-rank
 * offsets in off[], total bytes returned (pool not touched) */
static size_t region_layout(mvx_comm_t *c, rank_exec_t *X, const job_t *J, const mvx_plan *Q, size_t *off)
{
    size_t need = 0;
    int r;
    for (r = 0; r < J->nr; r++) {
        X[r].P = &Q[r];
        X[r].c = c;
        off[r] = (need + 255) & ~(size_t)255;
        need = off[r] + exec_layout(&X[r]);
    }
    return (need + 255) & ~(size_t)255;
}

static int job_layout(mvx_comm_t *c, rank_exec_t *X, const job_t *J, const mvx_plan *Q)
{
    size_t off[MVX_MAXP];
    const size_t need = region_layout(c, X, J, Q, off);
    int r, rc;
    if ((rc = grow(&c->pool, &c->pool_bytes, need))) return rc;
    for (r = 0; r < J->nr; r++) X[r].pool = c->pool + off[r];
    return MPI_SUCCESS;
}

/* ---- exchange variants (MVX_EXCH_*) -------------------------------------
 * PIPE: the plan runs in slices; slice t's exchange and slice t-2's
 * distribution go in one transfer group while slice t-1 is combined on a
 * second stream, so xGMI and HBM work at once.  Slices keep every block
 * boundary (plan_slice), so the bits are the unsliced plan's. */
static mvx_plan g_pipe[3][MVX_MAXP];

static int pipe_streams(mvx_comm_t *c)
{
    int i;
    if (c->cstream) return MPI_SUCCESS;
    if (hipStreamCreateWithFlags(&c->cstream, hipStreamNonBlocking) != hipSuccess) return MPI_ERR_OTHER;
    for (i = 0; i < 4; i++)
        if (hipEventCreateWithFlags(&c->pev[i], hipEventDisableTiming) != hipSuccess) return MPI_ERR_OTHER;
    return MPI_SUCCESS;
}

static int run_device_plain(mvx_comm_t *c, const job_t *J, hipStream_t st)
{
    rank_exec_t X[MVX_MAXP];
    int r, rc;
    for (r = 0; r < J->nr; r++) {
        X[r].sendbuf = J->send[r];
        X[r].recvbuf = J->recv[r];
    }
    if ((rc = job_layout(c, X, J, J->P))) return rc;
    return exec_group(X, J->t, J->nr, st, c);
}

static int run_device_pipe(mvx_comm_t *c, const job_t *J, hipStream_t st)
{
    static rank_exec_t X0[MVX_MAXP], X[3][MVX_MAXP];
    size_t off[MVX_MAXP], region;
    long span = 0, cs, nsl, t;
    int r, rc, q;
    const int ns = c->exch_slices > 0 ? c->exch_slices : 4;
    for (r = 0; r < J->nr; r++)
        if (plan_span(&J->P[r]) > span) span = plan_span(&J->P[r]);
    cs = (span + ns - 1) / ns;
    cs = (cs + 255) & ~255L;
    nsl = (span + cs - 1) / cs;
    if (nsl <= 1) return run_device_plain(c, J, st);
    if ((rc = pipe_streams(c))) return rc;
    c->ran_exch = MVX_EXCH_PIPE;
    for (r = 0; r < J->nr; r++) {
        plan_slice(&J->P[r], 0, cs, &g_pipe[0][r]);
        X0[r].sendbuf = J->send[r];
        X0[r].recvbuf = J->recv[r];
    }
    region = region_layout(c, X0, J, g_pipe[0], off);   /* slice 0 is the largest */
    if ((rc = grow(&c->pool, &c->pool_bytes, 2 * region))) return rc;
    if ((rc = tev(c, 0, st))) return rc;
    for (t = 0; t < nsl + 2; t++) {
        const int a = t < nsl, dist = t >= 2;
        const int cur = (int)(t % 3), old = (int)((t + 1) % 3);   /* old = (t - 2) % 3 */
        if (a)
            for (r = 0; r < J->nr; r++) {
                X[cur][r] = X0[r];
                plan_slice(&J->P[r], t, cs, &g_pipe[cur][r]);
                X[cur][r].P = &g_pipe[cur][r];
                X[cur][r].pool = c->pool + (t & 1) * region + off[r];
            }
        /* slice t-2's combine is done before its blocks leave and before
         * slice t reuses its staging region */
        if (dist && hipStreamWaitEvent(st, c->pev[2 + (int)(t & 1)], 0) != hipSuccess) return MPI_ERR_OTHER;
        for (r = 0; r < J->nr; r++) {
            mvx_xport *x = &J->t[r];
            if ((rc = x->start(x))) return rc;
            if (a && (rc = exec_phase_a(&X[cur][r], x, st))) return rc;
            if (dist && (rc = exec_phase_c(&X[old][r], x, st))) return rc;
            if ((rc = x->end(x))) return rc;
        }
        if (J->t[0].lb && (rc = lb_flush(J->t[0].lb, st))) return rc;
        if (!a) continue;
        if (hipEventRecord(c->pev[t & 1], st) != hipSuccess ||
            hipStreamWaitEvent(c->cstream, c->pev[t & 1], 0) != hipSuccess)
            return MPI_ERR_OTHER;
        for (q = 0; q < J->nr; q++)
            if ((rc = exec_phase_b(&X[cur][q], c->cstream))) return rc;
        if (hipEventRecord(c->pev[2 + (int)(t & 1)], c->cstream) != hipSuccess) return MPI_ERR_OTHER;
    }
    if ((rc = tev(c, 3, st))) return rc;
    if (c->timing) c->tev_kind = TEV_TOTAL;
    return MPI_SUCCESS;
}

/* COLL: a regular plan -- every rank holds p equal blocks in rank order and
 * combines block `rank` -- exchanges with ncclAllToAll and (Allreduce)
 * distributes with an in-place ncclAllGather instead of grouped send /
 * receive.  Every rank sees the same count and size, so all ranks choose
 * the same variant. */
static int coll_regular(const mvx_plan *P, long *blk)
{
    const long b = P->c_cnt;
    int s;
    if (P->p < 2 || !P->has_combine || b <= 0 || P->c_dst_tmp) return 0;
    if (P->coll != MVX_COLL_ALLREDUCE && P->coll != MVX_COLL_REDUCE_SCATTER) return 0;
    if (P->count != b * P->p || P->c_src_off != b * P->rank) return 0;
    if (P->c_dst_off != (P->coll == MVX_COLL_ALLREDUCE ? b * P->rank : 0)) return 0;
    for (s = 0; s < P->p; s++) {
        if (s == P->rank) continue;
        if (P->a_send[s].off != b * s || P->a_send[s].cnt != b) return 0;
        if (P->a_recv[s].off != b * P->rank || P->a_recv[s].cnt != b) return 0;
        if (P->coll == MVX_COLL_ALLREDUCE) {
            if (P->b_send[s].off != b * P->rank || P->b_send[s].cnt != b) return 0;
            if (P->b_recv[s].off != b * s || P->b_recv[s].cnt != b) return 0;
        } else if (P->b_send[s].cnt || P->b_recv[s].cnt) {
            return 0;
        }
    }
    *blk = b;
    return 1;
}

static int run_device_coll(mvx_comm_t *c, const job_t *J, long b, hipStream_t st)
{
    const mvx_plan *P = &J->P[0];
    mvx_xport *t = &J->t[0];
    const size_t bb = (size_t)(b * P->esize);
    const char *leafp[MVX_MAXP];
    rank_exec_t X;
    scratch_t S;
    size_t stage;
    int s, rc;
    X.P = P; X.c = c; X.sendbuf = J->send[0]; X.recvbuf = J->recv[0];
    stage = al256(bb * (size_t)P->p);
    X.wide_n = wide_temps(P);
    X.wide_slot = al256(bb + SLOT_STAGGER);
    if ((rc = grow(&c->pool, &c->pool_bytes, stage + X.wide_slot * (size_t)X.wide_n))) return rc;
    c->ran_exch = MVX_EXCH_COLL;
    if ((rc = tev(c, 0, st))) return rc;
    if ((rc = t->alltoall(t, J->send[0], c->pool, bb, st))) return rc;
    if ((rc = tev(c, 1, st))) return rc;
    for (s = 0; s < P->p; s++)
        leafp[s] = s == P->rank ? J->send[0] + (size_t)P->rank * bb : c->pool + (size_t)s * bb;
    S.base = c->pool + stage; S.slot = X.wide_slot; S.used = 0; S.cap = X.wide_n;
    if ((rc = combine(c, P, leafp, J->recv[0] + P->c_dst_off * P->esize, &S, st))) return rc;
    if ((rc = tev(c, 2, st))) return rc;
    if (P->coll == MVX_COLL_ALLREDUCE && (rc = t->allgather(t, J->recv[0], bb, st))) return rc;
    if ((rc = tev(c, 3, st))) return rc;
    if (c->timing) c->tev_kind = TEV_PHASES;
    return MPI_SUCCESS;
}

/* all buffers in HBM */
static int run_device(mvx_comm_t *c, const job_t *J, hipStream_t st)
{
    long blk;
    c->ran_exch = MVX_EXCH_P2P;   /* unless a variant below takes the call */
    if (c->exch == MVX_EXCH_PIPE) return run_device_pipe(c, J, st);
    if (c->exch == MVX_EXCH_COLL && J->nr == 1 && J->t[0].alltoall && J->t[0].allgather &&
        J->P[0].opkind == MVX_OPKIND_PREDEFINED && coll_regular(&J->P[0], &blk))
        return run_device_coll(c, J, blk, st);
    return run_device_plain(c, J, st);
}

/* ---- host buffers: a sliced pipeline ------------------------------------
 * Slice i of every local rank's plan is staged in (H2D on stream sh), run
 * (phases A-C on the caller's stream), and staged out (D2H on stream sd);
 * the host drains slice i-1 while the device works on slice i, so host
 * copies, both PCIe directions and the collective overlap.  Page-locked
 * buffers are moved by DMA directly; pageable ones go through pinned bounce
 * slots filled and emptied by the copy pool (mvx_host.c). */
#define STAGE_SLICE_BYTES (16L << 20)
#define STAGE_NB 3

static struct {
    int ready;
    hipStream_t sh, sd;
    char *bin[STAGE_NB], *bout[STAGE_NB];
    size_t bbytes;
    hipEvent_t ein[STAGE_NB], eout[STAGE_NB], ex[STAGE_NB];
} g_stage;

static int stage_init(size_t bounce)
{
    int b;
    if (!g_stage.ready) {
        if (hipStreamCreateWithFlags(&g_stage.sh, hipStreamNonBlocking) != hipSuccess ||
            hipStreamCreateWithFlags(&g_stage.sd, hipStreamNonBlocking) != hipSuccess)
            return MPI_ERR_OTHER;
        for (b = 0; b < STAGE_NB; b++)
            if (hipEventCreateWithFlags(&g_stage.ein[b], hipEventDisableTiming) != hipSuccess ||
                hipEventCreateWithFlags(&g_stage.eout[b], hipEventDisableTiming) != hipSuccess ||
                hipEventCreateWithFlags(&g_stage.ex[b], hipEventDisableTiming) != hipSuccess)
                return MPI_ERR_OTHER;
        g_stage.ready = 1;
    }
    if (bounce > g_stage.bbytes) {
        for (b = 0; b < STAGE_NB; b++) {
            if (g_stage.bin[b]) hipHostFree(g_stage.bin[b]);
            if (g_stage.bout[b]) hipHostFree(g_stage.bout[b]);
            g_stage.bin[b] = g_stage.bout[b] = NULL;
        }
        g_stage.bbytes = 0;
        for (b = 0; b < STAGE_NB; b++)
            if (hipHostMalloc((void **)&g_stage.bin[b], bounce, hipHostMallocDefault) != hipSuccess ||
                hipHostMalloc((void **)&g_stage.bout[b], bounce, hipHostMallocDefault) != hipSuccess)
                return MPI_ERR_OTHER;
        g_stage.bbytes = bounce;
    }
    return MPI_SUCCESS;
}

typedef struct {
    const job_t *J;
    char *dsend[MVX_MAXP], *drecv[MVX_MAXP];   /* device buffers the plans run on */
    int shost[MVX_MAXP], rhost[MVX_MAXP];      /* 1: caller's buffer is host memory */
    int spin[MVX_MAXP], rpin[MVX_MAXP];        /* ... and page-locked */
    long cs;                                   /* slice length, elements */
    int single;                                /* the job is one slice */
} stage_job_t;


/* slice i in: host -> device for every host send buffer.  A job of one
 * slice (S->single) copies on the caller's stream itself: nothing to overlap,
 * and no event round trips on the small-message path. */
static int stage_in(stage_job_t *S, const mvx_plan *Q, long i, hipStream_t st)
{
    const int b = (int)(i % STAGE_NB);
    const hipStream_t hs = S->single ? st : g_stage.sh;
    mvx_range v[MVX_MAXP + 1];
    size_t boff = 0;
    int r, n, j;
    if (!S->single && i >= STAGE_NB && hipEventSynchronize(g_stage.ein[b]) != hipSuccess) return MPI_ERR_OTHER;
    for (r = 0; r < S->J->nr; r++) {
        const long E = Q[r].esize;
        if (!S->shost[r]) continue;
        n = send_ranges(&Q[r], v);
        for (j = 0; j < n; j++) {
            const size_t o = (size_t)(v[j].off * E), bytes = (size_t)(v[j].cnt * E);
            const char *src = S->J->send[r] + o;
            if (!S->spin[r]) {
                mvx_pcopy(g_stage.bin[b] + boff, src, bytes);
                src = g_stage.bin[b] + boff;
                boff += al256(bytes);
            }
            if (hipMemcpyAsync(S->dsend[r] + o, src, bytes, hipMemcpyHostToDevice, hs) != hipSuccess)
                return MPI_ERR_OTHER;
        }
    }
    if (S->single) return MPI_SUCCESS;
    if (hipEventRecord(g_stage.ein[b], g_stage.sh) != hipSuccess ||
        hipStreamWaitEvent(st, g_stage.ein[b], 0) != hipSuccess)
        return MPI_ERR_OTHER;
    return MPI_SUCCESS;
}

/* slice i out, enqueue: device -> host (bounce or page-locked target) */
static int stage_out(stage_job_t *S, const mvx_plan *Q, long i, hipStream_t st)
{
    const int b = (int)(i % STAGE_NB);
    const hipStream_t ds = S->single ? st : g_stage.sd;
    mvx_range v[MVX_MAXP + 1];
    size_t boff = 0;
    int r, n, j;
    if (!S->single && (hipEventRecord(g_stage.ex[b], st) != hipSuccess ||
                       hipStreamWaitEvent(g_stage.sd, g_stage.ex[b], 0) != hipSuccess))
        return MPI_ERR_OTHER;
    for (r = 0; r < S->J->nr; r++) {
        const long E = Q[r].esize;
        if (!S->rhost[r]) continue;
        n = recv_ranges(&Q[r], v);
        for (j = 0; j < n; j++) {
            const size_t o = (size_t)(v[j].off * E), bytes = (size_t)(v[j].cnt * E);
            char *dst = S->rpin[r] ? S->J->recv[r] + o : g_stage.bout[b] + boff;
            if (!S->rpin[r]) boff += al256(bytes);
            if (hipMemcpyAsync(dst, S->drecv[r] + o, bytes, hipMemcpyDeviceToHost, ds) != hipSuccess)
                return MPI_ERR_OTHER;
        }
    }
    if (S->single) return MPI_SUCCESS;
    return hipEventRecord(g_stage.eout[b], g_stage.sd) == hipSuccess ? MPI_SUCCESS : MPI_ERR_OTHER;
}

/* slice i out, finish: wait for its D2H, bounce -> pageable target */
static int stage_drain(stage_job_t *S, const mvx_plan *Q, long i, hipStream_t st)
{
    const int b = (int)(i % STAGE_NB);
    mvx_range v[MVX_MAXP + 1];
    size_t boff = 0;
    int r, n, j;
    if ((S->single ? hipStreamSynchronize(st) : hipEventSynchronize(g_stage.eout[b])) != hipSuccess)
        return MPI_ERR_OTHER;
    for (r = 0; r < S->J->nr; r++) {
        const long E = Q[r].esize;
        if (!S->rhost[r] || S->rpin[r]) continue;
        n = recv_ranges(&Q[r], v);
        for (j = 0; j < n; j++) {
            const size_t o = (size_t)(v[j].off * E), bytes = (size_t)(v[j].cnt * E);
            mvx_pcopy(S->J->recv[r] + o, g_stage.bout[b] + boff, bytes);
            boff += al256(bytes);
        }
    }
    return MPI_SUCCESS;
}

static mvx_plan g_slice[2][MVX_MAXP];   /* slice plans: current and previous */

static int run_staged(mvx_comm_t *c, const job_t *J, hipStream_t st)
{
    stage_job_t S;
    rank_exec_t X[MVX_MAXP];
    size_t need = 0, off[2 * MVX_MAXP], bounce;
    long span = 0, nsl, i;
    int r, rc, pieces = 0;
    mvx_range v[MVX_MAXP + 1];

    memset(&S, 0, sizeof S);
    S.J = J;
    for (r = 0; r < J->nr; r++) {
        const long E = J->P[r].esize;
        int ns = send_ranges(&J->P[r], v), nv = recv_ranges(&J->P[r], v);
        S.shost[r] = J->skind[r] != MVX_BUF_DEVICE;
        S.rhost[r] = J->rkind[r] != MVX_BUF_DEVICE;
        S.spin[r] = J->skind[r] == MVX_BUF_PINNED;
        S.rpin[r] = J->rkind[r] == MVX_BUF_PINNED;
        off[2 * r] = need;
        if (S.shost[r]) need = al256(need + (size_t)(J->nsend[r] * E));
        off[2 * r + 1] = need;
        if (S.rhost[r]) need = al256(need + (size_t)(J->nrecv[r] * E));
        pieces += (ns > nv ? ns : nv);
        if (plan_span(&J->P[r]) > span) span = plan_span(&J->P[r]);
    }
    if ((rc = grow(&c->hpool, &c->hpool_bytes, need + 256))) return rc;
    for (r = 0; r < J->nr; r++) {
        S.dsend[r] = S.shost[r] ? c->hpool + off[2 * r] : (char *)J->send[r];
        S.drecv[r] = S.rhost[r] ? c->hpool + off[2 * r + 1] : J->recv[r];
        X[r].sendbuf = S.dsend[r];
        X[r].recvbuf = S.drecv[r];
    }
    /* slice length.  One rank per process: STAGE_SLICE_BYTES spread over p
     * pieces (a rank's plan reads at most p ranges of its sendbuf -- p - 1
     * blocks out plus its own -- and writes at most p of its recvbuf).  That
     * depends only on p and the type, never on this rank's plan, so every
     * rank of a call slices alike and its transfers pair up.  A virtual
     * communicator (all ranks in this process, sliced together) fills one
     * slot of STAGE_SLICE_BYTES per local rank with all its ranks' pieces:
     * without the nr factor its pieces shrink to ~1 MiB and per-copy
     * overheads dominate.  The bounce slots hold this process's pieces. */
    c->ran_exch = MVX_EXCH_P2P;
    {
        const long E = J->P[0].esize;
        /* slices start at multiples of 256 bytes of every vector (each
         * operand keeps its alignment): cs a multiple of m elements; for a
         * large packed element m is 1 and a slice may hold a single element,
         * where a fixed 256-element floor would size the bounce slots at
         * 256 elements of it */
        long g = E, h = 256, m;
        while (h) { const long t = g % h; g = h; h = t; }      /* gcd(E, 256) */
        m = 256 / g;
        long cs = J->nr > 1 ? STAGE_SLICE_BYTES * J->nr / (E * (pieces > 0 ? pieces : 1))
                            : STAGE_SLICE_BYTES / (E * J->P[0].p);
        cs -= cs % m;
        if (cs < m) cs = m;
        S.cs = cs;
        bounce = (size_t)pieces * al256((size_t)(cs * E));
        if (bounce < 4096) bounce = 4096;
    }
    nsl = span > 0 ? (span + S.cs - 1) / S.cs : 0;
    S.single = nsl <= 1;
    if ((rc = stage_init(bounce))) return rc;
    for (r = 0; r < J->nr; r++) plan_slice(&J->P[r], 0, S.cs, &g_slice[0][r]);
    if ((rc = job_layout(c, X, J, g_slice[0]))) return rc;   /* slice 0 is the largest */
    for (i = 0; i < nsl; i++) {
        mvx_plan *Q = g_slice[i & 1];
        for (r = 0; r < J->nr; r++) {
            plan_slice(&J->P[r], i, S.cs, &Q[r]);
            X[r].P = &Q[r];
        }
        if ((rc = stage_in(&S, Q, i, st))) return rc;
        if ((rc = exec_group(X, J->t, J->nr, st, NULL))) return rc;
        if ((rc = stage_out(&S, Q, i, st))) return rc;
        if (i > 0 && (rc = stage_drain(&S, g_slice[(i - 1) & 1], i - 1, st))) return rc;
    }
    if (nsl > 0 && (rc = stage_drain(&S, g_slice[(nsl - 1) & 1], nsl - 1, st))) return rc;
    return hipStreamSynchronize(st) == hipSuccess ? MPI_SUCCESS : MPI_ERR_OTHER;
}

/* ---- datatypes with holes: the job on packed copies ----------------------
 * Each rank's send vector is packed on the device (from an HBM mirror of
 * its extent-layout region when it is host memory), the plans run on the
 * packed bytes (what the reference's MPI_Sendrecv moves), and the packed
 * result is unpacked into recvbuf: type-map bytes only -- a host recvbuf is
 * mirrored in first so its other bytes come back unchanged. */
typedef struct { long ext, size, lo, hi; } tspan_t;

static int type_span(int dt, tspan_t *T)
{
    if (mvx_type_describe(dt, NULL, NULL, &T->ext, &T->size) ||
        mvx_type_layout(dt, NULL, NULL, NULL, NULL, &T->lo, &T->hi))
        return MPI_ERR_TYPE;
    return MPI_SUCCESS;
}

/* bytes from origin + lo covering the type maps of n elements */
static size_t span_bytes(const tspan_t *T, long n)
{
    return n > 0 ? (size_t)((n - 1) * T->ext + (T->hi - T->lo)) : 0;
}

typedef struct {
    const char *sorg[MVX_MAXP];   /* device origins of the send vectors */
    char *rorg[MVX_MAXP];         /* device origins of the recv vectors */
    char *smir[MVX_MAXP], *rmir[MVX_MAXP], *psend[MVX_MAXP], *precv[MVX_MAXP];
} packed_bufs_t;

static int packed_setup(mvx_comm_t *c, const job_t *J, const tspan_t *T, packed_bufs_t *B, hipStream_t st)
{
    const int dt = J->P[0].dtype;
    size_t need = 0, off[4 * MVX_MAXP];
    int r, rc;
    for (r = 0; r < J->nr; r++) {
        const int sh = J->nsend[r] > 0 && !is_device_ptr(J->send[r]);
        const int rh = J->nrecv[r] > 0 && !is_device_ptr(J->recv[r]);
        off[4 * r] = need;     need = al256(need + (sh ? span_bytes(T, J->nsend[r]) : 0));
        off[4 * r + 1] = need; need = al256(need + (size_t)(J->nsend[r] * T->size));
        off[4 * r + 2] = need; need = al256(need + (rh ? span_bytes(T, J->nrecv[r]) : 0));
        off[4 * r + 3] = need; need = al256(need + (size_t)(J->nrecv[r] * T->size));
        B->smir[r] = sh ? (char *)1 : NULL;
        B->rmir[r] = rh ? (char *)1 : NULL;
    }
    if ((rc = grow(&c->hpool, &c->hpool_bytes, need + 256))) return rc;
    for (r = 0; r < J->nr; r++) {
        B->psend[r] = c->hpool + off[4 * r + 1];
        B->precv[r] = c->hpool + off[4 * r + 3];
        B->sorg[r] = J->send[r];
        B->rorg[r] = J->recv[r];
        if (B->smir[r]) {
            B->smir[r] = c->hpool + off[4 * r];
            if (hipMemcpyAsync(B->smir[r], J->send[r] + T->lo, span_bytes(T, J->nsend[r]), hipMemcpyHostToDevice,
                               st) != hipSuccess)
                return MPI_ERR_OTHER;
            B->sorg[r] = B->smir[r] - T->lo;
        }
        if (B->rmir[r]) {
            B->rmir[r] = c->hpool + off[4 * r + 2];
            if (hipMemcpyAsync(B->rmir[r], J->recv[r] + T->lo, span_bytes(T, J->nrecv[r]), hipMemcpyHostToDevice,
                               st) != hipSuccess)
                return MPI_ERR_OTHER;
            B->rorg[r] = B->rmir[r] - T->lo;
        }
        if (J->nsend[r] > 0 && (rc = mvx_type_pack(dt, B->sorg[r], B->psend[r], (size_t)J->nsend[r], st)))
            return rc;
    }
    return MPI_SUCCESS;
}

static int packed_finish(const job_t *J, const tspan_t *T, packed_bufs_t *B, hipStream_t st, int sync)
{
    const int dt = J->P[0].dtype;
    int r, rc;
    for (r = 0; r < J->nr; r++) {
        if (J->nrecv[r] <= 0) continue;
        if ((rc = mvx_type_unpack(dt, B->precv[r], B->rorg[r], (size_t)J->nrecv[r], st))) return rc;
        if (B->rmir[r] && hipMemcpyAsync(J->recv[r] + T->lo, B->rmir[r], span_bytes(T, J->nrecv[r]),
                                         hipMemcpyDeviceToHost, st) != hipSuccess)
            return MPI_ERR_OTHER;
    }
    return (sync && hipStreamSynchronize(st) != hipSuccess) ? MPI_ERR_OTHER : MPI_SUCCESS;
}

static int run_device(mvx_comm_t *c, const job_t *J, hipStream_t st);

static int run_job_packed(mvx_comm_t *c, const job_t *J, hipStream_t st, int blocking)
{
    static job_t K;
    static packed_bufs_t B;
    tspan_t T;
    int r, rc, host = 0;
    if ((rc = type_span(J->P[0].dtype, &T))) return rc;
    for (r = 0; r < J->nr; r++)
        host |= (J->nsend[r] > 0 && !is_device_ptr(J->send[r])) || (J->nrecv[r] > 0 && !is_device_ptr(J->recv[r]));
    if (host && !blocking) return MPI_ERR_BUFFER;
    if ((rc = packed_setup(c, J, &T, &B, st))) return rc;
    K = *J;
    for (r = 0; r < J->nr; r++) {
        K.send[r] = B.psend[r];
        K.recv[r] = B.precv[r];
    }
    if ((rc = run_device(c, &K, st))) return rc;
    return packed_finish(J, &T, &B, st, blocking || host);
}

/* recvbuf = sendbuf over the type map (MPIR_intra_Scan's self copy when its
 * op is undefined, intra_scan.c:100-106): through the packed form */
static int typed_copy(mvx_comm_t *c, int dt, long n, const char *send, char *recv, hipStream_t st, int sync)
{
    static job_t K;
    static packed_bufs_t B;
    static mvx_plan P0;
    tspan_t T;
    int rc;
    memset(&P0, 0, sizeof P0);
    P0.dtype = dt;
    K.nr = 1; K.P = &P0; K.send[0] = send; K.recv[0] = recv; K.nsend[0] = n; K.nrecv[0] = n;
    if ((rc = type_span(dt, &T)) || (rc = packed_setup(c, &K, &T, &B, st))) return rc;
    if (n > 0 && hipMemcpyAsync(B.precv[0], B.psend[0], (size_t)(n * T.size), hipMemcpyDeviceToDevice, st) != hipSuccess)
        return MPI_ERR_OTHER;
    return packed_finish(&K, &T, &B, st, sync || B.smir[0] || B.rmir[0]);
}

static int run_job(mvx_comm_t *c, job_t *J, hipStream_t st, int blocking)
{
    int rc;
    if (J->P[0].packed) return run_job_packed(c, J, st, blocking);
    if (job_kinds(J)) return blocking ? run_staged(c, J, st) : MPI_ERR_BUFFER;
    rc = run_device(c, J, st);
    if (rc == MPI_SUCCESS && blocking && hipStreamSynchronize(st) != hipSuccess) rc = MPI_ERR_OTHER;
    return rc;
}

/* ---------------------------------------------------------------------- */
/* collective bodies (after the API-level argument checks)                */

typedef struct {
    int coll;
    const char *sendbuf;
    char *recvbuf;
    long count;           /* Allreduce / Reduce */
    const int *recvcnts;  /* Reduce_scatter */
    MPI_Datatype dt;
    MPI_Op op;
    int root;
} call_t;

/* element counts of rank `rank`'s send / recv vectors */
static void call_sizes(const call_t *k, int p, int rank, long *nsend, long *nrecv)
{
    if (k->coll == MVX_COLL_REDUCE_SCATTER) {
        long t = 0;
        int i;
        for (i = 0; i < p; i++) t += k->recvcnts[i];
        *nsend = t;
        *nrecv = k->recvcnts[rank];
    } else {
        *nsend = k->count;
        *nrecv = (k->coll == MVX_COLL_REDUCE && rank != k->root) ? 0 : k->count;
    }
}

/* An undefined (op, type) still runs the reference's transfers, with ops
 * that leave their inout operand as it is -- except under the _SMP_ collops,
 * whose len = 0 test of a predefined op (intra_fns_new.c:5054-5058,
 * 5841-5845) returns on every rank before anything moves. */
static int undefined_moves(const mvx_comm_t *c, int coll)
{
    return !(c->tune.smp && (coll == MVX_COLL_ALLREDUCE || coll == MVX_COLL_REDUCE));
}

/* 1 if rank's plan sends or receives anything */
static int plan_moves(const mvx_plan *P)
{
    int s;
    for (s = 0; s < P->p; s++)
        if (P->a_send[s].cnt || P->a_recv[s].cnt || P->b_send[s].cnt || P->b_recv[s].cnt) return 1;
    return 0;
}

static int run(mvx_comm_t *c, const call_t *k, hipStream_t st, int blocking)
{
    static mvx_plan P;
    job_t J;
    mvx_xport t;
    int rc, verdict, keep = 0, vrc = MPI_SUCCESS;
    long nsend, nrecv;
    int e, ts;

    if (c->local) return MPI_ERR_COMM;   /* virtual comms use *_multi */
    c->ran_exch = -1;
    mvx_dtype_info(k->dt, &e, &ts);
    rc = mvx_plan_build_tuned(&P, k->coll, c->size, c->rank, k->count, k->recvcnts,
                              k->dt, k->op, k->root, op_kind(k->op), &c->tune);
    if (rc) return rc;
    if (P.alg == MVX_ALG_NONE) return MPI_SUCCESS;
    verdict = op_verdict(k->op, k->dt);
    call_sizes(k, c->size, c->rank, &nsend, &nrecv);
    if (verdict == MVX_ERR_OP_NOT_DEFINED && k->coll == MVX_COLL_SCAN) {
        /* MPIR_intra_Scan ignores MPIR_Op_errno: recvbuf keeps the self copy
         * (intra_scan.c:100-106) and the call succeeds */
        if (P.packed) return typed_copy(c, k->dt, nsend, k->sendbuf, k->recvbuf, st, blocking);
        if (hipMemcpyAsync(k->recvbuf, k->sendbuf, (size_t)(nsend * e), hipMemcpyDefault, st) != hipSuccess)
            return MPI_ERR_OTHER;
        return (blocking && hipStreamSynchronize(st) != hipSuccess) ? MPI_ERR_OTHER : MPI_SUCCESS;
    }
    if (verdict == MVX_ERR_OP_NOT_DEFINED) {
        /* 329 on the ranks that call (*uop); the data still moves as the
         * reference's algorithm moves it (undefined_moves) */
        vrc = P.calls_uop ? verdict : MPI_SUCCESS;
        if (!undefined_moves(c, k->coll)) return vrc;
        keep = 1;
    } else if (verdict) {
        return verdict;
    }

    memset(&t, 0, sizeof t);
    if (c->has_ops) {
        t.start = op_start; t.end = op_end; t.send = op_send; t.recv = op_recv;
        if (c->ops.alltoall && c->ops.allgather) { t.alltoall = op_alltoall; t.allgather = op_allgather; }
        t.ops = &c->ops; t.st = st;
    } else {
        t.start = nc_start; t.end = nc_end; t.send = nc_send; t.recv = nc_recv;
        t.alltoall = nc_alltoall; t.allgather = nc_allgather;
        t.nccl = c->nccl;
    }
    t.me = c->rank;
    J.nr = 1;
    J.kinds = 0;
    J.P = &P;
    J.send[0] = k->sendbuf;
    J.recv[0] = k->recvbuf;
    J.nsend[0] = nsend;
    J.nrecv[0] = nrecv;
    J.t = &t;
    c->keep = keep;
    rc = run_job(c, &J, st, blocking);
    c->keep = 0;
    if (!plan_moves(&P)) c->ran_exch = -1;   /* nothing crossed between ranks */
    return rc ? rc : vrc;
}

/* ---------------------------------------------------------------------- */
/* MPI API                                                                */

/* The reference's argument tests (mpi_error.h:403-405, 524-526; non-
 * OLD_ERRMSGS build): each failing test calls MPIR_Err_setmsg (advancing the
 * error ring) and overwrites mpi_errno, so when several fail the last one's
 * code is returned.  MPI_BOTTOM (NULL) buffers never alias. */
static void test_count(long count, int *rc)
{
    if (count < 0) *rc = setmsg_code(MPI_ERR_COUNT, ERR_KIND_DEFAULT);
}

static void test_alias(const void *b1, const void *b2, int *rc)
{
    if (b1 == b2 && b1 != MPI_BOTTOM) *rc = setmsg_code(MPI_ERR_BUFFER, ERR_KIND_ALIAS);
}

int mvx_coll_allreduce(void *sendbuf, void *recvbuf, int count, MPI_Datatype dt,
                       MPI_Op op, MPI_Comm comm)
{
    mvx_comm_t *c = get_comm(comm);
    call_t k;
    int rc = MPI_SUCCESS;
    if (!c) return ERR_COMM_NULL_CODE;                       /* TEST_MPI_COMM */
    if (mvx_dtype_info(dt, NULL, NULL)) return ERR_TYPE_NULL_CODE;  /* TEST_DTYPE */
    test_count(count, &rc);                                 /* allreduce.c:76-77 */
    test_alias(sendbuf, recvbuf, &rc);
    if (rc) return rc;
    if (count == 0) return MPI_SUCCESS;                     /* 5479 */
    if (!predefined(op) && !user_op(op)) return MPI_ERR_OP; /* TEST_MPI_OP */
    k.coll = MVX_COLL_ALLREDUCE; k.sendbuf = sendbuf; k.recvbuf = recvbuf;
    k.count = count; k.recvcnts = NULL; k.dt = dt; k.op = op; k.root = 0;
    return run(c, &k, c->stream, 1);
}

int mvx_coll_reduce(void *sendbuf, void *recvbuf, int count, MPI_Datatype dt,
                    MPI_Op op, int root, MPI_Comm comm)
{
    mvx_comm_t *c = get_comm(comm);
    call_t k;
    int rc = MPI_SUCCESS;
    if (!c) return ERR_COMM_NULL_CODE;
    if (mvx_dtype_info(dt, NULL, NULL)) return ERR_TYPE_NULL_CODE;
    test_alias(sendbuf, recvbuf, &rc);                      /* reduce.c:82-83 */
    test_count(count, &rc);
    if (rc) return rc;
    if (count == 0) return MPI_SUCCESS;                     /* 4541 */
    if (root >= c->size) rc = setmsg_code(MPI_ERR_ROOT, ERR_KIND_ROOT_TOOBIG);
    if (root < 0) rc = setmsg_code(MPI_ERR_ROOT, ERR_KIND_DEFAULT);
    if (rc) return rc;
    if (!predefined(op) && !user_op(op)) return MPI_ERR_OP;
    k.coll = MVX_COLL_REDUCE; k.sendbuf = sendbuf; k.recvbuf = recvbuf;
    k.count = count; k.recvcnts = NULL; k.dt = dt; k.op = op; k.root = root;
    return run(c, &k, c->stream, 1);
}

int mvx_coll_reduce_scatter(void *sendbuf, void *recvbuf, int *recvcnts,
                            MPI_Datatype dt, MPI_Op op, MPI_Comm comm)
{
    mvx_comm_t *c = get_comm(comm);
    call_t k;
    int rc = MPI_SUCCESS;
    if (!c) return ERR_COMM_NULL_CODE;
    if (mvx_dtype_info(dt, NULL, NULL)) return ERR_TYPE_NULL_CODE;
    test_alias(recvbuf, sendbuf, &rc);                      /* red_scat.c:77 */
    if (rc) return rc;
    if (!predefined(op) && !user_op(op)) return MPI_ERR_OP;
    if (!recvcnts) return MPI_ERR_ARG;
    k.coll = MVX_COLL_REDUCE_SCATTER; k.sendbuf = sendbuf; k.recvbuf = recvbuf;
    k.count = 0; k.recvcnts = recvcnts; k.dt = dt; k.op = op; k.root = 0;
    return run(c, &k, c->stream, 1);
}

int mvx_coll_scan(void *sendbuf, void *recvbuf, int count, MPI_Datatype dt,
                  MPI_Op op, MPI_Comm comm)
{
    mvx_comm_t *c = get_comm(comm);
    call_t k;
    int rc = MPI_SUCCESS;
    if (!c) return ERR_COMM_NULL_CODE;                       /* scan.c:74-80 */
    if (mvx_dtype_info(dt, NULL, NULL)) return ERR_TYPE_NULL_CODE;
    test_alias(sendbuf, recvbuf, &rc);
    test_count(count, &rc);
    if (rc) return rc;
    if (count == 0) return MPI_SUCCESS;                     /* scan.c:85 */
    if (!predefined(op) && !user_op(op)) return MPI_ERR_OP;
    k.coll = MVX_COLL_SCAN; k.sendbuf = sendbuf; k.recvbuf = recvbuf;
    k.count = count; k.recvcnts = NULL; k.dt = dt; k.op = op; k.root = 0;
    return run(c, &k, c->stream, 1);
}

int MPI_Scan(void *a, void *b, int n, MPI_Datatype d, MPI_Op o, MPI_Comm c)
{ return mvx_coll_scan(a, b, n, d, o, c); }
int PMPI_Scan(void *a, void *b, int n, MPI_Datatype d, MPI_Op o, MPI_Comm c)
{ return mvx_coll_scan(a, b, n, d, o, c); }
int MPI_Reduce(void *a, void *b, int n, MPI_Datatype d, MPI_Op o, int r, MPI_Comm c)
{ return mvx_coll_reduce(a, b, n, d, o, r, c); }
int MPI_Allreduce(void *a, void *b, int n, MPI_Datatype d, MPI_Op o, MPI_Comm c)
{ return mvx_coll_allreduce(a, b, n, d, o, c); }
int MPI_Reduce_scatter(void *a, void *b, int *n, MPI_Datatype d, MPI_Op o, MPI_Comm c)
{ return mvx_coll_reduce_scatter(a, b, n, d, o, c); }
int PMPI_Reduce(void *a, void *b, int n, MPI_Datatype d, MPI_Op o, int r, MPI_Comm c)
{ return mvx_coll_reduce(a, b, n, d, o, r, c); }
int PMPI_Allreduce(void *a, void *b, int n, MPI_Datatype d, MPI_Op o, MPI_Comm c)
{ return mvx_coll_allreduce(a, b, n, d, o, c); }
int PMPI_Reduce_scatter(void *a, void *b, int *n, MPI_Datatype d, MPI_Op o, MPI_Comm c)
{ return mvx_coll_reduce_scatter(a, b, n, d, o, c); }
int PMPI_Op_create(MPI_User_function *f, int cm, MPI_Op *o) { return MPI_Op_create(f, cm, o); }
int PMPI_Op_free(MPI_Op *o) { return MPI_Op_free(o); }

const mvx_collops MVX_device_collops = { mvx_coll_reduce, mvx_coll_allreduce,
                                         mvx_coll_reduce_scatter, mvx_coll_scan };

int mvx_buffer_is_device(const void *p) { return is_device_ptr(p); }

/* stream-ordered variants: device buffers, no host synchronisation */
static int async_checks(mvx_comm_t *c, MPI_Datatype dt, MPI_Op op)
{
    if (!c) return ERR_COMM_NULL_CODE;
    if (mvx_dtype_info(dt, NULL, NULL)) return ERR_TYPE_NULL_CODE;
    if (!predefined(op) && !user_op(op)) return MPI_ERR_OP;
    return MPI_SUCCESS;
}

int mvx_allreduce_async(const void *sendbuf, void *recvbuf, int count,
                        MPI_Datatype dt, MPI_Op op, MPI_Comm comm, void *stream)
{
    mvx_comm_t *c = get_comm(comm);
    call_t k;
    int rc = async_checks(c, dt, op);
    if (rc) return rc;
    if (count < 0) return MPI_ERR_COUNT;
    if (sendbuf == recvbuf) return MPI_ERR_BUFFER;
    k.coll = MVX_COLL_ALLREDUCE; k.sendbuf = sendbuf; k.recvbuf = recvbuf;
    k.count = count; k.recvcnts = NULL; k.dt = dt; k.op = op; k.root = 0;
    return run(c, &k, (hipStream_t)stream, 0);
}

int mvx_reduce_async(const void *sendbuf, void *recvbuf, int count,
                     MPI_Datatype dt, MPI_Op op, int root, MPI_Comm comm, void *stream)
{
    mvx_comm_t *c = get_comm(comm);
    call_t k;
    int rc = async_checks(c, dt, op);
    if (rc) return rc;
    if (count < 0) return MPI_ERR_COUNT;
    if (root < 0 || root >= c->size) return MPI_ERR_ROOT;
    if (sendbuf == recvbuf) return MPI_ERR_BUFFER;
    k.coll = MVX_COLL_REDUCE; k.sendbuf = sendbuf; k.recvbuf = recvbuf;
    k.count = count; k.recvcnts = NULL; k.dt = dt; k.op = op; k.root = root;
    return run(c, &k, (hipStream_t)stream, 0);
}

int mvx_scan_async(const void *sendbuf, void *recvbuf, int count,
                   MPI_Datatype dt, MPI_Op op, MPI_Comm comm, void *stream)
{
    mvx_comm_t *c = get_comm(comm);
    call_t k;
    int rc = async_checks(c, dt, op);
    if (rc) return rc;
    if (count < 0) return MPI_ERR_COUNT;
    if (sendbuf == recvbuf) return MPI_ERR_BUFFER;
    k.coll = MVX_COLL_SCAN; k.sendbuf = sendbuf; k.recvbuf = recvbuf;
    k.count = count; k.recvcnts = NULL; k.dt = dt; k.op = op; k.root = 0;
    return run(c, &k, (hipStream_t)stream, 0);
}

int mvx_reduce_scatter_async(const void *sendbuf, void *recvbuf, const int *recvcnts,
                             MPI_Datatype dt, MPI_Op op, MPI_Comm comm, void *stream)
{
    mvx_comm_t *c = get_comm(comm);
    call_t k;
    int rc = async_checks(c, dt, op);
    if (rc) return rc;
    if (!recvcnts) return MPI_ERR_ARG;
    if (sendbuf == recvbuf) return MPI_ERR_BUFFER;
    k.coll = MVX_COLL_REDUCE_SCATTER; k.sendbuf = sendbuf; k.recvbuf = recvbuf;
    k.count = 0; k.recvcnts = recvcnts; k.dt = dt; k.op = op; k.root = 0;
    return run(c, &k, (hipStream_t)stream, 0);
}

/* ---------------------------------------------------------------------- */
/* virtual communicators: every rank's plan on one device                 */

/* Virtual communicators: every rank's plan in this process, loopback
 * transport.  Device buffers are stream-ordered; host buffers take the
 * staged pipeline and the call returns when they are written.  The plan,
 * transport and slice tables are static: one call at a time (MPI-1.2 is
 * not thread-safe either, coll.h:61-68). */
static int run_multi(mvx_comm_t *c, int coll, void *const *sendbufs,
                     void *const *recvbufs, long count, const int *recvcnts,
                     MPI_Datatype dt, MPI_Op op, int root, int *rcs,
                     hipStream_t st)
{
    static mvx_plan plans[MVX_MAXP];
    static mvx_xport t[MVX_MAXP];
    static loopback_t lb;
    static job_t J;
    const int p = c->size;
    int r, rc, verdict, e, ts, host = 0;
    call_t k;

    if (mvx_dtype_info(dt, &e, &ts)) return ERR_TYPE_NULL_CODE;
    for (r = 0; r < p; r++) rcs[r] = 0;
    if (!predefined(op) && !user_op(op)) { for (r = 0; r < p; r++) rcs[r] = MPI_ERR_OP; return MPI_SUCCESS; }
    for (r = 0; r < p; r++) {
        rc = mvx_plan_build_tuned(&plans[r], coll, p, r, count, recvcnts, dt, op, root, op_kind(op),
                                  &c->tune);
        if (rc) return rc;
    }
    if (plans[0].alg == MVX_ALG_NONE) return MPI_SUCCESS;
    verdict = op_verdict(op, dt);
    if (verdict) {
        for (r = 0; r < p; r++) {
            rcs[r] = (verdict == MVX_ERR_OP_NOT_DEFINED && !plans[r].calls_uop) ? 0 : verdict;
            if (coll == MVX_COLL_SCAN && verdict == MVX_ERR_OP_NOT_DEFINED && count > 0) {
                if (plans[r].packed) {
                    if ((rc = typed_copy(c, dt, count, sendbufs[r], recvbufs[r], st, 1))) return rc;
                } else if (hipMemcpyAsync(recvbufs[r], sendbufs[r], (size_t)(count * e), hipMemcpyDefault, st) !=
                           hipSuccess) {
                    return MPI_ERR_OTHER;
                }
            }
        }
        if (verdict != MVX_ERR_OP_NOT_DEFINED || coll == MVX_COLL_SCAN || !undefined_moves(c, coll))
            return MPI_SUCCESS;
    }
    k.coll = coll; k.count = count; k.recvcnts = recvcnts; k.root = root;
    J.nr = p;
    J.P = plans;
    J.t = t;
    lb.ns = lb.nr = 0;
    for (r = 0; r < p; r++) {
        call_sizes(&k, p, r, &J.nsend[r], &J.nrecv[r]);
        J.send[r] = (const char *)sendbufs[r];
        J.recv[r] = (char *)recvbufs[r];
        if (J.nsend[r] && J.send[r] == J.recv[r]) return MPI_ERR_BUFFER;
        memset(&t[r], 0, sizeof t[r]);
        t[r].start = lb_nop; t[r].end = lb_nop; t[r].send = lb_send; t[r].recv = lb_recv;
        t[r].lb = &lb; t[r].me = r;
    }
    J.kinds = 0;
    host = job_kinds(&J);
    c->keep = verdict == MVX_ERR_OP_NOT_DEFINED;    /* the transfers of an undefined pair */
    if (plans[0].packed) rc = run_job_packed(c, &J, st, host);
    else rc = host ? run_staged(c, &J, st) : run_device(c, &J, st);
    c->keep = 0;
    return rc;
}

int mvx_allreduce_multi(void *const *sendbufs, void *const *recvbufs, int count,
                        MPI_Datatype dt, MPI_Op op, MPI_Comm comm, int *rc, void *stream)
{
    mvx_comm_t *c = get_comm(comm);
    if (!c || !c->local) return ERR_COMM_NULL_CODE;
    if (count < 0) return MPI_ERR_COUNT;
    return run_multi(c, MVX_COLL_ALLREDUCE, sendbufs, recvbufs, count, NULL, dt, op,
                     0, rc, (hipStream_t)stream);
}

int mvx_reduce_multi(void *const *sendbufs, void *const *recvbufs, int count,
                     MPI_Datatype dt, MPI_Op op, int root, MPI_Comm comm, int *rc,
                     void *stream)
{
    mvx_comm_t *c = get_comm(comm);
    if (!c || !c->local) return ERR_COMM_NULL_CODE;
    if (count < 0) return MPI_ERR_COUNT;
    if (root < 0 || root >= c->size) return MPI_ERR_ROOT;
    return run_multi(c, MVX_COLL_REDUCE, sendbufs, recvbufs, count, NULL, dt, op,
                     root, rc, (hipStream_t)stream);
}

int mvx_scan_multi(void *const *sendbufs, void *const *recvbufs, int count,
                   MPI_Datatype dt, MPI_Op op, MPI_Comm comm, int *rc, void *stream)
{
    mvx_comm_t *c = get_comm(comm);
    if (!c || !c->local) return ERR_COMM_NULL_CODE;
    if (count < 0) return MPI_ERR_COUNT;
    return run_multi(c, MVX_COLL_SCAN, sendbufs, recvbufs, count, NULL, dt, op, 0, rc,
                     (hipStream_t)stream);
}

int mvx_reduce_scatter_multi(void *const *sendbufs, void *const *recvbufs,
                             const int *recvcnts, MPI_Datatype dt, MPI_Op op,
                             MPI_Comm comm, int *rc, void *stream)
{
    mvx_comm_t *c = get_comm(comm);
    if (!c || !c->local) return ERR_COMM_NULL_CODE;
    if (!recvcnts) return MPI_ERR_ARG;
    return run_multi(c, MVX_COLL_REDUCE_SCATTER, sendbufs, recvbufs, 0, recvcnts, dt,
                     op, 0, rc, (hipStream_t)stream);
}

/* ---------------------------------------------------------------------- */
/* the predefined ops as MPI_User_functions                               */

static int g_op_errno = 0;   /* MPIR_Op_errno, global_ops.c:41 */

int mvx_op_errno(void)
{
    int e = g_op_errno;
    g_op_errno = 0;
    return e;
}

/* Host-resident operands (the reference's MPI user buffers): a chunked
 * pipeline over HOP_NB slots.  Chunk c: a pageable operand is copied into a
 * pinned bounce slot by the copy pool (mvx_host.c) and DMA'd from there; a
 * page-locked operand is DMA'd directly.  The kernel runs on stream 0, the
 * D2H of the result on stream 1 (into the bounce, or straight into a
 * page-locked inout), and the host drains chunk c-1 out of the bounce while
 * chunk c is in flight, so host copies, both PCIe directions and the kernel
 * overlap.  Below HOP_BOUNCE_MIN bytes per operand the bounce's per-chunk
 * overheads (pool wake-ups, one more copy) cost more than they hide, and
 * pageable operands are handed to HIP's own pageable copy path instead
 * (tools/bench_host.py: 2 MiB 165 vs 299 us, 256 MiB 14.7 vs 12.8 ms;
 * profiles/r02/bench_host.jsonl).  Device operands are used in place; both
 * operands get an HBM mirror (HBM is plentiful, and no device slot is reused
 * while a copy may still read it). */
#define HOP_NB 3
#define HOP_BOUNCE_MIN (64L << 20)
#define HOP_CHUNK_MIN (1L << 20)
#define HOP_CHUNK_MAX (16L << 20)
#define HOP_PIN_CHUNK_MIN (4L << 20)
#define HOP_PIN_CHUNK_MAX (64L << 20)   /* tools/host_chunk_sweep.sh, profiles/r02/host_chunk_sweep.txt */
static struct {
    hipStream_t s[2];
    hipEvent_t ein[HOP_NB], ek[HOP_NB], eout[HOP_NB];
    char *bin, *bout, *dev;       /* HOP_NB bounce slots: bin 2 chunks, bout 1; dev: both operands */
    size_t bin_bytes, bout_bytes, dev_bytes;
} g_hop;

static int hop_init(size_t slot, size_t dev)
{
    int b;
    if (!g_hop.s[0]) {
        if (hipStreamCreateWithFlags(&g_hop.s[0], hipStreamNonBlocking) != hipSuccess ||
            hipStreamCreateWithFlags(&g_hop.s[1], hipStreamNonBlocking) != hipSuccess)
            return MPI_ERR_OTHER;
        for (b = 0; b < HOP_NB; b++)
            if (hipEventCreateWithFlags(&g_hop.ein[b], hipEventDisableTiming) != hipSuccess ||
                hipEventCreateWithFlags(&g_hop.ek[b], hipEventDisableTiming) != hipSuccess ||
                hipEventCreateWithFlags(&g_hop.eout[b], hipEventDisableTiming) != hipSuccess)
                return MPI_ERR_OTHER;
    }
    if ((slot && (grow_host(&g_hop.bin, &g_hop.bin_bytes, HOP_NB * 2 * slot) ||
                  grow_host(&g_hop.bout, &g_hop.bout_bytes, HOP_NB * slot))) ||
        grow(&g_hop.dev, &g_hop.dev_bytes, dev))
        return MPI_ERR_OTHER;
    return MPI_SUCCESS;
}

static int host_apply(MPI_Op op, MPI_Datatype t, const char *in, char *inout, long len,
                      int in_dev, int io_dev)
{
    int e, ts, rc, bounce_in, bounce_io;
    long chunk, c, nch;
    size_t bytes, cb, slot;
    hipStream_t sd;
    mvx_dtype_info(t, &e, &ts);
    bytes = (size_t)len * e;
    bounce_in = !in_dev && bytes >= (size_t)HOP_BOUNCE_MIN && !mvx_host_pinned(in);
    bounce_io = !io_dev && bytes >= (size_t)HOP_BOUNCE_MIN && !mvx_host_pinned(inout);
    /* chunk: whole 256-element groups (the device operands keep the kernel's
     * 16-byte vector path) */
    if (bounce_in || bounce_io) {       /* pool copies pace the pipeline: ~8 chunks */
        cb = bytes / 8;
        if (cb < (size_t)HOP_CHUNK_MIN) cb = HOP_CHUNK_MIN;
        if (cb > (size_t)HOP_CHUNK_MAX) cb = HOP_CHUNK_MAX;
    } else if ((!in_dev && !mvx_host_pinned(in)) || (!io_dev && !mvx_host_pinned(inout))) {
        cb = 32L << 20;                 /* HIP stages pageable copies itself: whole 32 MiB pieces */
    } else {                            /* DMA only: fewer, larger copies */
        cb = bytes / 4;
        if (cb < (size_t)HOP_PIN_CHUNK_MIN) cb = HOP_PIN_CHUNK_MIN;
        if (cb > (size_t)HOP_PIN_CHUNK_MAX) cb = HOP_PIN_CHUNK_MAX;
    }
    {
        static long fixed = -1;       /* MVX_HOST_CHUNK_MIB: a fixed chunk (tuning) */
        if (fixed < 0) {
            const char *v = getenv("MVX_HOST_CHUNK_MIB");
            fixed = v ? atol(v) : 0;
        }
        if (fixed > 0) cb = (size_t)fixed << 20;
    }
    chunk = (long)(cb / ((size_t)e * 256)) * 256;
    if (chunk < 256) chunk = 256;
    if (chunk > len) chunk = len;
    slot = (bounce_in || bounce_io) ? al256((size_t)chunk * e) : 0;
    if ((rc = hop_init(slot, 2 * al256(bytes)))) return rc;
    nch = (len + chunk - 1) / chunk;
    sd = nch > 1 ? g_hop.s[1] : g_hop.s[0];    /* one chunk: everything in order on one stream */
    for (c = 0; c <= nch; c++) {
        if (c < nch) {
            const int b = (int)(c % HOP_NB);
            const long n = len - c * chunk < chunk ? len - c * chunk : chunk;
            const size_t o = (size_t)(c * chunk) * e, sz = (size_t)n * e;
            char *bi = slot ? g_hop.bin + (size_t)b * 2 * slot : NULL;
            char *din = in_dev ? (char *)in + o : g_hop.dev + o;
            char *dio = io_dev ? inout + o : g_hop.dev + al256(bytes) + o;
            /* bounce slot b was last read by the H2D of chunk c - HOP_NB */
            if (slot && c >= HOP_NB && hipEventSynchronize(g_hop.ein[b]) != hipSuccess) return MPI_ERR_OTHER;
            if (bounce_in) mvx_pcopy(bi, in + o, sz);
            if (bounce_io) mvx_pcopy(bi + slot, inout + o, sz);
            if (!in_dev && hipMemcpyAsync(din, bounce_in ? bi : in + o, sz, hipMemcpyHostToDevice,
                                          g_hop.s[0]) != hipSuccess)
                return MPI_ERR_OTHER;
            if (!io_dev && hipMemcpyAsync(dio, bounce_io ? bi + slot : inout + o, sz, hipMemcpyHostToDevice,
                                          g_hop.s[0]) != hipSuccess)
                return MPI_ERR_OTHER;
            if (slot && hipEventRecord(g_hop.ein[b], g_hop.s[0]) != hipSuccess) return MPI_ERR_OTHER;
            if ((rc = mvx_op_apply(op, t, din, dio, (size_t)n, g_hop.s[0]))) return rc;
            if (!io_dev) {
                if (sd != g_hop.s[0] &&
                    (hipEventRecord(g_hop.ek[b], g_hop.s[0]) != hipSuccess ||
                     hipStreamWaitEvent(sd, g_hop.ek[b], 0) != hipSuccess))
                    return MPI_ERR_OTHER;
                if (hipMemcpyAsync(bounce_io ? g_hop.bout + (size_t)b * slot : inout + o, dio, sz,
                                   hipMemcpyDeviceToHost, sd) != hipSuccess ||
                    (bounce_io && hipEventRecord(g_hop.eout[b], sd) != hipSuccess))
                    return MPI_ERR_OTHER;
            }
        }
        if (c > 0 && bounce_io) {   /* drain chunk c - 1 */
            const long p = c - 1;
            const int b = (int)(p % HOP_NB);
            const long n = len - p * chunk < chunk ? len - p * chunk : chunk;
            if (hipEventSynchronize(g_hop.eout[b]) != hipSuccess) return MPI_ERR_OTHER;
            mvx_pcopy(inout + (size_t)(p * chunk) * e, g_hop.bout + (size_t)b * slot, (size_t)n * e);
        }
    }
    if (hipStreamSynchronize(g_hop.s[0]) != hipSuccess || hipStreamSynchronize(sd) != hipSuccess)
        return MPI_ERR_OTHER;
    return MPI_SUCCESS;
}

static void uop_call(MPI_Op op, void *in, void *inout, int *len, MPI_Datatype *t)
{
    int rc;
    if (!len || !t) { g_op_errno = MPI_ERR_ARG; return; }
    rc = mvx_op_apply(op, *t, NULL, NULL, 0, NULL);   /* verdict first */
    if (rc == MPI_SUCCESS && *len > 0) {
        const int in_dev = is_device_ptr(in), io_dev = is_device_ptr(inout);
        if (in_dev && io_dev) {
            rc = mvx_op_apply(op, *t, in, inout, (size_t)*len, NULL);
            if (rc == MPI_SUCCESS && hipStreamSynchronize(NULL) != hipSuccess) rc = MPI_ERR_OTHER;
        } else if (!in || !inout) {
            rc = MPI_ERR_BUFFER;
        } else {
            rc = host_apply(op, *t, (const char *)in, (char *)inout, *len, in_dev, io_dev);
        }
    }
    if (rc) g_op_errno = rc;
}

#define UOP(NAME, OPH) \
    void NAME(void *in, void *io, int *len, MPI_Datatype *t) { uop_call(OPH, in, io, len, t); }
UOP(MPIR_MAXF, MPI_MAX)
UOP(MPIR_MINF, MPI_MIN)
UOP(MPIR_SUM, MPI_SUM)
UOP(MPIR_PROD, MPI_PROD)
UOP(MPIR_LAND, MPI_LAND)
UOP(MPIR_BAND, MPI_BAND)
UOP(MPIR_LOR, MPI_LOR)
UOP(MPIR_BOR, MPI_BOR)
UOP(MPIR_LXOR, MPI_LXOR)
UOP(MPIR_BXOR, MPI_BXOR)
UOP(MPIR_MAXLOC, MPI_MAXLOC)
UOP(MPIR_MINLOC, MPI_MINLOC)
