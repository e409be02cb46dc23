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
    mvx_tuning tune;     /* device flavour + knobs (mvx_coll.h) */
    int shmem_block;     /* claimed shmem collective block, -1 = none */
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

static mvx_comm_t *new_comm(MPI_Comm *out)
{
    int i;
    for (i = 0; i < MAX_COMMS; i++) {
        if (!g_comms[i].used) {
            memset(&g_comms[i], 0, sizeof g_comms[i]);
            g_comms[i].used = 1;
            g_comms[i].handle = g_have_world ? COMM_HANDLE_BASE + i : MPI_COMM_WORLD;
            g_have_world = 1;
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

/* a new communicator's flavour: MVX_DEVICE names the reference device */
static int comm_flavour(mvx_comm_t *c)
{
    const char *d = getenv("MVX_DEVICE");
    const int smp = d && (!strcmp(d, "ch_gen2") || !strcmp(d, "ch_smp") || !strcmp(d, "ch_gen2_ud"));
    int rc = mvx_tuning_from_env(&c->tune, smp);
    c->shmem_block = -1;
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
    return MPI_SUCCESS;
}

int mvx_comm_free(MPI_Comm *comm)
{
    mvx_comm_t *c = comm ? get_comm(*comm) : NULL;
    if (!c) return ERR_COMM_NULL_CODE;
    if (c->nccl) ncclCommDestroy(c->nccl);
    if (c->pool) hipFree(c->pool);
    if (c->hpool) hipFree(c->hpool);
    if (c->upool) hipFree(c->upool);
    if (c->uhost) hipHostFree(c->uhost);
    release_shmem_block(c);
    if (c->handle == MPI_COMM_WORLD) g_have_world = 0;
    memset(c, 0, sizeof *c);
    *comm = 0;
    return MPI_SUCCESS;
}

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

int mvx_op_create_device(MVX_Device_function *function, int commute, MPI_Op *op)
{
    if (!function) return MPI_ERR_ARG;
    return op_register(NULL, function, commute, op);
}

/* ---- derived datatypes (the table is libmvx_hip.so's) ------------------ */

int MPI_Type_contiguous(int count, MPI_Datatype old, MPI_Datatype *newtype)
{
    return mvx_type_contiguous(count, old, newtype);
}

int MPI_Type_commit(MPI_Datatype *datatype)   /* type_commit.c:41-143 */
{
    if (!datatype || mvx_type_describe(*datatype, NULL, NULL, NULL, NULL)) return MVX_ERR_TYPE_NULL;
    return MPI_SUCCESS;   /* contiguous types need no flattening */
}

int MPI_Type_free(MPI_Datatype *datatype) { return mvx_type_free(datatype); }

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

/* the plan kind of an op handle (an invalid handle plans as predefined and
 * is rejected by op_verdict) */
static int op_kind(MPI_Op op)
{
    const mvx_op_t *o = predefined(op) ? NULL : user_op(op);
    if (!o) return MVX_OPKIND_PREDEFINED;
    return o->commute ? MVX_OPKIND_USER_COMMUTE : MVX_OPKIND_USER_NONCOMMUTE;
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

#define NCCL_OK(x) do { if ((x) != ncclSuccess) return MPI_ERR_OTHER; } while (0)

/* ---- user ops: the combine program as a sequence of user calls --------
 * The reference hands a user function (*uop)(in, inout, &len, &type) its
 * operands in the roles the plan's program records, a swapped step being
 * uop(in = left, inout = right) whose result becomes the left value.  The
 * program runs over k scratch copies of the leaves (a user function writes
 * its inout operand, and leaves include the caller's send buffer); a swap
 * just renames which scratch buffer holds the left value. */
static int call_host(const mvx_op_t *o, const char *in, char *inout, long n, int esize,
                     MPI_Datatype dt)
{
    while (n > 0) {   /* the reference's len is an int */
        int len = n > 0x40000000L ? 0x40000000 : (int)n;
        MPI_Datatype t = dt;
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
    if (o->dop) return o->dop(in, inout, (size_t)n, dt, st) ? MPI_ERR_OTHER : MPI_SUCCESS;
    return call_host(o, in, inout, n, esize, dt);
}

static int combine_user(mvx_comm_t *c, const mvx_plan *P, const void *const *srcs,
                        const void *const *fold, void *dst, hipStream_t st)
{
    const mvx_op_t *o = user_op(P->op);
    const long n = P->c_cnt, E = P->esize;
    const size_t bytes = (size_t)(n * E), slot = (bytes + 255) & ~(size_t)255;
    const int dev = o && o->dop;
    const hipMemcpyKind in_kind = dev ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
    char *y[MVX_COMBINE_KMAX], *base;
    int q, l, rc;
    if (!o) return MPI_ERR_OP;
    if (dev) rc = grow(&c->upool, &c->upool_bytes, slot * (size_t)P->k * 2);
    else rc = grow_host(&c->uhost, &c->uhost_bytes, slot * (size_t)P->k * 2);
    if (rc) return rc;
    base = dev ? c->upool : c->uhost;
    for (q = 0; q < P->k; q++) {
        y[q] = base + slot * (size_t)q;
        if (hipMemcpyAsync(y[q], srcs[q], bytes, in_kind, st) != hipSuccess) return MPI_ERR_OTHER;
        if (fold[q] && hipMemcpyAsync(base + slot * (size_t)(P->k + q), fold[q], bytes, in_kind, st) != hipSuccess)
            return MPI_ERR_OTHER;
    }
    if (!dev && hipStreamSynchronize(st) != hipSuccess) return MPI_ERR_OTHER;
    for (q = 0; q < P->k; q++)   /* leaf q = op(leaf, fold): fold is `in` */
        if (fold[q] && (rc = user_step(o, base + slot * (size_t)(P->k + q), y[q], n, (int)E, P->dtype, st)))
            return rc;
    for (l = 0; l < 3; l++)
        for (q = 0; q + (1 << l) < P->k; q++) {
            const unsigned bit = 1u << (l * 8 + q);
            char *a = y[q], *b = y[q + (1 << l)];
            if (!(P->tree_mask & bit)) continue;
            if (P->tree_swap & bit) { rc = user_step(o, a, b, n, (int)E, P->dtype, st); y[q] = b; y[q + (1 << l)] = a; }
            else rc = user_step(o, b, a, n, (int)E, P->dtype, st);
            if (rc) return rc;
        }
    for (q = 1; q < P->k; q++) {
        const unsigned bit = 1u << q;
        char *a = y[0], *b = y[q];
        if (!(P->chain_mask & bit)) continue;
        if (P->chain_swap & bit) { rc = user_step(o, a, b, n, (int)E, P->dtype, st); y[0] = b; y[q] = a; }
        else rc = user_step(o, b, a, n, (int)E, P->dtype, st);
        if (rc) return rc;
    }
    if (hipMemcpyAsync(dst, y[0], bytes, dev ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, st) != hipSuccess)
        return MPI_ERR_OTHER;
    /* the pinned scratch is reused by the next call */
    return (!dev && hipStreamSynchronize(st) != hipSuccess) ? MPI_ERR_OTHER : MPI_SUCCESS;
}

static int combine(mvx_comm_t *c, const mvx_plan *P, const char *const *leafp, void *dst,
                   hipStream_t st)
{
    const void *srcs[MVX_COMBINE_KMAX], *fold[MVX_COMBINE_KMAX];
    int q;
    if (P->k > MVX_COMBINE_KMAX) return MPI_ERR_INTERN;  /* p > 8 per node */
    for (q = 0; q < P->k; q++) {
        srcs[q] = leafp[P->leaf[q]];
        fold[q] = P->leaf_fold[q] >= 0 ? leafp[P->leaf_fold[q]] : NULL;
    }
    if (P->opkind != MVX_OPKIND_PREDEFINED) return combine_user(c, P, srcs, fold, dst, st);
    return mvx_op_program(P->op, P->dtype, srcs, fold, P->k, P->tree_mask,
                          P->chain_mask, dst, (size_t)P->c_cnt, st);
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
    ncclComm_t nccl;
    loopback_t *lb;
    int me;
} mvx_xport;

static int nc_start(mvx_xport *t) { (void)t; return ncclGroupStart() == ncclSuccess ? 0 : MPI_ERR_OTHER; }
static int nc_end(mvx_xport *t) { (void)t; return ncclGroupEnd() == ncclSuccess ? 0 : MPI_ERR_OTHER; }
static int nc_send(mvx_xport *t, const void *b, size_t n, int peer, hipStream_t st)
{ return ncclSend(b, n, ncclUint8, peer, t->nccl, st) == ncclSuccess ? 0 : MPI_ERR_OTHER; }
static int nc_recv(mvx_xport *t, void *b, size_t n, int peer, hipStream_t st)
{ return ncclRecv(b, n, ncclUint8, peer, t->nccl, st) == ncclSuccess ? 0 : MPI_ERR_OTHER; }

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
    const mvx_plan *P;
    mvx_comm_t *c;
    const char *sendbuf;
    char *recvbuf;
    char *pool;                     /* this rank's staging region */
    size_t slot[MVX_MAXP], tmp_off;
} rank_exec_t;

/* staging layout: one slot per received shard, plus the temporary result
 * of a non-root Reduce; returns the bytes this rank needs.  Consecutive
 * slots are 4 KiB apart beyond their size: back-to-back equal-size shards put
 * the same chunk of every leaf at the same DRAM interleave position, and the
 * k-leaf combine then ran 5-6 % slower (tools/tune_combine_layout.py,
 * profiles/r01/tune_combine_layout.jsonl: 53.9 vs 51.2 us for 8 x 32 MiB). */
#define SLOT_STAGGER 4096
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
    int s;
    if (!P->has_combine || P->c_cnt == 0) return MPI_SUCCESS;
    for (s = 0; s < P->p; s++)
        leafp[s] = (s == P->rank) ? X->sendbuf + P->c_src_off * E : X->pool + X->slot[s];
    return combine(X->c, P, leafp, exec_out(X), st);
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

/* run one rank's plan over RCCL */
static int exec_plan(mvx_comm_t *c, const mvx_plan *P, const char *sendbuf,
                     char *recvbuf, hipStream_t st)
{
    rank_exec_t X;
    mvx_xport t;
    int rc;
    memset(&t, 0, sizeof t);
    t.start = nc_start; t.end = nc_end; t.send = nc_send; t.recv = nc_recv;
    t.nccl = c->nccl; t.me = c->rank;
    X.P = P; X.c = c; X.sendbuf = sendbuf; X.recvbuf = recvbuf;
    if ((rc = grow(&c->pool, &c->pool_bytes, exec_layout(&X)))) return rc;
    X.pool = c->pool;
    if ((rc = exec_phase_a(&X, &t, st))) return rc;
    if ((rc = exec_phase_b(&X, st))) return rc;
    return exec_phase_c(&X, &t, st);
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

/* element counts of this rank's send / recv vectors */
static void call_sizes(const call_t *k, mvx_comm_t *c, long *nsend, long *nrecv)
{
    if (k->coll == MVX_COLL_REDUCE_SCATTER) {
        long t = 0;
        int i;
        for (i = 0; i < c->size; i++) t += k->recvcnts[i];
        *nsend = t;
        *nrecv = k->recvcnts[c->rank];
    } else {
        *nsend = k->count;
        *nrecv = (k->coll == MVX_COLL_REDUCE && c->rank != k->root) ? 0 : k->count;
    }
}

static int run(mvx_comm_t *c, const call_t *k, hipStream_t st, int blocking)
{
    mvx_plan P;
    int rc, verdict, sdev, rdev;
    long nsend, nrecv;
    int e, ts;

    if (c->local) return MPI_ERR_COMM;   /* virtual comms use *_multi */
    mvx_dtype_info(k->dt, &e, &ts);
    rc = mvx_plan_build_tuned(&P, k->coll, c->size, c->rank, k->count, k->recvcnts,
                              k->dt, k->op, k->root, op_kind(k->op), &c->tune);
    if (rc) return rc;
    if (P.alg == MVX_ALG_NONE) return MPI_SUCCESS;
    verdict = op_verdict(k->op, k->dt);
    call_sizes(k, c, &nsend, &nrecv);
    if (verdict == MVX_ERR_OP_NOT_DEFINED && k->coll == MVX_COLL_SCAN) {
        /* MPIR_intra_Scan ignores MPIR_Op_errno: recvbuf keeps the self copy
         * (intra_scan.c:100-106) and the call succeeds */
        if (hipMemcpyAsync(k->recvbuf, k->sendbuf, (size_t)(nsend * e), hipMemcpyDefault, st) != hipSuccess)
            return MPI_ERR_OTHER;
        return (blocking && hipStreamSynchronize(st) != hipSuccess) ? MPI_ERR_OTHER : MPI_SUCCESS;
    }
    if (verdict == MVX_ERR_OP_NOT_DEFINED) return P.calls_uop ? verdict : MPI_SUCCESS;
    if (verdict) return verdict;

    sdev = nsend == 0 || is_device_ptr(k->sendbuf);
    rdev = nrecv == 0 || is_device_ptr(k->recvbuf);
    if (sdev && rdev) {
        rc = exec_plan(c, &P, k->sendbuf, k->recvbuf, st);
        if (rc == MPI_SUCCESS && blocking && hipStreamSynchronize(st) != hipSuccess)
            rc = MPI_ERR_OTHER;
        return rc;
    }
    if (!blocking) return MPI_ERR_BUFFER;
    {   /* host buffers: stage through HBM (H2D, device collective, D2H) */
        const size_t sb = (size_t)(nsend * e), rb = (size_t)(nrecv * e);
        const size_t roff = (sb + 255) & ~(size_t)255;
        char *ds, *dr;
        if ((rc = grow(&c->hpool, &c->hpool_bytes, roff + rb + 256))) return rc;
        ds = sdev ? (char *)k->sendbuf : c->hpool;
        dr = rdev ? k->recvbuf : c->hpool + roff;
        if (!sdev && sb && hipMemcpyAsync(ds, k->sendbuf, sb, hipMemcpyHostToDevice, st) != hipSuccess)
            return MPI_ERR_OTHER;
        rc = exec_plan(c, &P, ds, dr, st);
        if (rc) return rc;
        if (!rdev && rb && hipMemcpyAsync(k->recvbuf, dr, rb, hipMemcpyDeviceToHost, st) != hipSuccess)
            return MPI_ERR_OTHER;
        return hipStreamSynchronize(st) == hipSuccess ? MPI_SUCCESS : MPI_ERR_OTHER;
    }
}

/* ---------------------------------------------------------------------- */
/* MPI API                                                                */

int mvx_coll_allreduce(void *sendbuf, void *recvbuf, int count, MPI_Datatype dt,
                       MPI_Op op, MPI_Comm comm)
{
    mvx_comm_t *c = get_comm(comm);
    call_t k;
    if (!c) return ERR_COMM_NULL_CODE;                       /* TEST_MPI_COMM */
    if (mvx_dtype_info(dt, NULL, NULL)) return ERR_TYPE_NULL_CODE;  /* TEST_DTYPE */
    if (count < 0) return setmsg_code(MPI_ERR_COUNT, ERR_KIND_DEFAULT);
    if (sendbuf == recvbuf) return setmsg_code(MPI_ERR_BUFFER, ERR_KIND_ALIAS);
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
    int rc = 0;
    if (!c) return ERR_COMM_NULL_CODE;
    if (mvx_dtype_info(dt, NULL, NULL)) return ERR_TYPE_NULL_CODE;
    if (sendbuf == recvbuf) return setmsg_code(MPI_ERR_BUFFER, ERR_KIND_ALIAS);
    if (count < 0) return setmsg_code(MPI_ERR_COUNT, ERR_KIND_DEFAULT);
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
    if (!c) return ERR_COMM_NULL_CODE;
    if (mvx_dtype_info(dt, NULL, NULL)) return ERR_TYPE_NULL_CODE;
    if (recvbuf == sendbuf) return setmsg_code(MPI_ERR_BUFFER, ERR_KIND_ALIAS);
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
    if (!c) return ERR_COMM_NULL_CODE;                       /* scan.c:74-80 */
    if (mvx_dtype_info(dt, NULL, NULL)) return ERR_TYPE_NULL_CODE;
    if (sendbuf == recvbuf) return setmsg_code(MPI_ERR_BUFFER, ERR_KIND_ALIAS);
    if (count < 0) return setmsg_code(MPI_ERR_COUNT, ERR_KIND_DEFAULT);
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

static int run_multi(mvx_comm_t *c, int coll, void *const *sendbufs,
                     void *const *recvbufs, long count, const int *recvcnts,
                     MPI_Datatype dt, MPI_Op op, int root, int *rcs,
                     hipStream_t st)
{
    static mvx_plan plans[MVX_MAXP];
    static rank_exec_t X[MVX_MAXP];
    static mvx_xport t[MVX_MAXP];
    static loopback_t lb;
    const int p = c->size;
    int r, rc, verdict, e, ts;
    size_t need = 0, base[MVX_MAXP];

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
            if (coll == MVX_COLL_SCAN && verdict == MVX_ERR_OP_NOT_DEFINED &&
                hipMemcpyAsync(recvbufs[r], sendbufs[r], (size_t)(count * e), hipMemcpyDefault, st) != hipSuccess)
                return MPI_ERR_OTHER;
        }
        return MPI_SUCCESS;
    }
    for (r = 0; r < p; r++) {
        long nsend = plans[r].count, nrecv;
        nrecv = coll == MVX_COLL_REDUCE_SCATTER ? recvcnts[r]
              : (coll == MVX_COLL_REDUCE && r != root) ? 0 : count;
        if ((nsend && !is_device_ptr(sendbufs[r])) || (nrecv && !is_device_ptr(recvbufs[r])))
            return MPI_ERR_BUFFER;
        if (sendbufs[r] == recvbufs[r]) return MPI_ERR_BUFFER;
        X[r].P = &plans[r];
        X[r].c = c;
        X[r].sendbuf = (const char *)sendbufs[r];
        X[r].recvbuf = (char *)recvbufs[r];
        base[r] = (need + 255) & ~(size_t)255;
        need = base[r] + exec_layout(&X[r]);
    }
    if ((rc = grow(&c->pool, &c->pool_bytes, need))) return rc;
    for (r = 0; r < p; r++) {
        X[r].pool = c->pool + base[r];
        t[r].start = lb_nop; t[r].end = lb_nop; t[r].send = lb_send; t[r].recv = lb_recv;
        t[r].lb = &lb; t[r].me = r;
    }
    /* the RCCL path's phase code, every rank in turn, loopback transfers */
    lb.ns = lb.nr = 0;
    for (r = 0; r < p; r++)
        if ((rc = exec_phase_a(&X[r], &t[r], st))) return rc;
    if ((rc = lb_flush(&lb, st))) return rc;
    for (r = 0; r < p; r++)
        if ((rc = exec_phase_b(&X[r], st))) return rc;
    for (r = 0; r < p; r++)
        if ((rc = exec_phase_c(&X[r], &t[r], st))) return rc;
    return lb_flush(&lb, st);
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

/* Host-resident operands (the reference's MPI user buffers): chunked
 * pipeline -- H2D of chunk c and its kernel on one stream, D2H of chunk c on
 * a second stream, so the two PCIe directions and the kernel overlap.
 * Device operands are used in place. */
#define HOST_CHUNK_BYTES (32L << 20)
static char *g_hop_pool;
static size_t g_hop_bytes;
static hipStream_t g_hop_s[2];
static hipEvent_t g_hop_ev;

static int host_apply(MPI_Op op, MPI_Datatype t, const char *in, char *inout, long len,
                      int in_dev, int io_dev)
{
    int e, ts, rc;
    long chunk, off;
    size_t bytes;
    char *din, *dio;
    mvx_dtype_info(t, &e, &ts);
    bytes = (size_t)len * e;
    if (!g_hop_s[0]) {
        if (hipStreamCreateWithFlags(&g_hop_s[0], hipStreamNonBlocking) != hipSuccess ||
            hipStreamCreateWithFlags(&g_hop_s[1], hipStreamNonBlocking) != hipSuccess ||
            hipEventCreateWithFlags(&g_hop_ev, hipEventDisableTiming) != hipSuccess)
            return MPI_ERR_OTHER;
    }
    if ((rc = grow(&g_hop_pool, &g_hop_bytes, 2 * ((bytes + 255) & ~(size_t)255)))) return rc;
    din = in_dev ? (char *)in : g_hop_pool;
    dio = io_dev ? inout : g_hop_pool + ((bytes + 255) & ~(size_t)255);
    chunk = HOST_CHUNK_BYTES / e;
    for (off = 0; off < len; off += chunk) {
        const long n = len - off < chunk ? len - off : chunk;
        const size_t o = (size_t)off * e, b = (size_t)n * e;
        if (!in_dev && hipMemcpyAsync(din + o, in + o, b, hipMemcpyHostToDevice, g_hop_s[0]) != hipSuccess)
            return MPI_ERR_OTHER;
        if (!io_dev && hipMemcpyAsync(dio + o, inout + o, b, hipMemcpyHostToDevice, g_hop_s[0]) != hipSuccess)
            return MPI_ERR_OTHER;
        if ((rc = mvx_op_apply(op, t, din + o, dio + o, (size_t)n, g_hop_s[0]))) return rc;
        if (!io_dev) {
            if (hipEventRecord(g_hop_ev, g_hop_s[0]) != hipSuccess ||
                hipStreamWaitEvent(g_hop_s[1], g_hop_ev, 0) != hipSuccess ||
                hipMemcpyAsync(inout + o, dio + o, b, hipMemcpyDeviceToHost, g_hop_s[1]) != hipSuccess)
                return MPI_ERR_OTHER;
        }
    }
    if (hipStreamSynchronize(g_hop_s[0]) != hipSuccess || hipStreamSynchronize(g_hop_s[1]) != hipSuccess)
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
