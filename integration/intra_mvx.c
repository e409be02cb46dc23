/*
 * intra_mvx.c -- MVAPICH's reduction collectives on the MI355X path.
 *
 * A file a maintainer adds to the reference tree as src/coll/intra_mvx.c and
 * builds with the device's own headers (-Iinclude -Impid/<device>
 * -I<this repo>/include), linking -lmvx_embed (libmvx_embed.so exports only
 * mvx_* names, so nothing collides with MVAPICH's MPI_* / MPIR_* symbols).
 * MPIR_Comm_collops_init (src/context/comm_util.c:321-331) then installs
 * MPIR_mvx_collops for intra-communicators.
 *
 * The table is MPIR_intra_collops (include/mpicoll.h:59) with Reduce,
 * Allreduce, Reduce_scatter and Scan replaced.  Each replacement sends a call
 * in which some rank's buffers are device memory (or every call, with
 * MVX_HOST_BUFFERS=1) to libmvx on every rank, which computes the
 * reference's bits in the reference's combine order; a call with host
 * buffers on every rank runs MVAPICH's own function unchanged (Route below).
 *
 * What it reads of the reference's objects (nothing is added to them):
 *   struct MPIR_COMMUNICATOR  np, local_rank, self        mpid/ch2/comm.h:65-113
 *                             _SMP_: shmem_coll_ok, leader_comm
 *                                                         mpid/ch_gen2/comm.h:162-181
 *   struct MPIR_DATATYPE      dte_type, permanent, self, count, blocklen,
 *                             stride, indices, blocklens, old_type, old_types,
 *                             extent, size, lb, ub        mpid/ch2/datatype.h:26-56
 *   struct MPIR_OP            op, commute, permanent      include/mpiops.h:4-9
 *   MPIR_ToPointer, MPIR_GET_OP_PTR, MPIR_COMM_WORLD      include/mpiimpl.h:171-194
 *   MPIR_F_TRUE, MPIR_F_FALSE (Fortran-enabled builds)    src/fortran/src/initfutil.c:100-102
 * and keeps its per-communicator state in an attribute (MPI_Keyval_create
 * with a delete callback, src/context/keyvalcreate.c:57), so MPI_Comm_free
 * releases the libmvx communicator.
 *
 * Route (one per call, the same on every rank).  MPI lets ranks pass
 * buffers of different kinds to one call, and every algorithm assumes all
 * ranks run the same function (comm_util.c:321-331 installs one table per
 * communicator; intra_fns_new.c:5453), so the choice between libmvx and
 * MVAPICH's own function is agreed, never taken rank-locally:
 *   MVX_SHIM_ROUTE=agree (default)  one MPIR_intra_collops->Allreduce of three
 *                 ints (MPI_MAX of {this rank touches device memory, this
 *                 rank touches host memory, this rank's translation error})
 *                 on the host path: if any rank touches device memory (or
 *                 sets MVX_HOST_BUFFERS=1) every rank calls libmvx -- a
 *                 host-buffer rank through libmvx's host staging -- otherwise
 *                 every rank runs MVAPICH's function.  "Touches" counts only
 *                 the buffers the call uses on that rank: sendbuf when it
 *                 holds elements, recvbuf unless the rank is a non-root of
 *                 Reduce (or receives no element of a Reduce_scatter).  Skipped
 *                 at np == 1 and for an empty call (count 0 on every rank, as
 *                 MPI requires).
 *   MVX_SHIM_ROUTE=local   no agreement: the caller promises every rank's
 *                 buffers agree in kind in every call (the route is this
 *                 rank's own buffer test).
 *   MVX_SHIM_ROUTE must be the same on every rank, like any MVAPICH knob.
 *   The agreement also tells libmvx when no rank touches host memory
 *   (mvx_comm_set_call_kinds): large calls then keep the unsliced device
 *   schedule instead of the slices that pair with host-buffer ranks.  One
 *   rank's device sendbuf beside its host recvbuf counts as host.
 *   The datatype and op are translated before the agreement (below), so a
 *   rank that cannot translate makes every rank return its error.
 *
 * Translation, per call, cached:
 *   communicator  the first call routed to libmvx creates the twin, on every
 *                 rank together (the route is agreed): each rank checks its
 *                 device (mvx_device_check), rank 0 makes the RCCL id; an
 *                 MPI_MIN Allreduce agrees that all of it worked before any
 *                 rank enters RCCL's collective creation (a rank that cannot
 *                 would leave its peers in ncclCommInitRank for good); the id
 *                 is broadcast with MVAPICH's own Bcast; mvx_comm_init(
 *                 local_rank, np, device); a second MIN agrees creation
 *                 succeeded everywhere (ranks that got one abort it
 *                 otherwise).  A failure is recorded on every rank alike:
 *                 every later call routed to libmvx returns MPI_ERR_OTHER on
 *                 every rank.  device = $MVX_DEVICE_ID, else the
 *                 MPI_COMM_WORLD rank modulo the visible GPUs.
 *   datatype      (local, before the route agreement; cached)
 *                 a permanent type's handle is libmvx's handle (the values
 *                 of include/mpi.h:64-140); a derived type is rebuilt from
 *                 the node tree the reference's constructors stored
 *                 (type_contig.c:118-169, type_hvec.c:98-160,
 *                 type_hind.c:106-174, type_struct.c:160-330: MPI_Type_vector
 *                 and _indexed are already hvector / hindexed there) with
 *                 libmvx's mvx_type_* constructors, which restate the same
 *                 bounds rules; the rebuilt extent / size / lb / ub must equal
 *                 the reference's or the call fails with MPI_ERR_TYPE.  User
 *                 functions are given the caller's handle
 *                 (mvx_type_set_handle).
 *   op            (local, before the route agreement)
 *                 predefined ops pass unchanged; a user op
 *                 (!permanent) is registered once with mvx_op_create.
 *   flavour       _SMP_ builds pass the live knobs (enable_shmem_collectives,
 *                 the VIADEV_* thresholds, comm->shmem_coll_ok) so libmvx
 *                 plans intra_shmem_Reduce / _Allreduce's leader fold
 *                 (intra_fns_new.c:4992-5198, 5793-5940).  libmvx models one
 *                 node: a communicator spanning nodes (leader_comm size > 1)
 *                 is planned without the shmem step.

 */
#include <stdlib.h>
#include <string.h>

#include "mpiimpl.h"
#include "mpiops.h"
#include "mpicoll.h"
#include "mvx_embed.h"
#include "mvx_hip.h"

#ifdef _SMP_
extern int enable_shmem_collectives;     /* src/env/initutil.c:146 */
#endif
#ifndef MPID_NO_FORTRAN
extern MPI_Fint MPIR_F_TRUE, MPIR_F_FALSE;   /* src/fortran/src/initfutil.c:100-102 */
#endif

MPIR_COLLOPS MPIR_mvx_collops;           /* installed by MPIR_Comm_collops_init */

/* ---- per-communicator state (an attribute) ------------------------------ */

typedef struct {
    int mvx;     /* libmvx communicator handle, or -1: creation failed */
} mvx_shim_comm;

static int g_keyval = MPI_KEYVAL_INVALID;

static int shim_delete(MPI_Comm comm, int keyval, void *attr, void *extra)
{
    mvx_shim_comm *s = (mvx_shim_comm *)attr;
    (void)comm; (void)keyval; (void)extra;
    if (s) {
        if (s->mvx >= 0) mvx_comm_free(&s->mvx);
        free(s);
    }
    return MPI_SUCCESS;
}

static int shim_device(void)
{
    const char *e = getenv("MVX_DEVICE_ID");
    int n;
    if (e && *e) return atoi(e);
    n = mvx_device_count();
    return n > 0 ? MPIR_COMM_WORLD->local_rank % n : 0;
}

static void shim_tuning(int h, struct MPIR_COMMUNICATOR *comm)
{
    mvx_tuning t;
#ifdef _SMP_
    struct MPIR_COMMUNICATOR *leaders;
    if (mvx_tuning_from_env(&t, 1)) return;     /* the reference exits at init */
    t.enable_shmem_collectives = enable_shmem_collectives;
    leaders = comm->shmem_coll_ok == 1 ? MPIR_GET_COMM_PTR(comm->leader_comm) : NULL;
    t.shmem_coll_ok = comm->shmem_coll_ok == 1 && (!leaders || leaders->np == 1);
#else
    (void)comm;
    if (mvx_tuning_from_env(&t, 0)) return;     /* ch_shmem: intra_Reduce / intra_Allreduce */
#endif
    mvx_comm_set_tuning(h, &t);
}

/* MPI_MIN of `v` over the communicator (MVAPICH's own Allreduce); 0 if it
 * fails, so a broken agreement reads as "not everywhere" */
static int agree_min(int v, struct MPIR_COMMUNICATOR *comm)
{
    int all = 0;
    if (MPIR_intra_collops->Allreduce(&v, &all, 1, MPIR_GET_DTYPE_PTR(MPI_INT), MPI_MIN, comm) !=
        MPI_SUCCESS)
        return 0;
    return all;
}

/* create the twin on every rank together; s->mvx = handle, or -1 on every
 * rank when any rank could not take part */
static void twin_create(mvx_shim_comm *s, struct MPIR_COMMUNICATOR *comm)
{
    char id[MVX_UNIQUE_ID_BYTES];
    const int dev = shim_device();
    int ok;

    s->mvx = -1;
    memset(id, 0, sizeof id);
    /* this rank can enter RCCL's creation: a usable device, and rank 0 an id */
    ok = mvx_device_check(dev) == 0;
    if (ok && comm->local_rank == 0) ok = mvx_get_unique_id(id) == 0;
    if (!agree_min(ok, comm)) return;
    if (MPIR_intra_collops->Bcast(id, MVX_UNIQUE_ID_BYTES, MPIR_GET_DTYPE_PTR(MPI_BYTE), 0, comm) !=
        MPI_SUCCESS)
        ok = 0;
    if (ok && mvx_comm_init(&s->mvx, comm->local_rank, comm->np, dev, id) != 0) {
        s->mvx = -1;
        ok = 0;
    }
    if (!agree_min(ok, comm)) {
        if (s->mvx >= 0) mvx_comm_abort(&s->mvx);
        s->mvx = -1;
        return;
    }
    shim_tuning(s->mvx, comm);
#ifndef MPID_NO_FORTRAN
    /* MPI_LOGICAL's words, as mpir_init_flog set them (initfutil.c:189) */
    mvx_set_fortran_logical(MPIR_F_TRUE, MPIR_F_FALSE);
#endif
}

/* the libmvx twin of `comm`, created on first use by every rank together
 * (callers reach here only on an agreed route); -1 if creation failed */
static int shim_comm(struct MPIR_COMMUNICATOR *comm)
{
    mvx_shim_comm *s = NULL;
    int flag = 0;

    if (g_keyval == MPI_KEYVAL_INVALID &&
        MPI_Keyval_create(MPI_NULL_COPY_FN, shim_delete, &g_keyval, NULL) != MPI_SUCCESS)
        return -1;
    MPI_Attr_get(comm->self, g_keyval, &s, &flag);
    if (flag && s) return s->mvx;

    s = (mvx_shim_comm *)malloc(sizeof *s);
    if (!s) return -1;
    twin_create(s, comm);
    MPI_Attr_put(comm->self, g_keyval, s);
    return s->mvx;
}

/* ---- datatypes ---------------------------------------------------------- */

#define TYPE_CACHE 32
typedef struct {
    unsigned long long sig;   /* structural hash of the node tree */
    int self;                 /* the reference's handle */
    int type;                 /* libmvx handle (committed), 0 = empty slot */
    int ntemp, *temp;         /* every libmvx type built for it (freed together) */
    unsigned long long used;
} type_entry;
static type_entry g_types[TYPE_CACHE];
static unsigned long long g_clock;

static unsigned long long mix(unsigned long long h, unsigned long long v)
{
    h ^= v + 0x9e3779b97f4a7c15ull + (h << 6) + (h >> 2);
    return h * 0xff51afd7ed558ccdull;
}

static unsigned long long type_sig(struct MPIR_DATATYPE *d)
{
    unsigned long long h = mix(0, (unsigned long long)d->dte_type);
    int i;
    if (d->permanent) return mix(h, (unsigned long long)d->self);
    h = mix(h, (unsigned long long)d->count);
    h = mix(h, (unsigned long long)d->extent);
    h = mix(h, (unsigned long long)d->size);
    h = mix(h, (unsigned long long)d->lb);
    h = mix(h, (unsigned long long)d->ub);
    switch (d->dte_type) {
    case MPIR_CONTIG:
        return mix(h, type_sig(d->old_type));
    case MPIR_HVECTOR:
        h = mix(h, (unsigned long long)d->blocklen);
        h = mix(h, (unsigned long long)d->stride);
        return mix(h, type_sig(d->old_type));
    case MPIR_HINDEXED:
        for (i = 0; i < d->count; i++) {
            h = mix(h, (unsigned long long)d->blocklens[i]);
            h = mix(h, (unsigned long long)d->indices[i]);
        }
        return mix(h, type_sig(d->old_type));
    case MPIR_STRUCT:
        for (i = 0; i < d->count; i++) {
            h = mix(h, (unsigned long long)d->blocklens[i]);
            h = mix(h, (unsigned long long)d->indices[i]);
            h = mix(h, type_sig(d->old_types[i]));
        }
        return h;
    default:
        return h;
    }
}

static void entry_clear(type_entry *e)
{
    int i;
    if (e->type > 0) mvx_type_set_handle(e->type, e->type);
    for (i = e->ntemp - 1; i >= 0; i--) mvx_type_free(&e->temp[i]);
    free(e->temp);
    memset(e, 0, sizeof *e);
}

static int entry_push(type_entry *e, int t)
{
    int *n = (int *)realloc(e->temp, (size_t)(e->ntemp + 1) * sizeof(int));
    if (!n) return MPI_ERR_EXHAUSTED;
    e->temp = n;
    e->temp[e->ntemp++] = t;
    return MPI_SUCCESS;
}

/* rebuild the node tree rooted at d as a libmvx type (type_*.c fields) */
static int build(struct MPIR_DATATYPE *d, type_entry *e, int *out)
{
    int rc, old = 0, i, *types = NULL;
    long *idx = NULL;

    if (d->permanent) { *out = d->self; return MPI_SUCCESS; }
    switch (d->dte_type) {
    case MPIR_CONTIG:
        if ((rc = build(d->old_type, e, &old))) return rc;
        rc = mvx_type_contiguous(d->count, old, out);
        break;
    case MPIR_HVECTOR:
        if ((rc = build(d->old_type, e, &old))) return rc;
        rc = mvx_type_hvector(d->count, d->blocklen, (long)d->stride, old, out);
        break;
    case MPIR_HINDEXED:
        if ((rc = build(d->old_type, e, &old))) return rc;
        idx = (long *)malloc((size_t)(d->count > 0 ? d->count : 1) * sizeof(long));
        if (!idx) return MPI_ERR_EXHAUSTED;
        for (i = 0; i < d->count; i++) idx[i] = (long)d->indices[i];
        rc = mvx_type_hindexed(d->count, d->blocklens, idx, old, out);
        break;
    case MPIR_STRUCT:
        idx = (long *)malloc((size_t)(d->count > 0 ? d->count : 1) * sizeof(long));
        types = (int *)malloc((size_t)(d->count > 0 ? d->count : 1) * sizeof(int));
        if (!idx || !types) { free(idx); free(types); return MPI_ERR_EXHAUSTED; }
        for (i = 0, rc = 0; i < d->count && !rc; i++) {
            idx[i] = (long)d->indices[i];
            rc = build(d->old_types[i], e, &types[i]);
        }
        if (!rc) rc = mvx_type_struct(d->count, d->blocklens, idx, types, out);
        break;
    default:   /* MPIR_VECTOR / MPIR_INDEXED are never stored (datatype.h:12-14) */
        return MPI_ERR_TYPE;
    }
    free(idx);
    free(types);
    if (rc) return MPI_ERR_TYPE;
    return entry_push(e, *out);
}

/* libmvx handle for the reference datatype d (0 on success) */
int mvx_shim_type(struct MPIR_DATATYPE *d, int *out)
{
    unsigned long long sig;
    type_entry *e, *victim = &g_types[0];
    int i, t = 0, kind, dense;
    long lb, ub, extent, size;

    if (d->permanent) { *out = d->self; return MPI_SUCCESS; }
    sig = type_sig(d);
    for (i = 0; i < TYPE_CACHE; i++) {
        e = &g_types[i];
        if (e->type && e->sig == sig && e->self == d->self) {
            e->used = ++g_clock;
            *out = e->type;
            return MPI_SUCCESS;
        }
        if (!e->type || (victim->type && e->used < victim->used)) victim = e;
    }
    e = victim;
    entry_clear(e);
    if (build(d, e, &t) || mvx_type_commit(t) ||
        mvx_type_layout(t, &kind, &dense, &lb, &ub, NULL, NULL) ||
        mvx_type_describe(t, NULL, NULL, &extent, &size) ||
        extent != (long)d->extent || size != (long)d->size || lb != (long)d->lb ||
        ub != (long)d->ub || mvx_type_set_handle(t, d->self)) {
        entry_clear(e);
        return MPI_ERR_TYPE;
    }
    e->sig = sig;
    e->self = d->self;
    e->type = t;
    e->used = ++g_clock;
    *out = t;
    return MPI_SUCCESS;
}

/* ---- ops ---------------------------------------------------------------- */

#define OP_CACHE 16
static struct {
    MPI_Op op;
    MPI_User_function *fn;
    int commute, mvx;
    unsigned long long used;
} g_ops[OP_CACHE];

int mvx_shim_op(MPI_Op op, int *out)
{
    struct MPIR_OP *o;
    int i, v = 0;
    if (op >= MPI_MAX && op <= MPI_MAXLOC) { *out = (int)op; return MPI_SUCCESS; }
    o = MPIR_GET_OP_PTR(op);
    if (!o) return MPI_ERR_OP;
    if (o->permanent) { *out = (int)op; return MPI_SUCCESS; }
    for (i = 0; i < OP_CACHE; i++) {
        if (g_ops[i].mvx && g_ops[i].op == op && g_ops[i].fn == o->op &&
            g_ops[i].commute == o->commute) {
            g_ops[i].used = ++g_clock;
            *out = g_ops[i].mvx;
            return MPI_SUCCESS;
        }
        if (!g_ops[i].mvx || (g_ops[v].mvx && g_ops[i].used < g_ops[v].used)) v = i;
    }
    if (g_ops[v].mvx) mvx_op_free(&g_ops[v].mvx);
    if (mvx_op_create((mvx_user_function *)o->op, o->commute, &g_ops[v].mvx)) {
        g_ops[v].mvx = 0;
        return MPI_ERR_OP;
    }
    g_ops[v].op = op;
    g_ops[v].fn = o->op;
    g_ops[v].commute = o->commute;
    g_ops[v].used = ++g_clock;
    *out = g_ops[v].mvx;
    return MPI_SUCCESS;
}

/* ---- the collops members ------------------------------------------------ */

static int route_local(void)
{
    const char *e = getenv("MVX_SHIM_ROUTE");
    return e && !strcmp(e, "local");
}

/* What one call does with this rank's buffers: the buffers it touches here
 * (libmvx's own rule, mvx_api.c call_sizes: sendbuf when it holds elements;
 * recvbuf when this rank receives -- never at a non-root of Reduce, whose
 * recvbuf MPI leaves unspecified) and whether any of them is host memory. */
typedef struct {
    const void *sendbuf, *recvbuf;
    int send_used, recv_used;
    int empty;          /* no element on any rank (the same on every rank) */
} shim_call;

static int touches_device(const shim_call *k)
{
    return (k->send_used && mvx_buffer_is_device(k->sendbuf)) ||
           (k->recv_used && mvx_buffer_is_device(k->recvbuf));
}

static int touches_host(const shim_call *k)
{
    return (k->send_used && !mvx_buffer_is_device(k->sendbuf)) ||
           (k->recv_used && !mvx_buffer_is_device(k->recvbuf));
}

/* this rank's wish: 1 for libmvx (a device buffer, or MVX_HOST_BUFFERS=1) */
static int wants_mvx(const shim_call *k)
{
    const char *e = getenv("MVX_HOST_BUFFERS");
    if (e && atoi(e) == 1) return 1;
    return touches_device(k);
}

/* The route of one call, the same on every rank: 1 libmvx (*t, *o: the
 * datatype and op in libmvx's handles), 0 MVAPICH's own function, -1 with
 * *rc set: every rank returns *rc.  An empty call needs no agreement.
 *
 * A call that may go to libmvx is translated first -- locally, cached -- so
 * that the one agreement also carries whether every rank could: a rank whose
 * derived type does not rebuild to the reference's bounds, or whose user op
 * cannot be registered, makes every rank return its error instead of leaving
 * its peers inside RCCL.  The agreement is one MPI_MAX Allreduce of three
 * ints: {this rank wants libmvx, this rank touches host memory, this rank's
 * translation error}.  *kinds: MVX_KINDS_DEVICE when no rank touches host
 * memory (libmvx then keeps the unsliced device schedule for large calls),
 * else MVX_KINDS_UNKNOWN (the schedule that pairs with every kind). */
static int route(const shim_call *k, struct MPIR_DATATYPE *dt, MPI_Op op, struct MPIR_COMMUNICATOR *comm,
                 int *t, int *o, int *rc, int *kinds)
{
    int v[3], all[3], trc;
    const int mine = wants_mvx(k), local = comm->np == 1 || route_local();
    *kinds = MVX_KINDS_UNKNOWN;
    *rc = MPI_SUCCESS;
    if (k->empty || (local && !mine)) return 0;
    trc = mvx_shim_type(dt, t);
    if (trc == MPI_SUCCESS) trc = mvx_shim_op(op, o);
    if (local) {
        *rc = trc;
        return trc ? -1 : 1;
    }
    v[0] = mine;
    v[1] = touches_host(k);
    v[2] = trc;
    *rc = MPIR_intra_collops->Allreduce(v, all, 3, MPIR_GET_DTYPE_PTR(MPI_INT), MPI_MAX, comm);
    if (*rc != MPI_SUCCESS) return -1;
    if (!all[0]) return 0;
    if (all[2]) {           /* some rank cannot translate: every rank fails alike */
        *rc = all[2];
        return -1;
    }
    *kinds = all[1] ? MVX_KINDS_UNKNOWN : MVX_KINDS_DEVICE;
    return 1;
}

/* the communicator's twin (collective at first use: every rank is here, the
 * route being agreed) with the agreed kinds handed over for the call about
 * to be made on it; -1 if the twin could not be created */
static int twin_for_call(struct MPIR_COMMUNICATOR *comm, int kinds)
{
    const int h = shim_comm(comm);
    if (h >= 0 && kinds != MVX_KINDS_UNKNOWN) mvx_comm_set_call_kinds(h, kinds);
    return h;
}

static int mvx_Reduce(void *sendbuf, void *recvbuf, int count, struct MPIR_DATATYPE *dt, MPI_Op op,
                      int root, struct MPIR_COMMUNICATOR *comm)
{
    const shim_call k = {sendbuf, recvbuf, count > 0, count > 0 && comm->local_rank == root, count == 0};
    int h, t, o, rc, kinds;
    const int r = route(&k, dt, op, comm, &t, &o, &rc, &kinds);
    if (r < 0) return rc;
    if (!r) return MPIR_intra_collops->Reduce(sendbuf, recvbuf, count, dt, op, root, comm);
    if ((h = twin_for_call(comm, kinds)) < 0) return MPI_ERR_OTHER;
    return mvx_coll_reduce(sendbuf, recvbuf, count, t, o, root, h);
}

static int mvx_Allreduce(void *sendbuf, void *recvbuf, int count, struct MPIR_DATATYPE *dt,
                         MPI_Op op, struct MPIR_COMMUNICATOR *comm)
{
    const shim_call k = {sendbuf, recvbuf, count > 0, count > 0, count == 0};
    int h, t, o, rc, kinds;
    const int r = route(&k, dt, op, comm, &t, &o, &rc, &kinds);
    if (r < 0) return rc;
    if (!r) return MPIR_intra_collops->Allreduce(sendbuf, recvbuf, count, dt, op, comm);
    if ((h = twin_for_call(comm, kinds)) < 0) return MPI_ERR_OTHER;
    return mvx_coll_allreduce(sendbuf, recvbuf, count, t, o, h);
}

static int mvx_Reduce_scatter(void *sendbuf, void *recvbuf, int *recvcnts,
                              struct MPIR_DATATYPE *dt, MPI_Op op, struct MPIR_COMMUNICATOR *comm)
{
    shim_call k = {sendbuf, recvbuf, 0, 0, 1};
    int h, t, o, r, rc, i, kinds;
    for (i = 0; i < comm->np && recvcnts; i++) k.send_used |= recvcnts[i] > 0;  /* same counts everywhere */
    k.empty = !k.send_used;
    k.recv_used = recvcnts && recvcnts[comm->local_rank] > 0;
    r = route(&k, dt, op, comm, &t, &o, &rc, &kinds);
    if (r < 0) return rc;
    if (!r) return MPIR_intra_collops->Reduce_scatter(sendbuf, recvbuf, recvcnts, dt, op, comm);
    if ((h = twin_for_call(comm, kinds)) < 0) return MPI_ERR_OTHER;
    return mvx_coll_reduce_scatter(sendbuf, recvbuf, recvcnts, t, o, h);
}

static int mvx_Scan(void *sendbuf, void *recvbuf, int count, struct MPIR_DATATYPE *dt, MPI_Op op,
                    struct MPIR_COMMUNICATOR *comm)
{
    const shim_call k = {sendbuf, recvbuf, count > 0, count > 0, count == 0};
    int h, t, o, rc, kinds;
    const int r = route(&k, dt, op, comm, &t, &o, &rc, &kinds);
    if (r < 0) return rc;
    if (!r) return MPIR_intra_collops->Scan(sendbuf, recvbuf, count, dt, op, comm);
    if ((h = twin_for_call(comm, kinds)) < 0) return MPI_ERR_OTHER;
    return mvx_coll_scan(sendbuf, recvbuf, count, t, o, h);
}

/* Called once (MPIR_Init, after MPIR_intra_collops exists): the table is a
 * copy of MPIR_intra_collops with the four reductions replaced; its
 * ref_count starts at 1 so MPI_Comm_free never frees it (comm_free.c:143-149). */
void MPIR_mvx_collops_init(void)
{
    static struct _MPIR_COLLOPS table;
    table = *MPIR_intra_collops;
    table.Reduce = mvx_Reduce;
    table.Allreduce = mvx_Allreduce;
    table.Reduce_scatter = mvx_Reduce_scatter;
    table.Scan = mvx_Scan;
    table.ref_count = 1;
    MPIR_mvx_collops = &table;
}
