/*
 * mvx_api.c -- the MPI entry points of libmvx.so (include/mvx_coll.h):
 *   MPI_Allreduce (allreduce.c:57-92) -> collops->Allreduce -> intra_Allreduce
 *   MPI_Reduce    (reduce.c:62-96)    -> collops->Reduce    -> intra_Reduce
 *   MPI_Reduce_scatter (red_scat.c:60-90) -> intra_Reduce_scatter
 *   MPI_Scan      (scan.c:55-95)      -> MPIR_intra_Scan
 * Argument checks keep the reference's order and codes; one call becomes
 * this rank's plan (mvx_plan.c) run as a job (mvx_exec.c / mvx_stage.c).
 */
#include <string.h>

#include "mvx_internal.h"

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
    int kinds;            /* every rank's buffer kinds, if agreed (MVX_KINDS_*) */
} call_t;

/* the hint mvx_comm_set_call_kinds left for this call; consumed by every
 * call, an early-returning one included */
static int take_kinds(mvx_comm_t *c)
{
    int k;
    if (!c) return MVX_KINDS_UNKNOWN;
    k = c->call_kinds;
    c->call_kinds = MVX_KINDS_UNKNOWN;
    return k;
}

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

static int run_on(mvx_comm_t *c, const call_t *k, hipStream_t st, int blocking);

/* every call runs on its communicator's device; the caller's stays current */
static int run(mvx_comm_t *c, const call_t *k, hipStream_t st, int blocking)
{
    const int prev = mvxi_dev_enter(c->device);
    int rc;
    if (prev == MVXI_DEV_FAILED) return MPI_ERR_OTHER;
    c->call_kinds = blocking ? k->kinds : MVX_KINDS_UNKNOWN;
    rc = run_on(c, k, st, blocking);
    c->call_kinds = MVX_KINDS_UNKNOWN;
    mvxi_dev_leave(c->device, prev);
    return rc;
}

static int run_on(mvx_comm_t *c, const call_t *k, hipStream_t st, int blocking)
{
    mvx_work *w = mvxi_work(c);
    mvx_plan *Pp;
    job_t J;
    mvx_xport t;
    int rc, verdict, keep = 0, vrc = MPI_SUCCESS;
    long nsend, nrecv;
    int e, ts;

    if (c->local) return MPI_ERR_COMM;   /* virtual comms use *_multi */
    if (!w) return MPI_ERR_INTERN;
    Pp = &w->call_plan;
    c->ran_exch = -1;
    c->last_st = st;
    mvx_dtype_info(k->dt, &e, &ts);
    rc = mvx_plan_build_tuned(Pp, k->coll, c->size, c->rank, k->count, k->recvcnts,
                              k->dt, k->op, k->root, mvxi_op_kind(k->op), &c->tune);
    if (rc) return rc;
    if (Pp->alg == MVX_ALG_NONE) return MPI_SUCCESS;
    verdict = mvxi_op_verdict(k->op, k->dt);
    call_sizes(k, c->size, c->rank, &nsend, &nrecv);
    if (verdict == MVX_ERR_OP_NOT_DEFINED && k->coll == MVX_COLL_SCAN) {
        /* MPIR_intra_Scan ignores MPIR_Op_errno: recvbuf keeps the self copy
         * (intra_scan.c:100-106) and the call succeeds */
        if (Pp->packed) return mvxi_typed_copy(c, k->dt, nsend, k->sendbuf, k->recvbuf, st, blocking);
        return mvxi_copy_any(c, k->recvbuf, k->sendbuf, (size_t)(nsend * e), st, blocking);
    }
    if (verdict == MVX_ERR_OP_NOT_DEFINED) {
        /* 329 on the ranks that call (*uop); the data still moves as the
         * reference's algorithm moves it (undefined_moves) */
        vrc = Pp->calls_uop ? verdict : MPI_SUCCESS;
        if (!undefined_moves(c, k->coll)) return vrc;
        keep = 1;
    } else if (verdict) {
        return verdict;
    }

    mvxi_xport_comm(&t, c, st);
    J.nr = 1;
    J.kinds = 0;
    J.P = Pp;
    J.send[0] = k->sendbuf;
    J.recv[0] = k->recvbuf;
    J.nsend[0] = nsend;
    J.nrecv[0] = nrecv;
    J.t = &t;
    c->keep = keep;
    rc = mvxi_run_job(c, &J, st, blocking);
    mvxi_job_release(&J, rc);
    c->keep = 0;
    if (!plan_moves(Pp)) c->ran_exch = -1;   /* nothing crossed between ranks */
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
    if (count < 0) *rc = mvxi_setmsg_code(MPI_ERR_COUNT, ERR_KIND_DEFAULT);
}

static void test_alias(const void *b1, const void *b2, int *rc)
{
    if (b1 == b2 && b1 != MPI_BOTTOM) *rc = mvxi_setmsg_code(MPI_ERR_BUFFER, ERR_KIND_ALIAS);
}

int mvx_coll_allreduce(void *sendbuf, void *recvbuf, int count, MPI_Datatype dt,
                       MPI_Op op, MPI_Comm comm)
{
    mvx_comm_t *c = mvxi_get_comm(comm);
    call_t k;
    k.kinds = take_kinds(c);
    int rc = MPI_SUCCESS;
    if (!c) return ERR_COMM_NULL_CODE;                       /* TEST_MPI_COMM */
    if (mvx_dtype_info(dt, NULL, NULL)) return ERR_TYPE_NULL_CODE;  /* TEST_DTYPE */
    test_count(count, &rc);                                 /* allreduce.c:76-77 */
    test_alias(sendbuf, recvbuf, &rc);
    if (rc) return rc;
    if (count == 0) return MPI_SUCCESS;                     /* 5479 */
    if (!mvxi_predefined(op) && !mvxi_user_op(op)) return MPI_ERR_OP; /* TEST_MPI_OP */
    k.coll = MVX_COLL_ALLREDUCE; k.sendbuf = sendbuf; k.recvbuf = recvbuf;
    k.count = count; k.recvcnts = NULL; k.dt = dt; k.op = op; k.root = 0;
    return run(c, &k, c->stream, 1);
}

int mvx_coll_reduce(void *sendbuf, void *recvbuf, int count, MPI_Datatype dt,
                    MPI_Op op, int root, MPI_Comm comm)
{
    mvx_comm_t *c = mvxi_get_comm(comm);
    call_t k;
    k.kinds = take_kinds(c);
    int rc = MPI_SUCCESS;
    if (!c) return ERR_COMM_NULL_CODE;
    if (mvx_dtype_info(dt, NULL, NULL)) return ERR_TYPE_NULL_CODE;
    test_alias(sendbuf, recvbuf, &rc);                      /* reduce.c:82-83 */
    test_count(count, &rc);
    if (rc) return rc;
    if (count == 0) return MPI_SUCCESS;                     /* 4541 */
    if (root >= c->size) rc = mvxi_setmsg_code(MPI_ERR_ROOT, ERR_KIND_ROOT_TOOBIG);
    if (root < 0) rc = mvxi_setmsg_code(MPI_ERR_ROOT, ERR_KIND_DEFAULT);
    if (rc) return rc;
    if (!mvxi_predefined(op) && !mvxi_user_op(op)) return MPI_ERR_OP;
    k.coll = MVX_COLL_REDUCE; k.sendbuf = sendbuf; k.recvbuf = recvbuf;
    k.count = count; k.recvcnts = NULL; k.dt = dt; k.op = op; k.root = root;
    return run(c, &k, c->stream, 1);
}

int mvx_coll_reduce_scatter(void *sendbuf, void *recvbuf, int *recvcnts,
                            MPI_Datatype dt, MPI_Op op, MPI_Comm comm)
{
    mvx_comm_t *c = mvxi_get_comm(comm);
    call_t k;
    k.kinds = take_kinds(c);
    int rc = MPI_SUCCESS;
    if (!c) return ERR_COMM_NULL_CODE;
    if (mvx_dtype_info(dt, NULL, NULL)) return ERR_TYPE_NULL_CODE;
    test_alias(recvbuf, sendbuf, &rc);                      /* red_scat.c:77 */
    if (rc) return rc;
    if (!mvxi_predefined(op) && !mvxi_user_op(op)) return MPI_ERR_OP;
    if (!recvcnts) return MPI_ERR_ARG;
    k.coll = MVX_COLL_REDUCE_SCATTER; k.sendbuf = sendbuf; k.recvbuf = recvbuf;
    k.count = 0; k.recvcnts = recvcnts; k.dt = dt; k.op = op; k.root = 0;
    return run(c, &k, c->stream, 1);
}

int mvx_coll_scan(void *sendbuf, void *recvbuf, int count, MPI_Datatype dt,
                  MPI_Op op, MPI_Comm comm)
{
    mvx_comm_t *c = mvxi_get_comm(comm);
    call_t k;
    k.kinds = take_kinds(c);
    int rc = MPI_SUCCESS;
    if (!c) return ERR_COMM_NULL_CODE;                       /* scan.c:74-80 */
    if (mvx_dtype_info(dt, NULL, NULL)) return ERR_TYPE_NULL_CODE;
    test_alias(sendbuf, recvbuf, &rc);
    test_count(count, &rc);
    if (rc) return rc;
    if (count == 0) return MPI_SUCCESS;                     /* scan.c:85 */
    if (!mvxi_predefined(op) && !mvxi_user_op(op)) return MPI_ERR_OP;
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

/* stream-ordered variants: device buffers, no host synchronisation */
static int async_checks(mvx_comm_t *c, MPI_Datatype dt, MPI_Op op)
{
    if (!c) return ERR_COMM_NULL_CODE;
    if (mvx_dtype_info(dt, NULL, NULL)) return ERR_TYPE_NULL_CODE;
    if (!mvxi_predefined(op) && !mvxi_user_op(op)) return MPI_ERR_OP;
    return MPI_SUCCESS;
}

int mvx_allreduce_async(const void *sendbuf, void *recvbuf, int count,
                        MPI_Datatype dt, MPI_Op op, MPI_Comm comm, void *stream)
{
    mvx_comm_t *c = mvxi_get_comm(comm);
    call_t k;
    k.kinds = take_kinds(c);
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
    mvx_comm_t *c = mvxi_get_comm(comm);
    call_t k;
    k.kinds = take_kinds(c);
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
    mvx_comm_t *c = mvxi_get_comm(comm);
    call_t k;
    k.kinds = take_kinds(c);
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
    mvx_comm_t *c = mvxi_get_comm(comm);
    call_t k;
    k.kinds = take_kinds(c);
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
 * transport and slice tables are the communicator's: one call at a time per
 * communicator (MPI-1.2 is not thread-safe either, coll.h:61-68). */
static int run_multi_on(mvx_comm_t *c, int coll, void *const *sendbufs,
                        void *const *recvbufs, long count, const int *recvcnts,
                        MPI_Datatype dt, MPI_Op op, int root, int *rcs,
                        hipStream_t st);

static int run_multi(mvx_comm_t *c, int coll, void *const *sendbufs,
                     void *const *recvbufs, long count, const int *recvcnts,
                     MPI_Datatype dt, MPI_Op op, int root, int *rcs,
                     hipStream_t st)
{
    const int prev = mvxi_dev_enter(c->device);
    int rc;
    if (prev == MVXI_DEV_FAILED) return MPI_ERR_OTHER;
    rc = run_multi_on(c, coll, sendbufs, recvbufs, count, recvcnts, dt, op, root, rcs, st);
    mvxi_dev_leave(c->device, prev);
    return rc;
}

static int run_multi_on(mvx_comm_t *c, int coll, void *const *sendbufs,
                        void *const *recvbufs, long count, const int *recvcnts,
                        MPI_Datatype dt, MPI_Op op, int root, int *rcs,
                        hipStream_t st)
{
    mvx_work *w = mvxi_work(c);
    mvx_plan *plans;
    mvx_xport *t;
    job_t *J;
    const int p = c->size;
    int r, rc, verdict, e, ts, host = 0;
    call_t k;

    if (mvx_dtype_info(dt, &e, &ts)) return ERR_TYPE_NULL_CODE;
    if (!w) return MPI_ERR_INTERN;
    plans = w->multi_plans; t = w->multi_t; J = &w->multi_job;
    c->last_st = st;
    for (r = 0; r < p; r++) rcs[r] = 0;
    if (!mvxi_predefined(op) && !mvxi_user_op(op)) { for (r = 0; r < p; r++) rcs[r] = MPI_ERR_OP; return MPI_SUCCESS; }
    for (r = 0; r < p; r++) {
        rc = mvx_plan_build_tuned(&plans[r], coll, p, r, count, recvcnts, dt, op, root, mvxi_op_kind(op),
                                  &c->tune);
        if (rc) return rc;
    }
    if (plans[0].alg == MVX_ALG_NONE) return MPI_SUCCESS;
    verdict = mvxi_op_verdict(op, dt);
    if (verdict) {
        for (r = 0; r < p; r++) {
            rcs[r] = (verdict == MVX_ERR_OP_NOT_DEFINED && !plans[r].calls_uop) ? 0 : verdict;
            if (coll == MVX_COLL_SCAN && verdict == MVX_ERR_OP_NOT_DEFINED && count > 0) {
                if (plans[r].packed) {
                    if ((rc = mvxi_typed_copy(c, dt, count, sendbufs[r], recvbufs[r], st, 1))) return rc;
                } else if ((rc = mvxi_copy_any(c, recvbufs[r], sendbufs[r], (size_t)(count * e), st, 0))) {
                    return rc;
                }
            }
        }
        if (verdict != MVX_ERR_OP_NOT_DEFINED || coll == MVX_COLL_SCAN || !undefined_moves(c, coll))
            return MPI_SUCCESS;
    }
    k.coll = coll; k.count = count; k.recvcnts = recvcnts; k.root = root;
    J->nr = p;
    J->P = plans;
    J->t = t;
    w->lb.ns = w->lb.nr = 0;
    for (r = 0; r < p; r++) {
        call_sizes(&k, p, r, &J->nsend[r], &J->nrecv[r]);
        J->send[r] = (const char *)sendbufs[r];
        J->recv[r] = (char *)recvbufs[r];
        if (J->nsend[r] && J->send[r] == J->recv[r]) return MPI_ERR_BUFFER;
        mvxi_xport_loopback(&t[r], &w->lb, r);
    }
    J->kinds = 0;
    /* a packed job asks its spans' kinds itself (packed_setup) */
    host = plans[0].packed ? mvxi_job_packed_host(J) : mvxi_job_kinds(J);
    c->keep = verdict == MVX_ERR_OP_NOT_DEFINED;    /* the transfers of an undefined pair */
    if (plans[0].packed) rc = mvxi_run_job_packed(c, J, st, host);
    else rc = host ? mvxi_run_staged(c, J, st) : mvxi_run_device(c, J, st);
    mvxi_job_release(J, rc);
    c->keep = 0;
    return rc;
}

int mvx_allreduce_multi(void *const *sendbufs, void *const *recvbufs, int count,
                        MPI_Datatype dt, MPI_Op op, MPI_Comm comm, int *rc, void *stream)
{
    mvx_comm_t *c = mvxi_get_comm(comm);
    if (!c || !c->local) return ERR_COMM_NULL_CODE;
    if (count < 0) return MPI_ERR_COUNT;
    return run_multi(c, MVX_COLL_ALLREDUCE, sendbufs, recvbufs, count, NULL, dt, op,
                     0, rc, (hipStream_t)stream);
}

int mvx_reduce_multi(void *const *sendbufs, void *const *recvbufs, int count,
                     MPI_Datatype dt, MPI_Op op, int root, MPI_Comm comm, int *rc,
                     void *stream)
{
    mvx_comm_t *c = mvxi_get_comm(comm);
    if (!c || !c->local) return ERR_COMM_NULL_CODE;
    if (count < 0) return MPI_ERR_COUNT;
    if (root < 0 || root >= c->size) return MPI_ERR_ROOT;
    return run_multi(c, MVX_COLL_REDUCE, sendbufs, recvbufs, count, NULL, dt, op,
                     root, rc, (hipStream_t)stream);
}

int mvx_scan_multi(void *const *sendbufs, void *const *recvbufs, int count,
                   MPI_Datatype dt, MPI_Op op, MPI_Comm comm, int *rc, void *stream)
{
    mvx_comm_t *c = mvxi_get_comm(comm);
    if (!c || !c->local) return ERR_COMM_NULL_CODE;
    if (count < 0) return MPI_ERR_COUNT;
    return run_multi(c, MVX_COLL_SCAN, sendbufs, recvbufs, count, NULL, dt, op, 0, rc,
                     (hipStream_t)stream);
}

int mvx_reduce_scatter_multi(void *const *sendbufs, void *const *recvbufs,
                             const int *recvcnts, MPI_Datatype dt, MPI_Op op,
                             MPI_Comm comm, int *rc, void *stream)
{
    mvx_comm_t *c = mvxi_get_comm(comm);
    if (!c || !c->local) return ERR_COMM_NULL_CODE;
    if (!recvcnts) return MPI_ERR_ARG;
    return run_multi(c, MVX_COLL_REDUCE_SCATTER, sendbufs, recvbufs, 0, recvcnts, dt,
                     op, 0, rc, (hipStream_t)stream);
}
