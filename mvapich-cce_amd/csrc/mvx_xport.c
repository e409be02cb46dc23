/*
 * mvx_xport.c -- how a phase's transfers move (mvx_xport, mvx_internal.h):
 *   RCCL            grouped ncclSend / ncclRecv; ncclAllToAll and an
 *                   in-place ncclAllGather for the COLL variant
 *   caller-supplied the mvx_transport table of mvx_comm_init_transport
 *   loopback        every rank of a virtual communicator in this process:
 *                   transfers recorded per phase, paired and copied
 *                   device-to-device once all ranks have issued theirs
 * The reference moves the same blocks with MPI_Sendrecv between processes
 * (intra_fns_new.c, e.g. 5681-5699).
 */
#include <string.h>

#include "mvx_internal.h"

/* ---- RCCL ---------------------------------------------------------------- */
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

/* ---- caller-supplied ------------------------------------------------------
 * nested start / end pairs form one group */
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

/* ---- loopback ------------------------------------------------------------ */
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
int mvxi_lb_flush(loopback_t *lb, hipStream_t st)
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

void mvxi_xport_loopback(mvx_xport *t, loopback_t *lb, int me)
{
    memset(t, 0, sizeof *t);
    t->start = lb_nop; t->end = lb_nop; t->send = lb_send; t->recv = lb_recv;
    t->lb = lb; t->me = me;
}

/* the transport of a one-rank-per-process communicator: RCCL, or the
 * caller's table (with the COLL hooks when it has both) */
void mvxi_xport_comm(mvx_xport *t, mvx_comm_t *c, hipStream_t st)
{
    memset(t, 0, sizeof *t);
    if (c->has_ops) {
        t->start = op_start; t->end = op_end; t->send = op_send; t->recv = op_recv;
        if (c->ops.alltoall && c->ops.allgather) { t->alltoall = op_alltoall; t->allgather = op_allgather; }
        t->ops = &c->ops; t->st = st;
    } else {
        t->start = nc_start; t->end = nc_end; t->send = nc_send; t->recv = nc_recv;
        t->alltoall = nc_alltoall; t->allgather = nc_allgather;
        t->nccl = c->nccl;
    }
    t->me = c->rank;
}
