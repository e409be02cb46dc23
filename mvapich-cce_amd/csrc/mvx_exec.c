/*
 * mvx_exec.c -- one rank's plan on device buffers (the fast path): phase A
 * moves shards to the rank that combines them, phase B runs the combine
 * program, phase C sends combined blocks where they are needed.  Three
 * exchange variants drive the links (MVX_EXCH_*, include/mvx_coll.h); all
 * compute the same bits.  Reference schedules: intra_Allreduce /
 * intra_Reduce / intra_Reduce_scatter (intra_fns_new.c), as planned by
 * mvx_plan.c.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "mvx_internal.h"

static void gtrace(const char *what, int v);

/* ---- one rank's execution of its plan ---------------------------------- */

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
    X->wide_n = P->has_combine ? mvxi_wide_temps(P) : 0;
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
    return mvxi_combine(X->c, P, leafp, exec_out(X), &S, st);
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
int mvxi_exec_group(rank_exec_t *X, mvx_xport *t, int nr, hipStream_t st, mvx_comm_t *timed)
{
    int r, rc;
    if (timed && (rc = mvxi_tev(timed, 0, st))) return rc;
    for (r = 0; r < nr; r++)
        if ((rc = exec_phase_a(&X[r], &t[r], st))) return rc;
    if (t[0].lb && (rc = mvxi_lb_flush(t[0].lb, st))) return rc;
    if (timed && (rc = mvxi_tev(timed, 1, st))) return rc;
    for (r = 0; r < nr; r++)
        if ((rc = exec_phase_b(&X[r], st))) return rc;
    if (timed && (rc = mvxi_tev(timed, 2, st))) return rc;
    for (r = 0; r < nr; r++)
        if ((rc = exec_phase_c(&X[r], &t[r], st))) return rc;
    if (t[0].lb && (rc = mvxi_lb_flush(t[0].lb, st))) return rc;
    if (timed && (rc = mvxi_tev(timed, 3, st))) return rc;
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

void mvxi_plan_slice(const mvx_plan *P, long i, long cs, mvx_plan *Q)
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
long mvxi_plan_span(const mvx_plan *P)
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

int mvxi_send_ranges(const mvx_plan *Q, mvx_range *v)
{
    int n = 0, s;
    for (s = 0; s < Q->p; s++) add_range(v, &n, Q->a_send[s].off, Q->a_send[s].cnt);
    if (Q->has_combine) add_range(v, &n, Q->c_src_off, Q->c_cnt);
    return n;
}

int mvxi_recv_ranges(const mvx_plan *Q, mvx_range *v)
{
    int n = 0, s;
    if (Q->has_combine && !Q->c_dst_tmp) add_range(v, &n, Q->c_dst_off, Q->c_cnt);
    for (s = 0; s < Q->p; s++) add_range(v, &n, Q->b_recv[s].off, Q->b_recv[s].cnt);
    return n;
}


/* the buffers' kinds, one pointer query each (pageable ranges may come back
 * pinned from the registration cache, held for the job until
 * mvxi_job_release); returns 1 if any is host memory */
/* operand q of the job (2r: send of rank r, 2r + 1: its recv) */
static void job_operand(job_t *J, int q, const char **p, size_t *bytes, int **kind, unsigned long **hold)
{
    const int r = q >> 1;
    const size_t E = (size_t)J->P[r].esize;
    if (q & 1) { *p = J->recv[r]; *bytes = (size_t)J->nrecv[r] * E; *kind = &J->rkind[r]; *hold = &J->rhold[r]; }
    else { *p = J->send[r]; *bytes = (size_t)J->nsend[r] * E; *kind = &J->skind[r]; *hold = &J->shold[r]; }
}

int mvxi_job_kinds(job_t *J)
{
    int r, host = 0;
    if (!J->kinds) {
        unsigned long *mine[2 * MVX_MAXP];
        int q, nmine = 0, pass;
        for (q = 0; q < 2 * J->nr; q++) {
            const char *p;
            size_t bytes;
            int *kind;
            unsigned long *hold;
            job_operand(J, q, &p, &bytes, &kind, &hold);
            *hold = 0;
            *kind = bytes ? mvxi_buf_kind_hold(p, bytes, hold, mine, nmine) : MVX_BUF_DEVICE;
            if (*hold) mine[nmine++] = hold;
        }
        /* an operand whose registration was merged into another's union and
         * then lost (the union could not be registered) is asked again */
        for (pass = 0; pass < 2 * J->nr; pass++) {
            int again = 0;
            for (q = 0; q < 2 * J->nr; q++) {
                const char *p;
                size_t bytes;
                int *kind, i, n = 0;
                unsigned long *hold, *others[2 * MVX_MAXP];
                job_operand(J, q, &p, &bytes, &kind, &hold);
                if (*kind != MVX_BUF_PINNED || *hold || !bytes || mvx_host_pinned(p) == 1) continue;
                for (i = 0; i < nmine; i++)
                    if (mine[i] != hold) others[n++] = mine[i];
                *kind = mvxi_buf_kind_hold(p, bytes, hold, others, n);
                if (*hold) {
                    for (i = 0; i < nmine && mine[i] != hold; i++) ;
                    if (i == nmine) mine[nmine++] = hold;
                }
                again = 1;
            }
            if (!again) break;
        }
        J->kinds = 1;
    }
    for (r = 0; r < J->nr; r++) host |= J->skind[r] != MVX_BUF_DEVICE || J->rkind[r] != MVX_BUF_DEVICE;
    return host;
}

void mvxi_job_release(job_t *J, int rc)
{
    int r, any = 0;
    if (!J->kinds) return;
    for (r = 0; r < J->nr; r++) any |= J->shold[r] || J->rhold[r];
    if (!any) return;
    if (rc != MPI_SUCCESS && hipDeviceSynchronize() != hipSuccess) (void)hipGetLastError();
    for (r = 0; r < J->nr; r++) {
        mvxi_buf_release(J->shold[r]);
        mvxi_buf_release(J->rhold[r]);
        J->shold[r] = J->rhold[r] = 0;
    }
}


/* every local rank's staging region for plans Q: X[r].P / c set, per-rank
 * offsets in off[], total bytes returned (pool not touched) */
size_t mvxi_region_layout(mvx_comm_t *c, rank_exec_t *X, const job_t *J, const mvx_plan *Q, size_t *off)
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

int mvxi_job_layout(mvx_comm_t *c, rank_exec_t *X, const job_t *J, const mvx_plan *Q)
{
    size_t off[MVX_MAXP];
    const size_t need = mvxi_region_layout(c, X, J, Q, off);
    int r, rc;
    if ((rc = mvxi_grow_pool(c, need))) return rc;
    for (r = 0; r < J->nr; r++) X[r].pool = c->pool + off[r];
    return MPI_SUCCESS;
}

/* ---- exchange variants (MVX_EXCH_*) -------------------------------------
 * PIPE: phase A runs in slices, one transfer group per slice on the call's
 * stream; slice t's combine runs on a second stream as soon as slice t has
 * arrived, while slice t + 1 is still on the links; phase C is one transfer
 * group after the last combine, as P2P's.  On links that bound the step, the
 * combine is then exposed for one slice instead of whole.  Slices keep every
 * block boundary (plan_slice), so the bits are the unsliced plan's.
 *
 * Host cost (round 4, tools/graph_cost.c): every cross-stream dependency
 * (an event record or wait) costs about 4-5 us to issue on this runtime, a
 * replayed graph included, and every send / receive about 0.7-1 us.  So
 * the schedule uses one fork per slice and a single join (2 S + 2 event
 * operations, S + 1 transfer groups, 2(p - 1) operations per slice of A and
 * one phase C) -- not a join per slice and a group per step carrying slice
 * t's exchange with slice t - 2's distribution, which cost 4 S event
 * operations and twice the transfers for the same overlap where the links
 * are the bound.  Every slice has its own staging region (together about
 * the unsliced plan's) and a non-root Reduce's temporary result is kept
 * whole, so phase C is the unsliced plan's on every rank and the ranks'
 * messages pair up whatever each one's own plan holds.  The slice plans
 * and rank tables are the communicator's (mvx_work). */

/* The combine stream needs a hardware queue of its own (mvxi_queue_stream):
 * on a shared queue slice t + 1's transfers waited behind slice t's combine
 * (round 4, tools/prof_pipe_overlap.sh: 0.1 % of the combine time under a
 * transfer; 75-78 % of it with 4 slices on a queue of its own).  The queue
 * comes from a full CU mask rather than a raised priority: at equal
 * priority the dispatcher serves the transfer kernel's few workgroups
 * between the combine's, where a high-priority combine grid would be
 * dispatched whole first. */
static int pipe_streams(mvx_comm_t *c)
{
    int i;
    if (c->cstream) return MPI_SUCCESS;
    if (mvxi_queue_stream(&c->cstream, "MVX_PIPE_STREAM", "cumask") != hipSuccess) return MPI_ERR_OTHER;
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
    if ((rc = mvxi_job_layout(c, X, J, J->P))) return rc;
    return mvxi_exec_group(X, J->t, J->nr, st, c);
}

/* rank r's tables for slice t (staging region t); a non-root Reduce's
 * temporary result goes to its place in the unsliced temporary at tmp */
static void pipe_slice(const job_t *J, int r, long t, long cs, char *region_base, char *tmp,
                       const rank_exec_t *X0, rank_exec_t *X, mvx_plan *Q)
{
    *X = X0[r];
    mvxi_plan_slice(&J->P[r], t, cs, Q);
    X->P = Q;
    X->pool = region_base;
    if (Q->c_dst_tmp) X->tmp_off = (size_t)(tmp + t * cs * Q->esize - region_base);
}

static int graph_streams(mvx_comm_t *c);
static int run_device_pipe_on(mvx_comm_t *c, const job_t *J, hipStream_t st);

/* The combine stream may be a blocking stream (hipExtStreamCreateWithCUMask
 * takes no flags), and the legacy null stream waits for every blocking
 * stream: slice t + 1's transfers issued on it would wait for slice t's
 * combine.  A null-stream call therefore runs its slices on the
 * communicator's non-blocking stream, forked from the null stream and joined
 * back (as a null-stream graph launch does); a capture is already on it. */
static int run_device_pipe(mvx_comm_t *c, const job_t *J, hipStream_t st)
{
    int rc;
    if (st || mvxi_capturing) return run_device_pipe_on(c, J, st);
    if ((rc = graph_streams(c))) return rc;
    if (hipEventRecord(c->gev[0], st) != hipSuccess || hipStreamWaitEvent(c->gstream, c->gev[0], 0) != hipSuccess)
        return MPI_ERR_OTHER;
    rc = run_device_pipe_on(c, J, c->gstream);
    if (hipEventRecord(c->gev[1], c->gstream) != hipSuccess || hipStreamWaitEvent(st, c->gev[1], 0) != hipSuccess)
        return rc ? rc : MPI_ERR_OTHER;
    return rc;
}

static int run_device_pipe_on(mvx_comm_t *c, const job_t *J, hipStream_t st)
{
    mvx_work *w = mvxi_work(c);
    rank_exec_t *X0, (*X)[MVX_MAXP];
    mvx_plan (*pl)[MVX_MAXP];
    size_t off[MVX_MAXP], toff[MVX_MAXP], region, tmp_bytes = 0;
    long span = 0, cs, nsl, t;
    int r, rc;
    const int ns = c->exch_slices > 0 ? c->exch_slices : 4;
    if (!w) return MPI_ERR_INTERN;
    X0 = w->px0; X = w->px; pl = w->pipe;
    for (r = 0; r < J->nr; r++) {
        if (mvxi_plan_span(&J->P[r]) > span) span = mvxi_plan_span(&J->P[r]);
        toff[r] = tmp_bytes;
        if (J->P[r].c_dst_tmp) tmp_bytes = al256(tmp_bytes + (size_t)(J->P[r].c_cnt * J->P[r].esize));
    }
    cs = (span + ns - 1) / ns;
    cs = (cs + 255) & ~255L;
    nsl = (span + cs - 1) / cs;
    if (nsl <= 1) return run_device_plain(c, J, st);
    if ((rc = pipe_streams(c))) return rc;
    c->ran_exch = MVX_EXCH_PIPE;
    for (r = 0; r < J->nr; r++) {
        mvxi_plan_slice(&J->P[r], 0, cs, &pl[0][r]);
        /* a non-root Reduce's result goes to the shared unsliced temporary
         * (pipe_slice): no slot for it in the per-slice regions */
        pl[0][r].c_dst_tmp = 0;
        X0[r].sendbuf = J->send[r];
        X0[r].recvbuf = J->recv[r];
    }
    region = mvxi_region_layout(c, X0, J, pl[0], off);   /* slice 0 is the largest */
    if ((rc = mvxi_grow_pool(c, (size_t)nsl * region + tmp_bytes))) return rc;
    if ((rc = mvxi_tev(c, 0, st))) return rc;
    for (t = 0; t < nsl; t++) {
        const int k = (int)(t & 1);
        if (mvxi_capturing) gtrace("pipe slice", (int)t);
        for (r = 0; r < J->nr; r++) {
            pipe_slice(J, r, t, cs, c->pool + (size_t)t * region + off[r], c->pool + (size_t)nsl * region + toff[r],
                       X0, &X[k][r], &pl[k][r]);
            if ((rc = exec_phase_a(&X[k][r], &J->t[r], st))) return rc;
        }
        if (J->t[0].lb && (rc = mvxi_lb_flush(J->t[0].lb, st))) return rc;
        if (hipEventRecord(c->pev[k], st) != hipSuccess || hipStreamWaitEvent(c->cstream, c->pev[k], 0) != hipSuccess)
            return MPI_ERR_OTHER;
        for (r = 0; r < J->nr; r++)
            if ((rc = exec_phase_b(&X[k][r], c->cstream))) return rc;
    }
    if (hipEventRecord(c->pev[2], c->cstream) != hipSuccess || hipStreamWaitEvent(st, c->pev[2], 0) != hipSuccess)
        return MPI_ERR_OTHER;
    if (mvxi_capturing) gtrace("pipe combines joined", (int)nsl);
    /* phase C unsliced, as P2P's: the combined blocks are whole in recvbuf,
     * or in the unsliced temporary (a non-root Reduce), so every rank sends
     * and receives the same messages whatever its own plan holds */
    for (r = 0; r < J->nr; r++) {
        X[0][r] = X0[r];
        X[0][r].P = &J->P[r];
        if (J->P[r].c_dst_tmp) {
            X[0][r].pool = c->pool + (size_t)nsl * region + toff[r];
            X[0][r].tmp_off = 0;
        }
        if ((rc = exec_phase_c(&X[0][r], &J->t[r], st))) return rc;
    }
    if (J->t[0].lb && (rc = mvxi_lb_flush(J->t[0].lb, st))) return rc;
    if ((rc = mvxi_tev(c, 3, st))) return rc;
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
    X.wide_n = mvxi_wide_temps(P);
    X.wide_slot = al256(bb + SLOT_STAGGER);
    if ((rc = mvxi_grow_pool(c, stage + X.wide_slot * (size_t)X.wide_n))) return rc;
    c->ran_exch = MVX_EXCH_COLL;
    if ((rc = mvxi_tev(c, 0, st))) return rc;
    if ((rc = t->alltoall(t, J->send[0], c->pool, bb, st))) return rc;
    if ((rc = mvxi_tev(c, 1, st))) return rc;
    for (s = 0; s < P->p; s++)
        leafp[s] = s == P->rank ? J->send[0] + (size_t)P->rank * bb : c->pool + (size_t)s * bb;
    S.base = c->pool + stage; S.slot = X.wide_slot; S.used = 0; S.cap = X.wide_n;
    if ((rc = mvxi_combine(c, P, leafp, J->recv[0] + P->c_dst_off * P->esize, &S, st))) return rc;
    if ((rc = mvxi_tev(c, 2, st))) return rc;
    if (P->coll == MVX_COLL_ALLREDUCE && (rc = t->allgather(t, J->recv[0], bb, st))) return rc;
    if ((rc = mvxi_tev(c, 3, st))) return rc;
    if (c->timing) c->tev_kind = TEV_PHASES;
    return MPI_SUCCESS;
}

/* all buffers in HBM */
static int run_device_eager(mvx_comm_t *c, const job_t *J, hipStream_t st)
{
    long blk;
    c->ran_exch = MVX_EXCH_P2P;   /* unless a variant below takes the call */
    if (c->exch == MVX_EXCH_PIPE) return run_device_pipe(c, J, st);
    if (c->exch == MVX_EXCH_COLL && J->nr == 1 && J->t[0].alltoall && J->t[0].allgather &&
        J->P[0].opkind == MVX_OPKIND_PREDEFINED && coll_regular(&J->P[0], &blk))
        return run_device_coll(c, J, blk, st);
    return run_device_plain(c, J, st);
}

/* ---- graphs (mvx_comm_set_graphs) ---------------------------------------
 * The first call of a job runs eagerly (it also sizes the staging pool and
 * opens RCCL's connections); the second is captured into a HIP graph on the
 * call's stream -- RCCL's groups record their kernels, PIPE's combine stream
 * joins through its events -- and launched; later ones replay it.  A
 * capture that fails turns graphs off on the communicator (graph_error) and
 * the call runs eagerly.  Null-stream calls capture and replay on the
 * communicator's own stream, forked from and joined back to the null
 * stream with events. */
#define G_FREE 0
#define G_SEEN 1
#define G_LIVE 2
#define G_RETIRED 3

static unsigned long long graph_hash(const mvx_comm_t *c, const job_t *J, hipStream_t st)
{
    const unsigned char *b = (const unsigned char *)&J->P[0];
    unsigned long long h = 1469598103934665603ull;
    const uintptr_t v[6] = {(uintptr_t)J->send[0], (uintptr_t)J->recv[0], (uintptr_t)st, (uintptr_t)c->pool,
                            (uintptr_t)(c->exch * 4096 + c->exch_slices), (uintptr_t)c->keep};
    size_t i;
    for (i = 0; i < sizeof(mvx_plan); i++) h = (h ^ b[i]) * 1099511628211ull;
    for (i = 0; i < 6; i++) h = (h ^ v[i]) * 1099511628211ull;
    return h;
}

static int graph_match(const graph_ent_t *g, const mvx_comm_t *c, const job_t *J, hipStream_t st,
                       unsigned long long h)
{
    return (g->state == G_SEEN || g->state == G_LIVE) && g->hash == h && g->send == J->send[0] && g->recv == J->recv[0] && g->st == st &&
           g->pool == c->pool && g->exch == c->exch && g->slices == c->exch_slices && g->keep == c->keep &&
           !memcmp(&g->plan, &J->P[0], sizeof(mvx_plan));
}

/* Captured graphs live as long as their communicator.  Destroying one
 * mid-life -- an LRU eviction, or a graph made on a pool since reallocated
 * -- and then capturing another made the new graph die in hipGraphLaunch
 * (SIGSEGV, round 4, at p = 2 and 4 over RCCL's socket transport, with an
 * eager call between the two or not).  So nothing captured is destroyed
 * before mvx_comm_free (mvxi_graphs_clear, run before ncclCommDestroy): a
 * graph whose pool was reallocated is retired (state 3, never matched
 * again), seen-once entries are the only ones replaced, and a communicator
 * that has captured GRAPH_CACHE graphs runs its new jobs eagerly.
 *
 * Round 5 found the cause: HIP 7.0's hipGraphLaunch crashes after execs of
 * graphs with parallel branches were destroyed (tools/graph_probe2.c: a
 * fork / join graph of two memsets, captured, launched and destroyed in a
 * loop, dies within 30 rounds on HIP 7.0 and never on 7.2; kept alive, or
 * without the fork, it never dies; no RCCL needed).  So graphs are destroyed
 * mid-life again -- before the pool they were captured on is freed, and the
 * least recently used one when every slot holds a graph and a job seen
 * twice is about to be captured -- where the runtime allows
 * (mvxi_graph_evict_default): any graph from HIP 7.2 on, only single-branch
 * ones before it (PIPE's forked captures are retired there).
 * MVX_GRAPH_CACHE=n (<= 32) caps the graphs a communicator holds. */

static void graph_destroy(graph_ent_t *g)
{
    if ((g->state == G_LIVE || g->state == G_RETIRED) && g->exec) {
        gtrace("destroy graph of variant", g->exch);
        hipGraphExecDestroy(g->exec);
    }
    if (g->done) hipEventDestroy(g->done);
    memset(g, 0, sizeof *g);
}

/* a graph destroyed mid-life (counted for mvx_comm_graph_stats) */
static void graph_evict(mvx_comm_t *c, graph_ent_t *g)
{
    graph_destroy(g);
    c->w->graphs_destroyed++;
}

int mvx_comm_graph_stats(MPI_Comm comm, int *live, int *retired, long *destroyed)
{
    mvx_comm_t *c = mvxi_get_comm(comm);
    int i, l = 0, r = 0;
    if (!c) return ERR_COMM_NULL_CODE;
    for (i = 0; c->w && i < GRAPH_CACHE; i++) {
        l += c->w->graphs[i].state == G_LIVE;
        r += c->w->graphs[i].state == G_RETIRED;
    }
    if (live) *live = l;
    if (retired) *retired = r;
    if (destroyed) *destroyed = c->w ? c->w->graphs_destroyed : 0;
    return MPI_SUCCESS;
}

void mvxi_graphs_clear(mvx_comm_t *c)
{
    int i;
    if (!c->w) return;
    for (i = 0; i < GRAPH_CACHE; i++) {
        graph_destroy(&c->w->graphs[i]);
        memset(&c->w->seen[i], 0, sizeof c->w->seen[i]);
    }
}

/* may this graph's exec be destroyed now (mvxi_graph_evict_default)? */
static int graph_evictable(const mvx_comm_t *c, const graph_ent_t *g)
{
    if (c->graph_evict == MVX_GRAPH_EVICT_ALL) return 1;
    return c->graph_evict == MVX_GRAPH_EVICT_SERIAL && !g->forked;
}

/* 1 if the graph has parallel branches: a node with two or more successors,
 * or two or more roots (what HIP runs on parallel streams) */
static int graph_forked(hipGraph_t g)
{
    size_t ne = 0, nr = 0, i, j;
    hipGraphNode_t *from, *to;
    int forked = 0;
    if (hipGraphGetRootNodes(g, NULL, &nr) != hipSuccess || hipGraphGetEdges(g, NULL, NULL, &ne) != hipSuccess) {
        (void)hipGetLastError();
        return 1;                                   /* unknown: treat as forked */
    }
    if (nr > 1) return 1;
    if (!ne) return 0;
    from = (hipGraphNode_t *)malloc(ne * sizeof *from);
    to = (hipGraphNode_t *)malloc(ne * sizeof *to);
    if (!from || !to || hipGraphGetEdges(g, from, to, &ne) != hipSuccess) {
        (void)hipGetLastError();
        free(from);
        free(to);
        return 1;
    }
    for (i = 0; i < ne && !forked; i++)             /* out-degree >= 2 */
        for (j = i + 1; j < ne && !forked; j++) forked = from[i] == from[j];
    free(from);
    free(to);
    return forked;
}

/* The pool is about to be freed: every graph captured on it goes first --
 * destroyed where the runtime allows it (after its own last launch
 * completed, so none of it is in flight), else retired (kept, never matched
 * again, destroyed with the communicator). */
int mvxi_grow_pool(mvx_comm_t *c, size_t need)
{
    int i;
    if (need <= c->pool_bytes) return MPI_SUCCESS;
    if (c->w && c->pool && !mvxi_capturing) {
        int gone = 0;
        for (i = 0; i < GRAPH_CACHE; i++) {
            graph_ent_t *g = &c->w->graphs[i];
            if (c->w->seen[i].pool == c->pool) memset(&c->w->seen[i], 0, sizeof c->w->seen[i]);
            if (g->pool != c->pool) continue;
            if (g->state == G_LIVE) { g->state = G_RETIRED; gone += graph_evictable(c, g); }
        }
        if (gone) {
            for (i = 0; i < GRAPH_CACHE; i++) {
                graph_ent_t *g = &c->w->graphs[i];
                if (g->state != G_RETIRED || !graph_evictable(c, g)) continue;
                /* its last launch done (the pool it reads is about to go) */
                if (g->done && hipEventSynchronize(g->done) != hipSuccess) (void)hipGetLastError();
                graph_evict(c, g);
            }
        }
    }
    return mvxi_grow(&c->pool, &c->pool_bytes, need);
}

/* MVX_GRAPH_FORK=0: PIPE (whose capture forks to the combine stream and
 * joins back) runs eagerly even with graphs on (diagnostics) */
static int forked_capture_ok(void)
{
    static int ok = -1;
    if (ok < 0) {
        const char *e = getenv("MVX_GRAPH_FORK");
        ok = !e || atoi(e) != 0;
    }
    return ok;
}

static int graph_eligible(const mvx_comm_t *c, const job_t *J)
{
    return c->graphs && !c->graph_error && J->nr == 1 && !c->local && !c->has_ops && c->nccl && !c->timing &&
           J->P[0].opkind == MVX_OPKIND_PREDEFINED && !J->P[0].packed &&
           (c->exch != MVX_EXCH_PIPE || forked_capture_ok());
}

static int graph_streams(mvx_comm_t *c)
{
    if (c->gstream) return MPI_SUCCESS;
    if (hipStreamCreateWithFlags(&c->gstream, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&c->gev[0], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->gev[1], hipEventDisableTiming) != hipSuccess)
        return MPI_ERR_OTHER;
    return MPI_SUCCESS;
}

/* launch g's exec on `st` (the null stream: forked onto the graph stream and
 * joined back) and record g->done where it ran */
static int graph_launch(mvx_comm_t *c, graph_ent_t *g, hipStream_t st)
{
    hipStream_t on = st ? st : c->gstream;
    if (st) {
        gtrace("launch on the caller's stream", 0);
        if (hipGraphLaunch(g->exec, st) != hipSuccess) return MPI_ERR_OTHER;
    } else {
        gtrace("launch: fork from the null stream", 0);
        if (hipEventRecord(c->gev[0], st) != hipSuccess || hipStreamWaitEvent(c->gstream, c->gev[0], 0) != hipSuccess)
            return MPI_ERR_OTHER;
        gtrace("launch: hipGraphLaunch on the graph stream", 0);
        if (hipGraphLaunch(g->exec, c->gstream) != hipSuccess) return MPI_ERR_OTHER;
        gtrace("launch: join to the null stream", 0);
        if (hipEventRecord(c->gev[1], c->gstream) != hipSuccess || hipStreamWaitEvent(st, c->gev[1], 0) != hipSuccess)
            return MPI_ERR_OTHER;
    }
    return hipEventRecord(g->done, on) == hipSuccess ? MPI_SUCCESS : MPI_ERR_OTHER;
}

/* MVX_GRAPH_TRACE=1: each capture step on stderr (diagnostics) */
static void gtrace(const char *what, int v)
{
    static int on = -1;
    if (on < 0) {
        const char *e = getenv("MVX_GRAPH_TRACE");
        on = e && atoi(e) == 1;
    }
    if (on) fprintf(stderr, "mvx graph: %s %d\n", what, v);
}

/* capture the job on `cs` into an executable graph (nothing runs) */
static int graph_capture(mvx_comm_t *c, const job_t *J, hipStream_t cs, hipGraphExec_t *out, int *forked)
{
    hipGraph_t g = NULL;
    hipError_t e;
    int rc;
    *out = NULL;
    gtrace("begin capture, variant", c->exch);
    if (hipStreamBeginCapture(cs, hipStreamCaptureModeThreadLocal) != hipSuccess) {
        (void)hipGetLastError();
        return MPI_ERR_OTHER;
    }
    mvxi_capturing = 1;
    rc = run_device_eager(c, J, cs);
    mvxi_capturing = 0;
    gtrace("captured job, rc", rc);
    e = hipStreamEndCapture(cs, &g);
    gtrace("end capture, hip error", (int)e);
    if (rc || e != hipSuccess || !g) {
        if (g) hipGraphDestroy(g);
        (void)hipGetLastError();
        return rc ? rc : MPI_ERR_OTHER;
    }
    *forked = graph_forked(g);
    e = hipGraphInstantiate(out, g, NULL, NULL, 0);
    gtrace("instantiate, hip error", (int)e);
    gtrace("instantiated graph has parallel branches", *forked);
    hipGraphDestroy(g);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        *out = NULL;
        return MPI_ERR_OTHER;
    }
    return MPI_SUCCESS;
}

/* Graph slots hold captured graphs only; jobs seen once wait in a table of
 * their own (mvx_work.seen, least recently seen replaced).  A job runs
 * eagerly at its first sighting and is captured at its second: only then,
 * when every slot holds a graph, is the least recently used evictable one
 * destroyed -- after its own last launch completed (its done event), not
 * the whole device.  A communicator with more distinct jobs than slots thus
 * keeps its graphs instead of trading one for every new job it sees. */
static int run_device_graph(mvx_comm_t *c, const job_t *J, hipStream_t st)
{
    mvx_work *w = mvxi_work(c);
    const unsigned long long h = graph_hash(c, J, st);
    graph_ent_t *g = NULL, *slot = NULL, *seen = NULL, *sslot = NULL, *lru = NULL;
    hipGraphExec_t x;
    int i, rc, forked = 1;
    if (!w || (!st && graph_streams(c))) return run_device_eager(c, J, st);
    for (i = 0; i < c->graph_cap; i++) {
        graph_ent_t *e = &w->graphs[i];
        if (graph_match(e, c, J, st, h)) { g = e; break; }
        if (e->state == G_FREE && !slot) slot = e;
        if (e->state == G_LIVE && graph_evictable(c, e) && (!lru || e->stamp < lru->stamp)) lru = e;
    }
    if (g) {                                                   /* replay */
        g->stamp = ++w->graph_clock;
        c->ran_exch = g->ran_exch;
        c->last_graph = 1;
        return graph_launch(c, g, st);
    }
    for (i = 0; i < GRAPH_CACHE; i++) {
        graph_ent_t *e = &w->seen[i];
        if (graph_match(e, c, J, st, h)) { seen = e; break; }
        if (!sslot || (sslot->state != G_FREE && (e->state == G_FREE || e->stamp < sslot->stamp))) sslot = e;
    }
    if (!seen) {                                               /* first sighting: eager */
        c->last_graph = 0;
        rc = run_device_eager(c, J, st);
        if (rc) return rc;
        memset(sslot, 0, sizeof *sslot);
        sslot->state = G_SEEN;
        sslot->hash = graph_hash(c, J, st);                    /* the pool as the call left it */
        sslot->plan = J->P[0];
        sslot->send = J->send[0]; sslot->recv = J->recv[0]; sslot->st = st; sslot->pool = c->pool;
        sslot->exch = c->exch; sslot->slices = c->exch_slices; sslot->keep = c->keep;
        sslot->stamp = ++w->graph_clock;
        return MPI_SUCCESS;
    }
    /* second sighting: capture, into a free slot or the LRU graph's */
    if (!slot && lru) {
        if (lru->done && hipEventSynchronize(lru->done) != hipSuccess) (void)hipGetLastError();
        graph_evict(c, lru);
        slot = lru;
    }
    memset(seen, 0, sizeof *seen);
    if (!slot) {                                               /* every slot holds a graph it may not destroy */
        c->last_graph = 0;
        return run_device_eager(c, J, st);
    }
    if (hipEventCreateWithFlags(&slot->done, hipEventDisableTiming) != hipSuccess) {
        (void)hipGetLastError();
        slot->done = NULL;
        c->last_graph = 0;
        return run_device_eager(c, J, st);
    }
    rc = graph_capture(c, J, st ? st : c->gstream, &x, &forked);
    if (rc) {
        c->graph_error = rc;
        graph_destroy(slot);
        c->last_graph = 0;
        return run_device_eager(c, J, st);
    }
    slot->state = G_LIVE;
    slot->hash = graph_hash(c, J, st);
    slot->plan = J->P[0];
    slot->send = J->send[0]; slot->recv = J->recv[0]; slot->st = st; slot->pool = c->pool;
    slot->exch = c->exch; slot->slices = c->exch_slices; slot->keep = c->keep;
    slot->exec = x;
    slot->forked = forked;
    slot->ran_exch = c->ran_exch;
    slot->stamp = ++w->graph_clock;
    c->last_graph = 2;
    rc = graph_launch(c, slot, st);
    gtrace("first launch, rc", rc);
    return rc;
}

int mvxi_run_device(mvx_comm_t *c, const job_t *J, hipStream_t st)
{
    if (graph_eligible(c, J)) return run_device_graph(c, J, st);
    c->last_graph = 0;
    return run_device_eager(c, J, st);
}
