/*
 * mvx_stage.c -- host buffers and datatypes with holes.  MPI user buffers
 * live in the caller's address space (the reference's collectives read and
 * write them in place, src/coll/allreduce.c:57-92); no call computes on the
 * host, so host operands are streamed through HBM and the device path runs
 * on them there:
 *
 *   slice schedule   one rank per process at p > 1, a blocking call of at
 *                    least MVX_SLICE_MIN_MIB: every rank runs the call in the
 *                    same slices whatever its buffers' kind, so a host-buffer
 *                    rank overlaps H2D, the collective and D2H of successive
 *                    slices and still pairs with device-buffer ranks
 *   HBM mirrors      one rank per process at p > 1, smaller calls: the call
 *                    moves exactly what a device-buffer call moves, so ranks
 *                    may mix buffer kinds in one call, as MPI allows
 *   sliced pipeline  p = 1, virtual communicators, or every rank promising
 *                    host buffers (mvx_comm_set_host_pipeline): H2D, the
 *                    collective and D2H of successive slices overlap
 *   packed types     the plans run on packed type-map bytes
 *
 * All staging resources (streams, events, bounce slots, slice plans) are the
 * communicator's (mvx_work).
 */
#include <stdlib.h>
#include <string.h>

#include "mvx_internal.h"

/* ---- host buffers: a sliced pipeline ------------------------------------
 * Slice i of every local rank's plan is staged in (H2D on stream sh), run
 * (phases A-C on the caller's stream), and staged out (D2H on stream sd);
 * the host drains slice i-L after issuing slice i (L: mvxi_host_drain_lag,
 * mvx_host.c), so host
 * copies, both PCIe directions and the collective overlap.  Page-locked
 * buffers are moved by DMA directly; pageable ones go through pinned bounce
 * slots filled and emptied by the copy pool (mvx_host.c). */
#define STAGE_SLICE_BYTES (16L << 20)


static int stage_init(stage_res_t *R, size_t bounce)
{
    int b;
    if (!R->ready) {
        if (mvxi_queue_stream(&R->sh, "MVX_STAGE_STREAM", "plain") != hipSuccess ||
            mvxi_queue_stream(&R->sd, "MVX_STAGE_STREAM", "plain") != hipSuccess)
            return MPI_ERR_OTHER;
        for (b = 0; b < STAGE_NB; b++)
            if (hipEventCreateWithFlags(&R->ein[b], hipEventDisableTiming) != hipSuccess ||
                hipEventCreateWithFlags(&R->eout[b], hipEventDisableTiming) != hipSuccess ||
                hipEventCreateWithFlags(&R->ex[b], hipEventDisableTiming) != hipSuccess)
                return MPI_ERR_OTHER;
        R->ready = 1;
    }
    if (bounce > R->bbytes) {
        for (b = 0; b < STAGE_NB; b++) {
            if (R->bin[b]) hipHostFree(R->bin[b]);
            if (R->bout[b]) hipHostFree(R->bout[b]);
            R->bin[b] = R->bout[b] = NULL;
        }
        R->bbytes = 0;
        for (b = 0; b < STAGE_NB; b++)
            if (hipHostMalloc((void **)&R->bin[b], bounce, hipHostMallocDefault) != hipSuccess ||
                hipHostMalloc((void **)&R->bout[b], bounce, hipHostMallocDefault) != hipSuccess)
                return MPI_ERR_OTHER;
        R->bbytes = bounce;
    }
    return MPI_SUCCESS;
}

typedef struct {
    const job_t *J;
    stage_res_t *R;                            /* the communicator's streams / bounce slots */
    char *dsend[MVX_MAXP], *drecv[MVX_MAXP];   /* device buffers the plans run on */
    int shost[MVX_MAXP], rhost[MVX_MAXP];      /* 1: caller's buffer is host memory */
    int spin[MVX_MAXP], rpin[MVX_MAXP];        /* ... and page-locked */
    long cs;                                   /* slice length, elements */
    int single;                                /* the job is one slice */
    int any_host;                              /* some buffer is host memory */
} stage_job_t;


/* slice i in: host -> device for every host send buffer.  A job of one
 * slice (S->single) copies on the caller's stream itself: nothing to overlap,
 * and no event round trips on the small-message path. */
static int stage_in(stage_job_t *S, const mvx_plan *Q, long i, hipStream_t st)
{
    const int b = (int)(i % STAGE_NB);
    const hipStream_t hs = S->single ? st : S->R->sh;
    mvx_range v[MVX_MAXP + 1];
    size_t boff = 0;
    int r, n, j;
    if (!S->any_host) return MPI_SUCCESS;
    if (!S->single && i >= STAGE_NB && hipEventSynchronize(S->R->ein[b]) != hipSuccess) return MPI_ERR_OTHER;
    for (r = 0; r < S->J->nr; r++) {
        const long E = Q[r].esize;
        if (!S->shost[r]) continue;
        n = mvxi_send_ranges(&Q[r], v);
        for (j = 0; j < n; j++) {
            const size_t o = (size_t)(v[j].off * E), bytes = (size_t)(v[j].cnt * E);
            const char *src = S->J->send[r] + o;
            if (!S->spin[r]) {
                mvx_pcopy(S->R->bin[b] + boff, src, bytes);
                src = S->R->bin[b] + boff;
                boff += al256(bytes);
            }
            if (hipMemcpyAsync(S->dsend[r] + o, src, bytes, hipMemcpyHostToDevice, hs) != hipSuccess)
                return MPI_ERR_OTHER;
        }
    }
    if (S->single) return MPI_SUCCESS;
    if (hipEventRecord(S->R->ein[b], S->R->sh) != hipSuccess ||
        hipStreamWaitEvent(st, S->R->ein[b], 0) != hipSuccess)
        return MPI_ERR_OTHER;
    return MPI_SUCCESS;
}

/* slice i out, enqueue: device -> host (bounce or page-locked target) */
static int stage_out(stage_job_t *S, const mvx_plan *Q, long i, hipStream_t st)
{
    const int b = (int)(i % STAGE_NB);
    const hipStream_t ds = S->single ? st : S->R->sd;
    mvx_range v[MVX_MAXP + 1];
    size_t boff = 0;
    int r, n, j;
    if (!S->any_host) return MPI_SUCCESS;
    if (!S->single && (hipEventRecord(S->R->ex[b], st) != hipSuccess ||
                       hipStreamWaitEvent(S->R->sd, S->R->ex[b], 0) != hipSuccess))
        return MPI_ERR_OTHER;
    for (r = 0; r < S->J->nr; r++) {
        const long E = Q[r].esize;
        if (!S->rhost[r]) continue;
        n = mvxi_recv_ranges(&Q[r], v);
        for (j = 0; j < n; j++) {
            const size_t o = (size_t)(v[j].off * E), bytes = (size_t)(v[j].cnt * E);
            char *dst = S->rpin[r] ? S->J->recv[r] + o : S->R->bout[b] + boff;
            if (!S->rpin[r]) boff += al256(bytes);
            if (hipMemcpyAsync(dst, S->drecv[r] + o, bytes, hipMemcpyDeviceToHost, ds) != hipSuccess)
                return MPI_ERR_OTHER;
        }
    }
    if (S->single) return MPI_SUCCESS;
    return hipEventRecord(S->R->eout[b], S->R->sd) == hipSuccess ? MPI_SUCCESS : MPI_ERR_OTHER;
}

/* slice i out, finish: wait for its D2H, bounce -> pageable target */
static int stage_drain(stage_job_t *S, const mvx_plan *Q, long i, hipStream_t st)
{
    const int b = (int)(i % STAGE_NB);
    mvx_range v[MVX_MAXP + 1];
    size_t boff = 0;
    int r, n, j;
    if (!S->any_host) return MPI_SUCCESS;
    if ((S->single ? hipStreamSynchronize(st) : hipEventSynchronize(S->R->eout[b])) != hipSuccess)
        return MPI_ERR_OTHER;
    for (r = 0; r < S->J->nr; r++) {
        const long E = Q[r].esize;
        if (!S->rhost[r] || S->rpin[r]) continue;
        n = mvxi_recv_ranges(&Q[r], v);
        for (j = 0; j < n; j++) {
            const size_t o = (size_t)(v[j].off * E), bytes = (size_t)(v[j].cnt * E);
            mvx_pcopy(S->J->recv[r] + o, S->R->bout[b] + boff, bytes);
            boff += al256(bytes);
        }
    }
    return MPI_SUCCESS;
}

/* cs_fixed > 0: the slice length every rank of the call computed alike
 * (slice_elems); 0: the pipeline's own, from this process's pieces */
static int run_staged_cs(mvx_comm_t *c, const job_t *J, hipStream_t st, long cs_fixed);

int mvxi_run_staged(mvx_comm_t *c, const job_t *J, hipStream_t st)
{
    return run_staged_cs(c, J, st, 0);
}

static int run_staged_cs(mvx_comm_t *c, const job_t *J, hipStream_t st, long cs_fixed)
{
    mvx_work *w = mvxi_work(c);
    stage_job_t S;
    rank_exec_t X[MVX_MAXP];
    size_t need = 0, off[2 * MVX_MAXP], bounce;
    long span = 0, nsl, i, lag;
    int r, rc, pieces = 0;
    mvx_range v[MVX_MAXP + 1];

    if (!w) return MPI_ERR_INTERN;
    memset(&S, 0, sizeof S);
    S.J = J;
    S.R = &w->stage;
    for (r = 0; r < J->nr; r++) {
        const long E = J->P[r].esize;
        int ns = mvxi_send_ranges(&J->P[r], v), nv = mvxi_recv_ranges(&J->P[r], v);
        S.shost[r] = J->skind[r] != MVX_BUF_DEVICE;
        S.rhost[r] = J->rkind[r] != MVX_BUF_DEVICE;
        S.spin[r] = J->skind[r] == MVX_BUF_PINNED;
        S.rpin[r] = J->rkind[r] == MVX_BUF_PINNED;
        S.any_host |= S.shost[r] || S.rhost[r];
        off[2 * r] = need;
        if (S.shost[r]) need = al256(need + (size_t)(J->nsend[r] * E));
        off[2 * r + 1] = need;
        if (S.rhost[r]) need = al256(need + (size_t)(J->nrecv[r] * E));
        pieces += (ns > nv ? ns : nv);
        if (mvxi_plan_span(&J->P[r]) > span) span = mvxi_plan_span(&J->P[r]);
    }
    if ((rc = mvxi_grow(&c->hpool, &c->hpool_bytes, need + 256))) return rc;
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
        if (cs_fixed > 0) cs = cs_fixed;
        S.cs = cs;
        bounce = (size_t)pieces * al256((size_t)(cs * E));
        if (bounce < 4096) bounce = 4096;
    }
    nsl = span > 0 ? (span + S.cs - 1) / S.cs : 0;
    S.single = nsl <= 1;
    if (S.any_host && (rc = stage_init(S.R, bounce))) return rc;
    for (r = 0; r < J->nr; r++) mvxi_plan_slice(&J->P[r], 0, S.cs, &w->slice[0][r]);
    if ((rc = mvxi_job_layout(c, X, J, w->slice[0]))) return rc;   /* slice 0 is the largest */
    lag = mvxi_host_drain_lag();
    for (i = 0; i < nsl + lag; i++) {
        if (i < nsl) {
            mvx_plan *Q = w->slice[i % (STAGE_LAG_MAX + 1)];
            for (r = 0; r < J->nr; r++) {
                mvxi_plan_slice(&J->P[r], i, S.cs, &Q[r]);
                X[r].P = &Q[r];
            }
            if ((rc = stage_in(&S, Q, i, st))) return rc;
            if ((rc = mvxi_exec_group(X, J->t, J->nr, st, NULL))) return rc;
            if ((rc = stage_out(&S, Q, i, st))) return rc;
        }
        if (i >= lag && i - lag < nsl &&
            (rc = stage_drain(&S, w->slice[(i - lag) % (STAGE_LAG_MAX + 1)], i - lag, st)))
            return rc;
    }
    return hipStreamSynchronize(st) == hipSuccess ? MPI_SUCCESS : MPI_ERR_OTHER;
}

/* ---- host buffers at p > 1: HBM mirrors ---------------------------------
 * A rank of the same call may pass device buffers (MPI lets the kind differ
 * per rank), and a device-buffer call moves whole blocks, while the sliced
 * pipeline moves slices: mixed, the paired transfers would differ in size.
 * So by default a host-buffer call of a one-rank-per-process communicator
 * copies its send vector into an HBM mirror, runs the device path on the
 * mirrors -- the same plan, exchange variant and transfers as a device
 * call -- and copies the result out.  Pageable vectors of MIRROR_BOUNCE_MIN
 * bytes and more move in MIRROR_CHUNK chunks through the bounce slots, the
 * copy pool filling slot c while the DMA engines move chunk c - 1; smaller
 * ones take HIP's own pageable copies; page-locked ones (or ranges the
 * registration cache pinned) are DMA'd directly.  The price is the overlap
 * of the two PCIe directions, which only the sliced pipeline has
 * (mvx_comm_set_host_pipeline: every rank's buffers must then be host
 * memory in every call). */
#define MIRROR_CHUNK (16L << 20)
#define MIRROR_BOUNCE_MIN (64L << 20)

static int mirror_bounced(int kind, size_t bytes)
{
    return kind == MVX_BUF_BOUNCE || (kind == MVX_BUF_PAGEABLE && bytes >= (size_t)MIRROR_BOUNCE_MIN);
}

static int mirror_in(stage_res_t *R, char *dev, const char *host, size_t bytes, int kind, hipStream_t st)
{
    size_t o;
    long c = 0;
    if (!bytes) return MPI_SUCCESS;
    if (!mirror_bounced(kind, bytes))
        return hipMemcpyAsync(dev, host, bytes, hipMemcpyHostToDevice, st) == hipSuccess ? MPI_SUCCESS
                                                                                         : MPI_ERR_OTHER;
    for (o = 0; o < bytes; o += MIRROR_CHUNK, c++) {
        const int b = (int)(c % STAGE_NB);
        const size_t n = bytes - o < (size_t)MIRROR_CHUNK ? bytes - o : (size_t)MIRROR_CHUNK;
        /* slot b was last read by the DMA of chunk c - STAGE_NB */
        if (c >= STAGE_NB && hipEventSynchronize(R->ein[b]) != hipSuccess) return MPI_ERR_OTHER;
        mvx_pcopy(R->bin[b], host + o, n);
        if (hipMemcpyAsync(dev + o, R->bin[b], n, hipMemcpyHostToDevice, st) != hipSuccess ||
            hipEventRecord(R->ein[b], st) != hipSuccess)
            return MPI_ERR_OTHER;
    }
    return MPI_SUCCESS;
}

/* returns with the bytes in `host` (the caller's stream synchronised) */
static int mirror_out(stage_res_t *R, char *host, const char *dev, size_t bytes, int kind, hipStream_t st)
{
    size_t o;
    long c, nch, lag;
    if (!bytes) return hipStreamSynchronize(st) == hipSuccess ? MPI_SUCCESS : MPI_ERR_OTHER;
    if (!mirror_bounced(kind, bytes)) {
        if (hipMemcpyAsync(host, dev, bytes, hipMemcpyDeviceToHost, st) != hipSuccess) return MPI_ERR_OTHER;
        return hipStreamSynchronize(st) == hipSuccess ? MPI_SUCCESS : MPI_ERR_OTHER;
    }
    nch = (long)((bytes + MIRROR_CHUNK - 1) / MIRROR_CHUNK);
    lag = mvxi_host_drain_lag();
    for (c = 0; c < nch + lag; c++) {
        if (c < nch) {
            const int b = (int)(c % STAGE_NB);
            o = (size_t)c * MIRROR_CHUNK;
            const size_t n = bytes - o < (size_t)MIRROR_CHUNK ? bytes - o : (size_t)MIRROR_CHUNK;
            if (hipMemcpyAsync(R->bout[b], dev + o, n, hipMemcpyDeviceToHost, st) != hipSuccess ||
                hipEventRecord(R->eout[b], st) != hipSuccess)
                return MPI_ERR_OTHER;
        }
        if (c >= lag) {    /* drain chunk c - lag while the later ones are in flight */
            const long p = c - lag;
            const int b = (int)(p % STAGE_NB);
            o = (size_t)p * MIRROR_CHUNK;
            const size_t n = bytes - o < (size_t)MIRROR_CHUNK ? bytes - o : (size_t)MIRROR_CHUNK;
            if (hipEventSynchronize(R->eout[b]) != hipSuccess) return MPI_ERR_OTHER;
            mvx_pcopy(host + o, R->bout[b], n);
        }
    }
    return hipStreamSynchronize(st) == hipSuccess ? MPI_SUCCESS : MPI_ERR_OTHER;
}

static int run_mirrored(mvx_comm_t *c, const job_t *J, hipStream_t st)
{
    mvx_work *w = mvxi_work(c);
    const long E = J->P[0].esize;
    const size_t sb = (size_t)(J->nsend[0] * E), rb = (size_t)(J->nrecv[0] * E);
    const int sh = J->skind[0] != MVX_BUF_DEVICE, rh = J->rkind[0] != MVX_BUF_DEVICE;
    const size_t roff = sh ? al256(sb) : 0;
    job_t K;
    int rc;
    if (!w) return MPI_ERR_INTERN;
    if ((rc = mvxi_grow(&c->hpool, &c->hpool_bytes, roff + (rh ? al256(rb) : 0) + 256))) return rc;
    if ((sh && mirror_bounced(J->skind[0], sb)) || (rh && mirror_bounced(J->rkind[0], rb)))
        if ((rc = stage_init(&w->stage, MIRROR_CHUNK))) return rc;
    K = *J;
    if (sh) {
        K.send[0] = c->hpool;
        if ((rc = mirror_in(&w->stage, c->hpool, J->send[0], sb, J->skind[0], st))) return rc;
    }
    if (rh) K.recv[0] = c->hpool + roff;
    if ((rc = mvxi_run_device(c, &K, st))) return rc;
    if (rh) return mirror_out(&w->stage, J->recv[0], c->hpool + roff, rb, J->rkind[0], st);
    return hipStreamSynchronize(st) == hipSuccess ? MPI_SUCCESS : MPI_ERR_OTHER;
}

void mvxi_stage_release(stage_res_t *R)
{
    int b;
    if (!R->ready) return;
    for (b = 0; b < STAGE_NB; b++) {
        if (R->bin[b]) hipHostFree(R->bin[b]);
        if (R->bout[b]) hipHostFree(R->bout[b]);
        hipEventDestroy(R->ein[b]);
        hipEventDestroy(R->eout[b]);
        hipEventDestroy(R->ex[b]);
    }
    hipStreamDestroy(R->sh);
    hipStreamDestroy(R->sd);
    memset(R, 0, sizeof *R);
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


/* the kinds of the host spans a packed job copies (the type maps' hull of
 * each host send / recv vector), with the registration cache's holds on
 * them (J->shold / rhold, released by mvxi_job_release); device vectors read
 * MVX_BUF_DEVICE */
static void packed_kinds(job_t *J, const tspan_t *T)
{
    unsigned long *mine[2 * MVX_MAXP];
    int r, nmine = 0;
    for (r = 0; r < J->nr; r++) {
        J->shold[r] = J->rhold[r] = 0;
        J->skind[r] = J->rkind[r] = MVX_BUF_DEVICE;
        if (J->nsend[r] > 0 && !mvxi_is_device_ptr(J->send[r])) {
            J->skind[r] = mvxi_buf_kind_hold(J->send[r] + T->lo, span_bytes(T, J->nsend[r]), &J->shold[r], mine, nmine);
            if (J->shold[r]) mine[nmine++] = &J->shold[r];
        }
        if (J->nrecv[r] > 0 && !mvxi_is_device_ptr(J->recv[r])) {
            J->rkind[r] = mvxi_buf_kind_hold(J->recv[r] + T->lo, span_bytes(T, J->nrecv[r]), &J->rhold[r], mine, nmine);
            if (J->rhold[r]) mine[nmine++] = &J->rhold[r];
        }
    }
    /* a span whose registration was merged into a later one's union and
     * lost with it is asked again (as mvxi_job_kinds does) */
    for (r = 0; r < J->nr; r++) {
        if (J->skind[r] == MVX_BUF_PINNED && !J->shold[r] && mvx_host_pinned(J->send[r] + T->lo) != 1)
            J->skind[r] = mvxi_buf_kind_hold(J->send[r] + T->lo, span_bytes(T, J->nsend[r]), &J->shold[r], NULL, 0);
        if (J->rkind[r] == MVX_BUF_PINNED && !J->rhold[r] && mvx_host_pinned(J->recv[r] + T->lo) != 1)
            J->rkind[r] = mvxi_buf_kind_hold(J->recv[r] + T->lo, span_bytes(T, J->nrecv[r]), &J->rhold[r], NULL, 0);
    }
    J->kinds = 1;
}

static int packed_setup(mvx_comm_t *c, job_t *J, const tspan_t *T, packed_bufs_t *B, hipStream_t st)
{
    mvx_work *w = mvxi_work(c);
    const int dt = J->P[0].dtype;
    size_t need = 0, off[4 * MVX_MAXP];
    int r, rc, bounce = 0;
    if (!w) return MPI_ERR_INTERN;
    packed_kinds(J, T);
    for (r = 0; r < J->nr; r++) {
        const int sh = J->skind[r] != MVX_BUF_DEVICE, rh = J->rkind[r] != MVX_BUF_DEVICE;
        off[4 * r] = need;     need = al256(need + (sh ? span_bytes(T, J->nsend[r]) : 0));
        off[4 * r + 1] = need; need = al256(need + (size_t)(J->nsend[r] * T->size));
        off[4 * r + 2] = need; need = al256(need + (rh ? span_bytes(T, J->nrecv[r]) : 0));
        off[4 * r + 3] = need; need = al256(need + (size_t)(J->nrecv[r] * T->size));
        B->smir[r] = sh ? (char *)1 : NULL;
        B->rmir[r] = rh ? (char *)1 : NULL;
        bounce |= (sh && mirror_bounced(J->skind[r], span_bytes(T, J->nsend[r]))) ||
                  (rh && mirror_bounced(J->rkind[r], span_bytes(T, J->nrecv[r])));
    }
    if ((rc = mvxi_grow(&c->hpool, &c->hpool_bytes, need + 256))) return rc;
    if (bounce && (rc = stage_init(&w->stage, MIRROR_CHUNK))) return rc;
    for (r = 0; r < J->nr; r++) {
        B->psend[r] = c->hpool + off[4 * r + 1];
        B->precv[r] = c->hpool + off[4 * r + 3];
        B->sorg[r] = J->send[r];
        B->rorg[r] = J->recv[r];
        if (B->smir[r]) {      /* the send span into HBM (through the CPU where HIP may not copy it) */
            B->smir[r] = c->hpool + off[4 * r];
            if ((rc = mirror_in(&w->stage, B->smir[r], J->send[r] + T->lo, span_bytes(T, J->nsend[r]),
                                J->skind[r], st)))
                return rc;
            B->sorg[r] = B->smir[r] - T->lo;
        }
        if (B->rmir[r]) {      /* the recv span too: its bytes outside the type map go back as they were */
            B->rmir[r] = c->hpool + off[4 * r + 2];
            if ((rc = mirror_in(&w->stage, B->rmir[r], J->recv[r] + T->lo, span_bytes(T, J->nrecv[r]),
                                J->rkind[r], st)))
                return rc;
            B->rorg[r] = B->rmir[r] - T->lo;
        }
        if (J->nsend[r] > 0 && (rc = mvx_type_pack(dt, B->sorg[r], B->psend[r], (size_t)J->nsend[r], st)))
            return rc;
    }
    return MPI_SUCCESS;
}

static int packed_finish(mvx_comm_t *c, const job_t *J, const tspan_t *T, packed_bufs_t *B, hipStream_t st,
                         int sync)
{
    mvx_work *w = mvxi_work(c);
    const int dt = J->P[0].dtype;
    int r, rc;
    if (!w) return MPI_ERR_INTERN;
    for (r = 0; r < J->nr; r++) {
        if (J->nrecv[r] <= 0) continue;
        if ((rc = mvx_type_unpack(dt, B->precv[r], B->rorg[r], (size_t)J->nrecv[r], st))) return rc;
        if (B->rmir[r] && (rc = mirror_out(&w->stage, J->recv[r] + T->lo, B->rmir[r], span_bytes(T, J->nrecv[r]),
                                           J->rkind[r], st)))
            return rc;
    }
    return (sync && hipStreamSynchronize(st) != hipSuccess) ? MPI_ERR_OTHER : MPI_SUCCESS;
}

/* host vectors of a packed job (its spans are host memory) */
int mvxi_job_packed_host(const job_t *J)
{
    int r, host = 0;
    for (r = 0; r < J->nr; r++)
        host |= (J->nsend[r] > 0 && !mvxi_is_device_ptr(J->send[r])) ||
                (J->nrecv[r] > 0 && !mvxi_is_device_ptr(J->recv[r]));
    return host;
}

int mvxi_run_job_packed(mvx_comm_t *c, job_t *J, hipStream_t st, int blocking)
{
    mvx_work *w = mvxi_work(c);
    job_t *K;
    packed_bufs_t *B;
    tspan_t T;
    int r, rc, host;
    if (!w) return MPI_ERR_INTERN;
    K = &w->pk_job;
    B = &w->pk_bufs;
    if ((rc = type_span(J->P[0].dtype, &T))) return rc;
    host = mvxi_job_packed_host(J);
    if (host && !blocking) return MPI_ERR_BUFFER;
    if ((rc = packed_setup(c, J, &T, B, st))) return rc;
    *K = *J;
    for (r = 0; r < J->nr; r++) {
        K->send[r] = B->psend[r];
        K->recv[r] = B->precv[r];
    }
    if ((rc = mvxi_run_device(c, K, st))) return rc;
    return packed_finish(c, J, &T, B, st, blocking || host);
}

/* dst = src, bytes of any kinds (MPIR_intra_Scan's self copy of a contiguous
 * type when its op is undefined): device to device stream-ordered; with a
 * host side the host side's kind is asked of the registration cache (held
 * until the copy is done) and the copy is synchronous -- through the CPU
 * where HIP may not copy the memory (MVX_BUF_BOUNCE) */
int mvxi_copy_any(mvx_comm_t *c, void *dst, const void *src, size_t bytes, hipStream_t st, int sync)
{
    mvx_work *w = mvxi_work(c);
    const int sdev = mvxi_is_device_ptr(src), ddev = mvxi_is_device_ptr(dst);
    unsigned long hs = 0, hd = 0;
    int ks = MVX_BUF_DEVICE, kd = MVX_BUF_DEVICE, rc = MPI_SUCCESS;
    if (!bytes) return MPI_SUCCESS;
    if (sdev && ddev) {
        if (hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, st) != hipSuccess) return MPI_ERR_OTHER;
        return (sync && hipStreamSynchronize(st) != hipSuccess) ? MPI_ERR_OTHER : MPI_SUCCESS;
    }
    if (!w) return MPI_ERR_INTERN;
    if (!sdev) ks = mvxi_buf_kind_hold(src, bytes, &hs, NULL, 0);
    if (!ddev) {
        unsigned long *mine[1] = {&hs};
        kd = mvxi_buf_kind_hold(dst, bytes, &hd, mine, hs ? 1 : 0);
    }
    if (!sdev && !ddev) {                       /* host to host: the CPU, after the stream */
        if (hipStreamSynchronize(st) != hipSuccess) rc = MPI_ERR_OTHER;
        else memmove(dst, src, bytes);
    } else if ((ks == MVX_BUF_BOUNCE || kd == MVX_BUF_BOUNCE) && (rc = stage_init(&w->stage, MIRROR_CHUNK))) {
        ;
    } else if (!sdev) {
        rc = mirror_in(&w->stage, (char *)dst, (const char *)src, bytes, ks, st);
        if (!rc && hipStreamSynchronize(st) != hipSuccess) rc = MPI_ERR_OTHER;
    } else {
        rc = mirror_out(&w->stage, (char *)dst, (const char *)src, bytes, kd, st);   /* synchronises */
    }
    if (rc && hipDeviceSynchronize() != hipSuccess) (void)hipGetLastError();
    mvxi_buf_release(hs);
    mvxi_buf_release(hd);
    return rc;
}

/* recvbuf = sendbuf over the type map (MPIR_intra_Scan's self copy when its
 * op is undefined, intra_scan.c:100-106): through the packed form */
int mvxi_typed_copy(mvx_comm_t *c, int dt, long n, const char *send, char *recv, hipStream_t st, int sync)
{
    mvx_work *w = mvxi_work(c);
    job_t *K;
    packed_bufs_t *B;
    mvx_plan *P0;
    tspan_t T;
    int rc;
    if (!w) return MPI_ERR_INTERN;
    K = &w->tc_job; B = &w->tc_bufs; P0 = &w->tc_plan;
    memset(P0, 0, sizeof *P0);
    P0->dtype = dt;
    K->nr = 1; K->P = P0; K->send[0] = send; K->recv[0] = recv; K->nsend[0] = n; K->nrecv[0] = n;
    K->kinds = 0;
    if ((rc = type_span(dt, &T)) || (rc = packed_setup(c, K, &T, B, st))) {
        mvxi_job_release(K, rc ? rc : MPI_ERR_OTHER);
        return rc;
    }
    if (n > 0 && hipMemcpyAsync(B->precv[0], B->psend[0], (size_t)(n * T.size), hipMemcpyDeviceToDevice, st) !=
                     hipSuccess)
        rc = MPI_ERR_OTHER;
    if (!rc) rc = packed_finish(c, K, &T, B, st, sync || B->smir[0] || B->rmir[0]);
    mvxi_job_release(K, rc);
    return rc;
}

/* ---- the slice schedule: large calls at p > 1, any buffer kind ----------
 * MPI lets every rank of a call pass device or host memory.  A host-buffer
 * rank overlaps its PCIe copies with the collective only by running the
 * collective in slices, and RCCL pairs a rank's transfers with its peers'
 * only if they are the same messages -- so the slices cannot depend on the
 * kinds.  A blocking call at p > 1 whose vector (count x size: the same on
 * every rank) is at least MVX_SLICE_MIN_MIB (default 64) runs in slices on
 * every rank, of MVX_SLICE_MIB (default 32) of the vector each, from
 * quantities every rank holds alike (count, p, type size): slice i of every
 * block is its elements [i cs, (i + 1) cs) (mvxi_plan_slice), run as phases
 * A, B, C (P2P) on the call's stream.  A device-buffer rank issues its
 * slices back to back; a host-buffer rank wraps each slice in its H2D (one
 * stream) and D2H (another), so both PCIe directions and the collective
 * overlap (run_staged_cs).  The bits are the unsliced plan's (every slice
 * keeps every block boundary).  Stream-ordered calls (mvx_*_async, device
 * buffers by contract) and smaller calls keep the unsliced schedule.  A
 * caller that has agreed every rank's kinds says so per call
 * (mvx_comm_set_call_kinds): all device -- the unsliced device path, its
 * exchange variants and graphs; all host -- the sliced pipeline at any
 * size. */
static long env_mib(const char *name, long dflt)
{
    const char *v = getenv(name);
    return (v && atol(v) > 0 ? atol(v) : dflt) << 20;
}

/* elements per slice of every block, or 0: the call runs unsliced */
long mvxi_slice_elems(const mvx_plan *P)
{
    const long E = P->esize, N = P->count, p = P->p;
    const long vbytes = N * E, min = env_mib("MVX_SLICE_MIN_MIB", 64), per = env_mib("MVX_SLICE_MIB", 32);
    long g = E, h = 256, m, nsl, blk, cs;
    if (p < 2 || E <= 0 || N <= 0 || vbytes < min) return 0;
    nsl = (vbytes + per - 1) / per;
    if (nsl < 2) return 0;
    while (h) { const long t = g % h; g = h; h = t; }      /* gcd(E, 256) */
    m = 256 / g;                                            /* slices start 256-byte aligned */
    /* the longest range the algorithm moves: the whole vector (binomial
     * Reduce, Scan, recursive doubling, the SMP leader's fold) or a block of
     * about N / p (Rabenseifner, halving, pairwise); the algorithm is a
     * function of (coll, count, p, op kind, knobs), the same on every rank */
    switch (P->alg) {
    case MVX_ALG_RECDBL: case MVX_ALG_BINOMIAL: case MVX_ALG_SCAN_RECDBL: case MVX_ALG_SMP_LEADER:
        blk = N;
        break;
    default:
        blk = (N + p - 1) / p;
    }
    cs = (blk + nsl - 1) / nsl;
    cs = (cs + m - 1) / m * m;
    return cs;
}

int mvxi_run_job(mvx_comm_t *c, job_t *J, hipStream_t st, int blocking)
{
    int rc, host;
    long cs;
    const int kinds = blocking ? c->call_kinds : MVX_KINDS_UNKNOWN;
    if (J->P[0].packed) return mvxi_run_job_packed(c, J, st, blocking);
    if (kinds != MVX_KINDS_UNKNOWN && J->nr == 1) {
        /* The caller agreed every rank's kinds (mvx_comm_set_call_kinds).
         * Every rank runs the schedule the hint names, whatever its own
         * buffers, so a rank whose buffers contradict the hint still pairs
         * with its peers: under HOST the slices (a device buffer is used in
         * place), under DEVICE the unsliced device schedule on HBM mirrors
         * of this rank's host buffers. */
        host = mvxi_job_kinds(J);
        if (kinds == MVX_KINDS_HOST) return mvxi_run_staged(c, J, st);
        if (host) return run_mirrored(c, J, st);
    } else if (blocking && J->nr == 1 && !c->local && (cs = mvxi_slice_elems(&J->P[0])) > 0) {
        mvxi_job_kinds(J);
        return run_staged_cs(c, J, st, cs);
    } else if (mvxi_job_kinds(J)) {
        if (!blocking) return MPI_ERR_BUFFER;
        if (J->nr == 1 && J->P[0].p > 1 && !c->host_sliced) return run_mirrored(c, J, st);
        return mvxi_run_staged(c, J, st);
    }
    rc = mvxi_run_device(c, J, st);
    if (rc == MPI_SUCCESS && blocking && hipStreamSynchronize(st) != hipSuccess) rc = MPI_ERR_OTHER;
    return rc;
}
