/*
 * mvx_combine.c -- phase B of a plan: one rank's combine program in the
 * reference's order.  Predefined ops on <= 8 leaves are one kernel launch
 * (mvx_op_program, libmvx_hip.so); wider programs run as groups of 8 with the
 * same association; user functions get the reference's operand roles
 * (host MPI_User_functions through pinned scratch, device functions in
 * HBM); datatypes with holes are unpacked to the extent layout the op sees.
 * Reference: the (*uop) calls of intra_fns_new.c (e.g. 5505-5512, 5681-5699)
 * and global_ops.c.
 */
#include <string.h>

#include "mvx_internal.h"

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
    const MPI_Datatype uh = mvxi_user_handle(dt);
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
    if (o->dop) return o->dop(in, inout, (size_t)n, mvxi_user_handle(dt), st) ? MPI_ERR_OTHER : MPI_SUCCESS;
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
    const mvx_op_t *o = mvxi_user_op(P->op);
    const long n = P->c_cnt, E = P->esize;
    const size_t slot = (region + 255) & ~(size_t)255;
    const int dev = o && o->dop;
    const hipMemcpyKind in_kind = dev ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
    char *y[MVX_MAXK] = {0}, *base;
    int q, l, s, e, rc;
    if (!o) return MPI_ERR_OP;
    if (dev) rc = mvxi_grow(&c->upool, &c->upool_bytes, slot * (size_t)P->k * 2);
    else rc = mvxi_grow_host(&c->uhost, &c->uhost_bytes, slot * (size_t)P->k * 2);
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
int mvxi_wide_temps(const mvx_plan *P)
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
        wide = mvxi_wide_temps(&Q);
    }
    /* a slot covers the type map of n elements and the op's n * extent */
    a = lo < 0 ? lo : 0;
    b = (n - 1) * ext + hi;
    if (b < n * ext) b = n * ext;
    slot = al256((size_t)(b - a) + SLOT_STAGGER);
    for (q = 0; q < P->k; q++) nf += fold[q] != NULL;
    if ((rc = mvxi_grow(&c->xpool, &c->xpool_bytes, slot * (size_t)(P->k + nf + 1 + wide)))) return rc;
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

int mvxi_combine(mvx_comm_t *c, const mvx_plan *P, const char *const *leafp, void *dst,
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
