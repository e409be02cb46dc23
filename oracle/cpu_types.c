/*
 * cpu_types.c -- TEST INFRASTRUCTURE: the reference's derived-datatype
 * constructors restated on the CPU (bounds and type maps), for the oracle's
 * collectives over derived types.  Never linked by the product.
 *
 *   orc_type_contiguous  src/pt2pt/type_contig.c:52-187
 *   orc_type_vector      src/pt2pt/type_vec.c:44-110  (-> hvector / contiguous)
 *   orc_type_hvector     src/pt2pt/type_hvec.c:55-175
 *   orc_type_indexed     src/pt2pt/type_ind.c:74-134  (-> hindexed)
 *   orc_type_hindexed    src/pt2pt/type_hind.c:57-200
 *   orc_type_struct      src/pt2pt/type_struct.c:106-330 (ALIGNMENT_VALUE 0:
 *                        the x86-64 struct layout is "largest member",
 *                        util/structlayout.c)
 *   orc_type_commit      src/pt2pt/type_commit.c:41-143
 *   orc_type_free        src/pt2pt/type_free.c:60-105 with the reference
 *                        counts of MPIR_Type_dup / MPIR_Type_free
 *                        (type_util.c:29-130, 226-236)
 * Basic types as MPIR_Setup_base_datatype (initdte.c:281-310: lb 0, ub = size,
 * align = size, real_lb = real_ub = 0) and the pair structs of
 * MPIR_Init_dtes (169-222: struct {value, int} with an MPI_UB at sizeof).
 *
 * Pinning: the bounds these give are checked against the known answers of
 * the reference's own datatype tests (examples/test/pt2pt typeub.c,
 * typeub2.c, typeub3.c, typelb.c, structlb.c), tests/golden/
 * type_known_answers.json.
 */
#include <stdlib.h>
#include <string.h>
#include "oracle.h"

#define DT_BASE 256
#define DT_MAX 256
#define MAXMAP (1L << 22)

enum { KB = 0, KC, KHV, KHI, KS, KUB, KLB };

typedef struct {
    int used, ref, kind, old, count, is_contig, no_old, has_lb, has_ub;
    long align, extent, size, lb, ub, real_lb, real_ub;
    long nmap, *moff, *mlen;       /* one element's type map, merged */
    int nmem, *mtype, *mblk;       /* struct members (commit's test) */
    long *midx;
} dtype_t;

static dtype_t g_t[DT_MAX];

static dtype_t *derived(int h)
{
    int i = h - DT_BASE;
    return (i >= 0 && i < DT_MAX && g_t[i].used) ? &g_t[i] : NULL;
}

/* a view of a basic handle; returns 0 or 323 */
static int basic(int h, dtype_t *t, long *off2, long *len2)
{
    int e, s;
    memset(t, 0, sizeof *t);
    t->moff = off2; t->mlen = len2;
    if (h == 15 || h == 16) { t->kind = h == 16 ? KUB : KLB; t->is_contig = 1; return 0; }
    if (orc_dtype_info(h, &e, &s)) return 3 | (5 << 6);
    t->kind = KB; t->old = h; t->count = 1; t->is_contig = 1;
    t->extent = t->ub = e; t->size = s; t->align = s;
    t->nmap = 1; off2[0] = 0; len2[0] = s;
    switch (h) {
    case 17: t->has_ub = 1; t->align = 4; break;                       /* FLOAT_INT {0:4, 4:4} */
    case 18: case 19: t->has_ub = 1; t->align = 8; t->nmap = 2;        /* {0:8, 8:4} */
        len2[0] = 8; off2[1] = 8; len2[1] = 4; t->is_contig = 0; break;
    case 20: t->has_ub = 1; t->align = 4; t->nmap = 2;                 /* SHORT_INT {0:2, 4:4} */
        len2[0] = 2; off2[1] = 4; len2[1] = 4; t->is_contig = 0; break;
    case 22: t->has_ub = 1; t->align = 16; t->nmap = 2;                /* LONG_DOUBLE_INT {0:16, 16:4} */
        len2[0] = 16; off2[1] = 16; len2[1] = 4; t->is_contig = 0; break;
    case 21: t->align = 4; t->old = 6; t->count = 2; break;            /* 2INT = contig(2, INT) */
    case 23: t->align = 4; break;
    case 24: t->align = 8; break;
    /* the Fortran pairs, contiguous(2, old) (initfutil.c:263, 286, 318-323) */
    case 29: t->align = 4; t->old = 28; t->count = 2; break;           /* 2INTEGER */
    case 30: t->align = 4; t->old = 23; t->count = 2; break;           /* 2COMPLEX */
    case 31: t->align = 8; t->old = 24; t->count = 2; break;           /* 2DOUBLE_COMPLEX */
    case 32: t->align = 4; t->old = 10; t->count = 2; break;           /* 2REAL */
    case 33: t->align = 8; t->old = 11; t->count = 2; break;           /* 2DOUBLE_PRECISION */
    default: break;
    }
    return 0;
}

typedef struct { dtype_t t; long o[2], l[2]; } view_t;

static const dtype_t *get(int h, view_t *v)
{
    dtype_t *d = derived(h);
    if (d) return d;
    return basic(h, &v->t, v->o, v->l) ? NULL : &v->t;
}

static int map_add(dtype_t *n, long off, long len)
{
    if (n->nmap && n->moff[n->nmap - 1] + n->mlen[n->nmap - 1] == off) { n->mlen[n->nmap - 1] += len; return 0; }
    if (n->nmap >= MAXMAP) return -1;
    if ((n->nmap & (n->nmap - 1)) == 0) {   /* grow at powers of two */
        long cap = n->nmap ? 2 * n->nmap : 1;
        n->moff = (long *)realloc(n->moff, sizeof(long) * (size_t)cap);
        n->mlen = (long *)realloc(n->mlen, sizeof(long) * (size_t)cap);
    }
    n->moff[n->nmap] = off;
    n->mlen[n->nmap] = len;
    n->nmap++;
    return 0;
}

static int map_copies(dtype_t *n, const dtype_t *o, long base, long reps)
{
    long j, b;
    for (j = 0; j < reps; j++)
        for (b = 0; b < o->nmap; b++)
            if (map_add(n, base + j * o->extent + o->moff[b], o->mlen[b])) return -1;
    return 0;
}

/* MPIR_Type_dup, type_util.c:29-34 */
static void retain(int h)
{
    dtype_t *d = derived(h);
    if (d) d->ref++;
}

/* MPIR_Type_free, type_util.c:56-130: the last reference frees the type and
   the references it holds (old type :97-99, struct members :226-236) */
static void release(int h)
{
    dtype_t *t = derived(h);
    int i, kind, old, nmem, *mtype;
    if (!t) return;
    if (t->ref > 1) { t->ref--; return; }
    kind = t->kind; old = t->old; nmem = t->nmem; mtype = t->mtype;
    free(t->moff); free(t->mlen); free(t->mblk); free(t->midx);
    memset(t, 0, sizeof *t);
    if (kind == KS) {
        for (i = 0; i < nmem; i++) release(mtype[i]);
    } else {
        release(old);
    }
    free(mtype);
}

static int store(dtype_t *n, int *newtype)
{
    int i, j;
    for (i = 0; i < DT_MAX; i++) {
        if (g_t[i].used) continue;
        n->used = 1;
        n->ref = 1;
        if (n->kind == KS) {
            for (j = 0; j < n->nmem; j++) retain(n->mtype[j]);
        } else {
            retain(n->old);
        }
        g_t[i] = *n;
        *newtype = DT_BASE + i;
        return 0;
    }
    return 16;
}

int orc_type_contiguous(int count, int oldtype, int *newtype)
{
    view_t v, w;
    const dtype_t *o = get(oldtype, &v), *ot;
    dtype_t n;
    int has_old;
    if (!o) return 3 | (5 << 6);
    if (o->kind == KUB || o->kind == KLB) return count < 0 ? 2 : 3;
    if (count < 0) return 2;
    memset(&n, 0, sizeof n);
    n.kind = KC;
    if (count == 0) {               /* the empty type, 82-116 */
        n.old = oldtype; n.is_contig = 1; n.align = 4;
        return store(&n, newtype);
    }
    /* MPI_2INT and the Fortran pairs have an old type, as derived contiguous
       types do */
    has_old = (o->kind == KB && o->count == 2) || (derived(oldtype) && o->kind == KC && !o->no_old);
    if (o->is_contig && has_old) {  /* 139-142 */
        ot = get(o->old, &w);
        n.old = o->old; n.count = count * o->count; n.is_contig = 1;
    } else {                        /* 143-146 */
        ot = o;
        n.old = oldtype; n.count = count; n.is_contig = o->is_contig;
    }
    n.align = o->align;
    n.lb = ot->lb; n.has_lb = ot->has_lb;
    n.extent = (long)n.count * ot->extent;
    if (ot->has_ub) { n.ub = ot->ub + (long)(count - 1) * ot->extent; n.has_ub = 1; }
    else n.ub = n.lb + n.extent;
    n.size = (long)n.count * ot->size;
    n.real_lb = ot->real_lb;
    n.real_ub = (long)n.count * (ot->real_ub - ot->real_lb) + ot->real_lb;
    if (map_copies(&n, ot, 0, n.count)) return 16;
    return store(&n, newtype);
}

int orc_type_hvector(int count, int blocklen, long stride, int oldtype, int *newtype)
{
    view_t v;
    const dtype_t *o = get(oldtype, &v);
    dtype_t n;
    long i;
    if (!o) return 3 | (5 << 6);
    if (count < 0) return 2;
    if (blocklen < 0) return 12;
    if (o->kind == KUB || o->kind == KLB) return 3;
    if ((long)count * blocklen == 0) return orc_type_contiguous(0, 6, newtype);
    if ((long)blocklen * o->extent == stride || count == 1)
        return orc_type_contiguous(count * blocklen, oldtype, newtype);
    memset(&n, 0, sizeof n);
    n.kind = KHV; n.old = oldtype; n.count = count; n.align = o->align;
    n.has_ub = o->has_ub; n.has_lb = o->has_lb;
    if (o->has_ub) n.ub = stride > 0 ? o->ub + (count - 1) * stride + (long)(blocklen - 1) * o->extent : o->ub;
    if (o->has_lb) n.lb = stride < 0 ? o->lb + (count - 1) * stride + (long)(blocklen - 1) * o->extent : o->lb;
    n.extent = (count - 1) * stride + (long)blocklen * o->extent;
    if (n.extent < 0) {
        if (!o->has_ub) n.ub = o->lb;
        if (!o->has_lb) n.lb = n.ub + n.extent;
        n.real_ub = o->real_lb;
        n.real_lb = n.real_ub + (count - 1) * stride + blocklen * (o->real_ub - o->real_lb);
    } else {
        if (!o->has_lb) n.lb = o->lb;
        if (!o->has_ub) n.ub = n.lb + n.extent;
        n.real_lb = o->real_lb;
        n.real_ub = n.real_lb + (count - 1) * stride + blocklen * (o->real_ub - o->real_lb);
    }
    n.extent = n.ub - n.lb;
    n.size = (long)count * blocklen * o->size;
    for (i = 0; i < count; i++)
        if (map_copies(&n, o, i * stride, blocklen)) return 16;
    return store(&n, newtype);
}

int orc_type_vector(int count, int blocklen, int stride, int oldtype, int *newtype)
{
    view_t v;
    const dtype_t *o = get(oldtype, &v);
    if (!o) return 3 | (5 << 6);
    if (count < 0) return 2;
    if (blocklen < 0) return 12;
    if (o->kind == KUB || o->kind == KLB) return 3;
    if (blocklen == stride || count == 1) return orc_type_contiguous(count * blocklen, oldtype, newtype);
    return orc_type_hvector(count, blocklen, (long)stride * o->extent, oldtype, newtype);
}

int orc_type_hindexed(int count, const int *blocklens, const long *indices, int oldtype, int *newtype)
{
    view_t v;
    const dtype_t *o = get(oldtype, &v);
    dtype_t n;
    long total = 0, low, high, real_lb, real_ub, ubm = 0, lbm = 0;
    int i, ubf = 0, lbf = 0;
    if (!o) return 3 | (5 << 6);
    if (count < 0) return 2;
    if (o->kind == KUB || o->kind == KLB) return 3;
    for (i = 0; i < count; i++) {
        if (blocklens[i] < 0) return 12;
        total += blocklens[i];
    }
    if (total == 0) return orc_type_contiguous(0, 6, newtype);
    memset(&n, 0, sizeof n);
    n.kind = KHI; n.old = oldtype; n.count = count; n.align = o->align;
    n.has_ub = o->has_ub; n.has_lb = o->has_lb;
    low = indices[0];
    high = indices[0] + (long)blocklens[0] * o->extent;
    real_lb = indices[0];
    real_ub = real_lb;
    for (i = 0; i < count; i++) {
        long ub = indices[i] + (long)blocklens[i] * o->extent, lb = indices[i];
        if (ub > lb) { if (high < ub) high = ub; if (low > lb) low = lb; }
        else { if (high < lb) high = lb; if (low > ub) low = ub; }
        if (indices[i] < real_lb) real_lb = indices[i];
        if (indices[i] + blocklens[i] * (o->real_ub - o->real_lb) > real_ub)
            real_ub = indices[i] + blocklens[i] * (o->real_ub - o->real_lb);
        if (o->has_ub) {
            long t = o->ub + indices[i] + (long)(blocklens[i] - 1) * o->extent;
            if (!ubf || ubm < t) ubm = t;
            ubf = 1;
        }
        if (o->has_lb) {
            long t = o->lb + indices[i];
            if (!lbf || lbm > t) lbm = t;
            lbf = 1;
        }
    }
    if (o->real_lb != 0) {
        low += o->real_lb; high += o->real_lb; real_lb += o->real_lb;
        real_ub = o->real_lb;    /* type_hind.c's `real_ub =+ ...` */
    }
    n.lb = o->has_lb ? lbm : low;
    n.ub = o->has_ub ? ubm : high;
    n.extent = n.ub - n.lb;
    n.size = total * o->size;
    n.real_lb = real_lb; n.real_ub = real_ub;
    for (i = 0; i < count; i++)
        if (map_copies(&n, o, indices[i], blocklens[i])) return 16;
    return store(&n, newtype);
}

int orc_type_indexed(int count, const int *blocklens, const int *indices, int oldtype, int *newtype)
{
    view_t v;
    const dtype_t *o = get(oldtype, &v);
    long total = 0, *h;
    int i, rc;
    if (!o) return 3 | (5 << 6);
    if (count < 0) return 2;
    if (o->kind == KUB || o->kind == KLB) return 3;
    for (i = 0; i < count; i++) {
        total += blocklens[i];
        if (blocklens[i] < 0) return -(12 | (31 << 6));    /* setmsg ARG_ARRAY_VAL */
    }
    if (total == 0) return orc_type_contiguous(0, 6, newtype);
    h = (long *)malloc(sizeof(long) * (size_t)count);
    for (i = 0; i < count; i++) h[i] = (long)indices[i] * o->extent;
    rc = orc_type_hindexed(count, blocklens, h, oldtype, newtype);
    free(h);
    return rc;
}

int orc_type_struct(int count, const int *blocklens, const long *indices, const int *types, int *newtype)
{
    dtype_t n;
    long total = 0, high = 0, low = 0, real_ub = 0, real_lb = 0, ubm = 0, lbm = 0;
    int i, hi_i = 0, lo_i = 0, re_i = 0, ubf = 0, lbf = 0;
    if (count < 0) return -(2 | (1 << 6));
    if (count == 0) return orc_type_contiguous(0, 6, newtype);
    for (i = 0; i < count; i++) {
        total += blocklens[i];
        if (blocklens[i] < 0) return -(12 | (31 << 6));
        if (types[i] == 0) return -(3 | (13 << 6));
    }
    if (total == 0) return orc_type_contiguous(0, 6, newtype);
    memset(&n, 0, sizeof n);
    n.kind = KS; n.count = count; n.align = 1; n.old = types[0];
    n.nmem = count;
    n.mtype = (int *)malloc(sizeof(int) * (size_t)count);
    n.mblk = (int *)malloc(sizeof(int) * (size_t)count);
    n.midx = (long *)malloc(sizeof(long) * (size_t)count);
    for (i = 0; i < count; i++) {
        view_t v;
        const dtype_t *o = get(types[i], &v);
        if (!o) return 3 | (5 << 6);
        n.mtype[i] = types[i]; n.mblk[i] = blocklens[i]; n.midx[i] = indices[i];
        if (n.align < o->align) n.align = o->align;
        if (o->kind == KUB) {
            if (!ubf || indices[i] > ubm) ubm = indices[i];
            ubf = 1;
        } else if (o->kind == KLB) {
            if (!lbf || indices[i] < lbm) lbm = indices[i];
            lbf = 1;
        } else {
            long lb, ub;
            if (!re_i) { re_i = 1; real_lb = o->real_lb; real_ub = o->real_ub; }
            else { if (o->real_lb < real_lb) real_lb = o->real_lb; if (o->real_ub > real_ub) real_ub = o->real_ub; }
            if (o->has_ub) {
                long t = o->ub + indices[i] + (long)(blocklens[i] - 1) * o->extent;
                if (ubm < t || !ubf) ubm = t;
                ubf = 1;
            }
            if (o->has_lb) {
                if (!lbf || lbm > o->lb + indices[i]) lbm = o->lb + indices[i];
                lbf = 1;
            }
            lb = indices[i] + o->lb;
            ub = lb + (long)blocklens[i] * o->extent;
            if (!hi_i) { high = ub; hi_i = 1; } else if (ub > high) high = ub;
            if (!lo_i) { low = lb; lo_i = 1; } else if (lb < low) low = lb;
            if (ub > lb) { if (high < ub) high = ub; if (low > lb) low = lb; }
            else { if (high < lb) high = lb; if (low > ub) low = ub; }
            if (map_copies(&n, o, indices[i], blocklens[i])) return 16;
        }
        n.size += (long)blocklens[i] * o->size;
    }
    if (lbf) { n.lb = lbm; n.has_lb = 1; } else n.lb = lo_i ? low : 0;
    if (ubf) { n.ub = ubm; n.has_ub = 1; } else n.ub = hi_i ? high : 0;
    n.extent = n.ub - n.lb;
    n.real_ub = real_ub; n.real_lb = real_lb;
    if (!lbf && !ubf && n.extent % n.align > 0) {
        n.ub += n.align - n.extent % n.align;
        n.extent = n.ub - n.lb;
    }
    return store(&n, newtype);
}

int orc_type_commit(int h)
{
    dtype_t *t = derived(h);
    long offset;
    int j, contig;
    view_t v;
    if (!t) return get(h, &v) ? 0 : (3 | (5 << 6));
    if (t->is_contig || t->size != t->extent || t->kind != KS) return 0;
    offset = t->midx[0];
    contig = offset == 0;
    for (j = 0; contig && j < t->count - 1; j++) {
        const dtype_t *o = get(t->mtype[j], &v);
        if (!o->is_contig) { contig = 0; break; }
        if (offset + o->extent * t->mblk[j] != t->midx[j + 1]) { contig = 0; break; }
        offset += o->extent * t->mblk[j];
    }
    if (!get(t->mtype[t->count - 1], &v)->is_contig) contig = 0;
    if (contig) { t->is_contig = 1; t->no_old = 1; }
    return 0;
}

int orc_type_free(int *h)
{
    if (!derived(*h)) return 3 | (5 << 6);
    release(*h);
    *h = 0;
    return 0;
}

int orc_type_bounds(int h, long *lb, long *ub, long *extent, long *size)
{
    view_t v;
    const dtype_t *t = get(h, &v);
    if (!t) return 3 | (5 << 6);
    if (lb) *lb = t->lb;
    if (ub) *ub = t->ub;
    if (extent) *extent = t->extent;
    if (size) *size = t->size;
    return 0;
}

int orc_derived_info(int h, int *kind, int *old, int *count, long *extent, long *size)
{
    const dtype_t *t = derived(h);
    if (!t) return 3;
    if (kind) *kind = t->kind;
    if (old) *old = t->old;
    if (count) *count = t->count;
    if (extent) *extent = t->extent;
    if (size) *size = t->size;
    return 0;
}

int orc_type_parts(int dtype, int *old, int *count)
{
    const dtype_t *t = derived(dtype);
    if (!t) return 3;
    *old = t->old;
    *count = t->count;
    return 0;
}

/* n elements of a derived type, type-map bytes only (a message) */
int orc_type_copy(void *dst, const void *src, long n, int h)
{
    const dtype_t *t = derived(h);
    long i, b;
    if (!t) return 3;
    for (i = 0; i < n; i++)
        for (b = 0; b < t->nmap; b++)
            memcpy((char *)dst + i * t->extent + t->moff[b], (const char *)src + i * t->extent + t->moff[b],
                   (size_t)t->mlen[b]);
    return 0;
}

/* one element's type map: number of blocks, and block i */
long orc_type_nblocks(int h)
{
    const dtype_t *t = derived(h);
    return t ? t->nmap : -1;
}

int orc_type_block(int h, long i, long *off, long *len)
{
    const dtype_t *t = derived(h);
    if (!t || i < 0 || i >= t->nmap) return 3;
    *off = t->moff[i];
    *len = t->mlen[i];
    return 0;
}
