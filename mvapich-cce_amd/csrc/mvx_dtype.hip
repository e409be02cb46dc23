// mvx_dtype.hip -- the datatype engine of the reduction path (libmvx_hip.so).
//
// The reference's reductions take any datatype: MPI_Sendrecv moves the type
// map between ranks (pack on send, unpack into tmp buffers laid out by
// extent, intra_fns_new.c:5505-5512), and the op sees count elements at the
// type's extent.  This file keeps a handle table of derived types with the
// reference's bounds (lb / ub / extent / size, exactly as src/pt2pt computes
// them, markers and struct alignment included), the flattened type map of
// each, and the device pack / unpack kernels the executor moves non-dense
// types with.
//
//   MPI_Type_contiguous  type_contig.c:52-187
//   MPI_Type_vector      type_vec.c:44-110 (-> hvector, or contiguous)
//   MPI_Type_hvector     type_hvec.c:55-175
//   MPI_Type_indexed     type_ind.c:74-134 (-> hindexed)
//   MPI_Type_hindexed    type_hind.c:57-200
//   MPI_Type_struct      type_struct.c:106-330 (ALIGNMENT_VALUE 0: the x86-64
//                        "largest member" struct layout, util/structlayout.c)
//   MPI_Type_commit      type_commit.c:41-143 (dense structs become is_contig)
//   MPI_Type_free        type_free.c:60-105, with the reference counts of
//                        MPIR_Type_dup / MPIR_Type_free (type_util.c:29-130):
//                        a type holds a reference on every derived type it
//                        was built from, so freeing a member first leaves it
//                        in place (handle and all) until its last user goes
// Basic and pair handles are as MPIR_Init_dtes registers them
// (initdte.c:106-280, MPIR_Setup_base_datatype 281-310).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "mvx_mpi.h"
#include "mvx_hip.h"
#include "mvx_dtype.h"

namespace mvx {
namespace dt {

struct Blk { long off, len; };

struct Type {
    int used, ref, kind, old, count, is_contig, has_lb, has_ub, no_old;
    long align, extent, size, lb, ub, real_lb, real_ub;
    // STRUCT members (type_commit's contiguity test)
    std::vector<long> indices;
    std::vector<int> blocklens, types;
    std::vector<Blk> map;       // one element's type map, in order, merged
    int dense;
    // the map on the device, split into pieces of <= 64 bytes
    void *dmap;
    long dmap_n;
    // the map as W-byte units (W = 16, 8, 4, 2, 1: index 0 .. 4): each
    // unit's offset in the element, in packed order; 0: not built; -1: the
    // map does not split into W-byte units (2 and 1 serve the tile kernels
    // only)
    int *dunits[5];
    long units[5];
    // after the units in dunits[w] (W <= 8): the offsets of the G = 16 / W
    // units of a 16-byte packed chunk, per chunk phase -- tabP[w] phases
    // (a period of tabP chunks holds whole elements), 0: no table
    long tabP[5];
    // the tile kernels' LDS swizzle for W (swz_pick): 0 none, else s -- bits
    // [s, s + 3) of a tile byte address XORed into its 16-byte slot index
    int swz[5];
    // whole-word unpack (merge_ok): 0 not decided, 1 yes, -1 no; the map's
    // reach [mlo, mhi) around the element origin
    int merge;
    long mlo, mhi;
};

static Type g_t[MVX_TYPE_DERIVED_MAX];
static const long kMaxBlocks = 1L << 24;

static Type *slot(int h)
{
    const int i = h - MVX_TYPE_DERIVED_BASE;
    if (i < 0 || i >= MVX_TYPE_DERIVED_MAX || !g_t[i].used) return nullptr;
    return &g_t[i];
}

static void reset(Type &t)
{
    if (t.dmap) (void)hipFree(t.dmap);
    for (int w = 0; w < 5; ++w)
        if (t.dunits[w]) (void)hipFree(t.dunits[w]);
    t = Type();
}

// The basic and pair handles (initdte.c): fills a view, false if unknown.
static bool basic(int h, Type &t)
{
    t = Type();
    t.kind = K_BASIC;
    t.old = h;
    t.count = 1;
    t.is_contig = 1;
    t.dense = 1;
    auto base = [&](long s) { t.extent = t.size = t.ub = s; t.align = s; t.map.push_back({0, s}); };
    // the pair structs: {value, int loc} with an MPI_UB at sizeof (initdte.c:169-222)
    auto pair = [&](long vs, long loc_off, long ext, long al, int contig) {
        t.extent = t.ub = ext; t.size = vs + 4; t.align = al; t.has_ub = 1; t.is_contig = contig;
        if (loc_off == vs) t.map.push_back({0, vs + 4});
        else { t.map.push_back({0, vs}); t.map.push_back({loc_off, 4}); }
    };
    switch (h) {
    case MPI_CHAR: case MPI_UNSIGNED_CHAR: case MPI_BYTE: case MPI_PACKED: base(1); return true;
    case MPI_SHORT: case MPI_UNSIGNED_SHORT: base(2); return true;
    case MPI_INT: case MPI_UNSIGNED: case MPI_FLOAT: base(4); return true;
    case MPI_LONG: case MPI_UNSIGNED_LONG: case MPI_DOUBLE: case MPI_LONG_LONG_INT: base(8); return true;
    case MPI_LONG_DOUBLE: base(16); return true;
    case MPI_COMPLEX: base(8); t.align = 4; return true;
    case MPI_DOUBLE_COMPLEX: base(16); t.align = 8; return true;
    case MPI_2INT: base(8); t.align = 4; t.old = MPI_INT; t.count = 2; return true;   // contig(2, INT), :167
    // the Fortran types (initfutil.c:238-323; gfortran: 4-byte INTEGER /
    // REAL / LOGICAL, 8-byte DOUBLE PRECISION); the pairs are contiguous(2, x)
    // over the old type initfutil.c names, with that type's alignment
    case MPI_INTEGER: case MPI_REAL: case MPI_LOGICAL: base(4); return true;
    case MPI_DOUBLE_PRECISION: base(8); return true;
    case MPI_2INTEGER: base(8); t.align = 4; t.old = MPI_INTEGER; t.count = 2; return true;      // :323
    case MPI_2REAL: base(8); t.align = 4; t.old = MPI_FLOAT; t.count = 2; return true;           // :263
    case MPI_2DOUBLE_PRECISION: base(16); t.align = 8; t.old = MPI_DOUBLE; t.count = 2; return true;   // :286
    case MPI_2COMPLEX: base(16); t.align = 4; t.old = MPI_COMPLEX; t.count = 2; return true;     // :318
    case MPI_2DOUBLE_COMPLEX: base(32); t.align = 8; t.old = MPI_DOUBLE_COMPLEX; t.count = 2; return true;
    case MPI_FLOAT_INT: pair(4, 4, 8, 4, 1); return true;
    case MPI_DOUBLE_INT: pair(8, 8, 16, 8, 0); return true;
    case MPI_LONG_INT: pair(8, 8, 16, 8, 0); return true;
    case MPI_SHORT_INT: pair(2, 4, 8, 4, 0); return true;
    case MPI_LONG_DOUBLE_INT: pair(16, 16, 32, 16, 0); return true;
    case MPI_UB: t.kind = K_UB; t.old = h; return true;     // size 0 (MPIR_Setup_base_datatype)
    case MPI_LB: t.kind = K_LB; t.old = h; return true;
    default: return false;
    }
}

// a handle's record: the stored derived type, or a view of a basic one
static const Type *get(int h, Type &view)
{
    if (const Type *t = slot(h)) return t;
    return basic(h, view) ? &view : nullptr;
}

// append `n` copies of old's map at `base + j * old.extent`
static bool add_copies(std::vector<Blk> &m, const Type &old, long base, long n)
{
    if ((long)m.size() + n * (long)old.map.size() > kMaxBlocks) return false;
    for (long j = 0; j < n; ++j)
        for (const Blk &b : old.map) {
            const long off = base + j * old.extent + b.off;
            if (!m.empty() && m.back().off + m.back().len == off) m.back().len += b.len;
            else m.push_back({off, b.len});
        }
    return true;
}

// dense: one element is `extent` whole bytes from its origin (lb 0); the
// basic pair structs count as whole elements (their padding travels, as
// the plain path has always moved them)
static int is_dense(const Type &t)
{
    if (t.lb != 0) return 0;
    if (t.map.size() == 1 && t.map[0].off == 0 && t.map[0].len == t.extent) return 1;
    return 0;
}

// MPIR_Type_dup (type_util.c:29-34): one more reference on a derived type
// (basic and pair handles are permanent and never freed)
static void retain(int h)
{
    if (Type *t = slot(h)) ++t->ref;
}

// MPIR_Type_free (type_util.c:56-130): drop one reference; the last one
// frees the slot and, in turn, the references it held -- the old type
// (default case, :97-99) or every struct member (MPIR_Free_struct_internals,
// :226-236)
static void release(int h)
{
    Type *t = slot(h);
    if (!t) return;
    if (t->ref > 1) { --t->ref; return; }
    const int kind = t->kind, old = t->old;
    const std::vector<int> members = t->types;
    reset(*t);
    if (kind == K_STRUCT) {
        for (int m : members) release(m);
    } else {
        release(old);
    }
}

// a new type with one reference (the caller's), holding a reference on
// each derived type it was built from: its old type (type_contig.c:107,
// 140, 144; type_hvec.c:110; type_hind.c:115) or its members
// (type_struct.c:208)
static int store(Type &n, int *newtype)
{
    for (int i = 0; i < MVX_TYPE_DERIVED_MAX; ++i) {
        if (g_t[i].used) continue;
        n.used = 1;
        n.ref = 1;
        if (n.kind == K_STRUCT) {
            for (int m : n.types) retain(m);
        } else {
            retain(n.old);
        }
        g_t[i] = n;
        *newtype = MVX_TYPE_DERIVED_BASE + i;
        return MPI_SUCCESS;
    }
    return MPI_ERR_INTERN;
}

// type_contig.c:52-187
static int contiguous(int count, int oldtype, int *newtype)
{
    Type ov, iv;
    if (!newtype) return MPI_ERR_ARG;
    const Type *o = get(oldtype, ov);
    if (!o) return MVX_ERR_TYPE_NULL;                               // 66-67
    if (o->kind == K_UB || o->kind == K_LB) return count < 0 ? MPI_ERR_COUNT : MPI_ERR_TYPE;   // 69-71
    if (count < 0) return MPI_ERR_COUNT;
    Type n = Type();
    n.kind = K_CONTIG;
    if (count == 0) {                                              // 82-116: empty type
        n.old = oldtype; n.count = 0; n.is_contig = 1; n.align = 4;
        n.dense = 1;
        return store(n, newtype);
    }
    // 139-146: a contiguous old type that has an old type itself (MPI_2INT
    // and the Fortran pairs, which MPIR_Type_contiguous built; a derived
    // contiguous type) is flattened to that old type
    const bool has_old = (o->kind == K_BASIC && o->count == 2) ||
                         (slot(oldtype) && o->kind == K_CONTIG && !o->no_old);
    const Type *ot = o;
    if (o->is_contig && has_old) {
        ot = get(o->old, iv);
        n.old = o->old;
        n.count = count * o->count;
        n.is_contig = 1;
    } else {
        n.old = oldtype;
        n.count = count;
        n.is_contig = o->is_contig;
    }
    n.align = o->align;
    n.lb = ot->lb;                                                 // 149-150
    n.has_lb = ot->has_lb;
    n.extent = (long)n.count * ot->extent;                         // 151
    if (ot->has_ub) { n.ub = ot->ub + (long)(count - 1) * ot->extent; n.has_ub = 1; }   // 160-164
    else n.ub = n.lb + n.extent;
    n.size = (long)n.count * ot->size;                             // 169
    n.real_lb = ot->real_lb;
    n.real_ub = (long)n.count * (ot->real_ub - ot->real_lb) + ot->real_lb;
    if (!add_copies(n.map, *ot, 0, n.count)) return MPI_ERR_INTERN;
    n.dense = (ot->dense && n.lb == 0 && ot->lb == 0) ? 1 : is_dense(n);
    return store(n, newtype);
}

static int old_checks(const Type *o, int count)
{
    if (!o) return MVX_ERR_TYPE_NULL;                   // MPIR_TEST_DTYPE
    if (count < 0) return MPI_ERR_COUNT;
    return MPI_SUCCESS;
}

// type_hvec.c:55-175
static int hvector(int count, int blocklen, long stride, int oldtype, int *newtype)
{
    Type ov;
    const Type *o = get(oldtype, ov);
    int rc = old_checks(o, count);
    if (rc) return rc;
    if (blocklen < 0) return MPI_ERR_ARG;
    if (o->kind == K_UB || o->kind == K_LB) return MPI_ERR_TYPE;
    if ((long)count * blocklen == 0) return contiguous(0, MPI_INT, newtype);     // 87-90
    if ((long)blocklen * o->extent == stride || count == 1)                      // 93-97
        return contiguous(count * blocklen, oldtype, newtype);
    Type n = Type();
    n.kind = K_HVECTOR;
    n.old = oldtype;
    n.count = count;
    n.align = o->align;
    n.has_ub = o->has_ub;
    n.has_lb = o->has_lb;
    if (o->has_ub) n.ub = stride > 0 ? o->ub + (long)(count - 1) * stride + (long)(blocklen - 1) * o->extent : o->ub;
    if (o->has_lb) n.lb = stride < 0 ? o->lb + (long)(count - 1) * stride + (long)(blocklen - 1) * o->extent : o->lb;
    n.extent = (long)(count - 1) * stride + (long)blocklen * o->extent;          // 136
    if (n.extent < 0) {
        if (!o->has_ub) n.ub = o->lb;
        if (!o->has_lb) n.lb = n.ub + n.extent;
        n.real_ub = o->real_lb;
        n.real_lb = n.real_ub + (long)(count - 1) * stride + (long)blocklen * (o->real_ub - o->real_lb);
    } else {
        if (!o->has_lb) n.lb = o->lb;
        if (!o->has_ub) n.ub = n.lb + n.extent;
        n.real_lb = o->real_lb;
        n.real_ub = n.real_lb + (long)(count - 1) * stride + (long)blocklen * (o->real_ub - o->real_lb);
    }
    n.extent = n.ub - n.lb;                                                      // 158
    n.size = (long)count * blocklen * o->size;
    for (long i = 0; i < count; ++i)
        if (!add_copies(n.map, *o, i * stride, blocklen)) return MPI_ERR_INTERN;
    n.dense = is_dense(n);
    return store(n, newtype);
}

// type_vec.c:44-110
static int vector(int count, int blocklen, int stride, int oldtype, int *newtype)
{
    Type ov;
    const Type *o = get(oldtype, ov);
    int rc = old_checks(o, count);
    if (rc) return rc;
    if (blocklen < 0) return MPI_ERR_ARG;
    if (o->kind == K_UB || o->kind == K_LB) return MPI_ERR_TYPE;
    if (blocklen == stride || count == 1) return contiguous(count * blocklen, oldtype, newtype);
    return hvector(count, blocklen, (long)stride * o->extent, oldtype, newtype);
}

// type_hind.c:57-200
static int hindexed(int count, const int *blocklens, const long *indices, int oldtype, int *newtype)
{
    Type ov;
    const Type *o = get(oldtype, ov);
    int rc = old_checks(o, count);
    if (rc) return rc;
    if (o->kind == K_UB || o->kind == K_LB) return MPI_ERR_TYPE;
    long total = 0;
    for (int i = 0; i < count; ++i) {
        if (blocklens[i] < 0) return MPI_ERR_ARG;                                // 95-99
        total += blocklens[i];
    }
    if (total == 0) return contiguous(0, MPI_INT, newtype);
    Type n = Type();
    n.kind = K_HINDEXED;
    n.old = oldtype;
    n.count = count;
    n.align = o->align;
    n.has_ub = o->has_ub;
    n.has_lb = o->has_lb;
    long low = indices[0], high = indices[0] + (long)blocklens[0] * o->extent;
    long real_lb = indices[0], real_ub = real_lb, ub_marker = 0, lb_marker = 0;
    int ub_found = 0, lb_found = 0;
    for (int i = 0; i < count; ++i) {                                            // 136-170
        const long ub = indices[i] + (long)blocklens[i] * o->extent, lb = indices[i];
        if (ub > lb) { if (high < ub) high = ub; if (low > lb) low = lb; }
        else { if (high < lb) high = lb; if (low > ub) low = ub; }
        if (indices[i] < real_lb) real_lb = indices[i];
        if (indices[i] + (long)blocklens[i] * (o->real_ub - o->real_lb) > real_ub)
            real_ub = indices[i] + (long)blocklens[i] * (o->real_ub - o->real_lb);
        if (o->has_ub) {
            const long t = o->ub + indices[i] + (long)(blocklens[i] - 1) * o->extent;
            if (!ub_found || ub_marker < t) ub_marker = t;
            ub_found = 1;
        }
        if (o->has_lb) {
            const long t = o->lb + indices[i];
            if (!lb_found || lb_marker > t) lb_marker = t;
            lb_found = 1;
        }
    }
    if (o->real_lb != 0) {                                                       // 173-178
        low += o->real_lb;
        high += o->real_lb;
        real_lb += o->real_lb;
        real_ub = +o->real_lb;      // the reference's `real_ub =+ ...` (an assignment)
    }
    n.lb = o->has_lb ? lb_marker : low;
    n.ub = o->has_ub ? ub_marker : high;
    n.extent = n.ub - n.lb;
    n.size = total * o->size;
    n.real_lb = real_lb;
    n.real_ub = real_ub;
    for (int i = 0; i < count; ++i)
        if (!add_copies(n.map, *o, indices[i], blocklens[i])) return MPI_ERR_INTERN;
    n.dense = is_dense(n);
    return store(n, newtype);
}

// type_ind.c:74-134: displacements in old extents -> hindexed
static int indexed(int count, const int *blocklens, const int *indices, int oldtype, int *newtype)
{
    Type ov;
    const Type *o = get(oldtype, ov);
    int rc = old_checks(o, count);
    if (rc) return rc;
    if (o->kind == K_UB || o->kind == K_LB) return MPI_ERR_TYPE;
    long total = 0;
    for (int i = 0; i < count; ++i) {
        total += blocklens[i];
        if (blocklens[i] < 0) return MVX_SETMSG(MPI_ERR_ARG, MVX_ERR_KIND_ARG_ARRAY_VAL);   // 107-112
    }
    if (total == 0) return contiguous(0, MPI_INT, newtype);
    std::vector<long> h(count > 0 ? count : 1);
    for (int i = 0; i < count; ++i) h[i] = (long)indices[i] * o->extent;
    return hindexed(count, blocklens, h.data(), oldtype, newtype);
}

// type_struct.c:106-330
static int structure(int count, const int *blocklens, const long *indices, const int *types, int *newtype)
{
    if (count < 0) return MVX_SETMSG(MPI_ERR_COUNT, 1);                           // 124-129
    if (count == 0) return contiguous(0, MPI_INT, newtype);
    long total = 0;
    for (int i = 0; i < count; ++i) {                                            // 137-156
        total += blocklens[i];
        if (blocklens[i] < 0) return MVX_SETMSG(MPI_ERR_ARG, MVX_ERR_KIND_ARG_ARRAY_VAL);
        if (types[i] == MPI_DATATYPE_NULL) return MVX_SETMSG(MPI_ERR_TYPE, MVX_ERR_KIND_TYPE_ARRAY_NULL);
    }
    if (total == 0) return contiguous(0, MPI_INT, newtype);
    Type n = Type();
    n.kind = K_STRUCT;
    n.count = count;
    n.align = 1;
    n.old = types[0];
    long high = 0, low = 0, real_ub = 0, real_lb = 0, ub_marker = 0, lb_marker = 0;
    int high_init = 0, low_init = 0, real_init = 0, ub_found = 0, lb_found = 0;
    for (int i = 0; i < count; ++i) {                                            // 204-297
        Type ov;
        const Type *o = get(types[i], ov);
        if (!o) return MVX_ERR_TYPE_NULL;
        n.indices.push_back(indices[i]);
        n.blocklens.push_back(blocklens[i]);
        n.types.push_back(types[i]);
        if (n.align < o->align) n.align = o->align;
        if (o->kind == K_UB) {
            if (!ub_found || indices[i] > ub_marker) ub_marker = indices[i];
            ub_found = 1;
        } else if (o->kind == K_LB) {
            if (!lb_found || indices[i] < lb_marker) lb_marker = indices[i];
            lb_found = 1;
        } else {
            if (!real_init) { real_init = 1; real_lb = o->real_lb; real_ub = o->real_ub; }
            else { if (o->real_lb < real_lb) real_lb = o->real_lb; if (o->real_ub > real_ub) real_ub = o->real_ub; }
            if (o->has_ub) {
                const long t = o->ub + indices[i] + (long)(blocklens[i] - 1) * o->extent;
                if (ub_marker < t || !ub_found) ub_marker = t;
                ub_found = 1;
            }
            if (o->has_lb) {
                if (!lb_found || lb_marker > o->lb + indices[i]) lb_marker = o->lb + indices[i];
                lb_found = 1;
            }
            const long lb = indices[i] + o->lb, ub = lb + (long)blocklens[i] * o->extent;
            if (!high_init) { high = ub; high_init = 1; } else if (ub > high) high = ub;
            if (!low_init) { low = lb; low_init = 1; } else if (lb < low) low = lb;
            if (ub > lb) { if (high < ub) high = ub; if (low > lb) low = lb; }
            else { if (high < lb) high = lb; if (low > ub) low = ub; }
            if (!add_copies(n.map, *o, indices[i], blocklens[i])) return MPI_ERR_INTERN;
        }
        n.size += (long)blocklens[i] * o->size;
    }
    if (lb_found) { n.lb = lb_marker; n.has_lb = 1; } else n.lb = low_init ? low : 0;
    if (ub_found) { n.ub = ub_marker; n.has_ub = 1; } else n.ub = high_init ? high : 0;
    n.extent = n.ub - n.lb;
    n.real_ub = real_ub;
    n.real_lb = real_lb;
    if (!lb_found && !ub_found) {                                                // 316-326
        const long eps = n.extent % n.align;
        if (eps > 0) { n.ub += n.align - eps; n.extent = n.ub - n.lb; }
    }
    n.dense = is_dense(n);
    return store(n, newtype);
}

// type_commit.c:55-112: a struct whose members are contiguous and back to
// back from offset 0, with size == extent, is marked contiguous (and loses
// its old type, so a later MPI_Type_contiguous does not flatten it)
static int commit(int h)
{
    Type *t = slot(h);
    Type tmp;
    if (!t) return basic(h, tmp) ? MPI_SUCCESS : MVX_ERR_TYPE_NULL;
    if (t->is_contig || t->size != t->extent || t->kind != K_STRUCT) return MPI_SUCCESS;
    long offset = t->indices[0];
    int contig = offset == 0;
    for (int j = 0; contig && j < t->count - 1; ++j) {
        Type v;
        const Type *o = get(t->types[j], v);
        if (!o->is_contig) { contig = 0; break; }
        if (offset + o->extent * (long)t->blocklens[j] != t->indices[j + 1]) { contig = 0; break; }
        offset += o->extent * (long)t->blocklens[j];
    }
    {
        Type v;
        const Type *o = get(t->types[t->count - 1], v);
        if (!o->is_contig) contig = 0;
    }
    if (contig) { t->is_contig = 1; t->no_old = 1; }
    return MPI_SUCCESS;
}

bool info(int h, Info *out)
{
    Type v;
    const Type *t = get(h, v);
    if (!t) return false;
    out->kind = t->kind;
    out->old = t->old;
    out->count = t->count;
    out->is_contig = t->is_contig;
    out->dense = t->dense;
    out->extent = t->extent;
    out->size = t->size;
    out->lb = t->lb;
    out->ub = t->ub;
    out->span_lo = out->span_hi = 0;
    if (!t->map.empty()) {
        long lo = t->map[0].off, hi = t->map[0].off + t->map[0].len;
        for (const Blk &b : t->map) {
            if (b.off < lo) lo = b.off;
            if (b.off + b.len > hi) hi = b.off + b.len;
        }
        out->span_lo = lo;
        out->span_hi = hi;
    }
    return true;
}

// ---- pack / unpack --------------------------------------------------------
// One work item = one piece (<= 64 bytes) of one element's type map.
// Consecutive threads take consecutive pieces, so the packed side is
// written contiguously; each thread copies with the widest access its
// addresses allow.

struct DBlk { long off, poff; int len, pad; };

template <bool PACK>
__global__ void __launch_bounds__(256)
k_pack(const char *__restrict__ src, char *__restrict__ dst, const DBlk *__restrict__ map, long nblk,
       long count, long extent, long size)
{
    const long items = count * nblk;
    for (long t = (long)blockIdx.x * 256 + threadIdx.x; t < items; t += (long)gridDim.x * 256) {
        const long i = t / nblk;
        const DBlk m = map[t - i * nblk];
        const char *s = PACK ? src + i * extent + m.off : src + i * size + m.poff;
        char *d = PACK ? dst + i * size + m.poff : dst + i * extent + m.off;
        const uintptr_t a = (uintptr_t)s | (uintptr_t)d | (uintptr_t)m.len;
        if ((a & 15) == 0) {
            for (int b = 0; b < m.len; b += 16) *(uint4 *)(d + b) = *(const uint4 *)(s + b);
        } else if ((a & 3) == 0) {
            for (int b = 0; b < m.len; b += 4) *(uint32_t *)(d + b) = *(const uint32_t *)(s + b);
        } else {
            for (int b = 0; b < m.len; ++b) d[b] = s[b];
        }
    }
}

// Units of W bytes (tools/bench_pack.py: the piece kernel above reached
// 0.25-0.39 of HBM peak on every shape, 64 KiB of the packed stream per
// wave spread over 64 pieces and a 64-bit division per piece).  Lane l of
// the grid takes packed units l, l + T, l + 2T, ... (T the grid's threads):
// one wave reads or writes 64 consecutive units of the packed stream, and on
// the extent side the units of one block are consecutive too.  The unit's
// (element, unit-in-element) pair advances by the grid stride's (D, R) with
// no division after the first; U units per lane are in flight at once.
typedef uint32_t pu32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t pu32x4 __attribute__((ext_vector_type(4)));
template <int W> struct UnitT;
template <> struct UnitT<1> { typedef uint8_t t; };
template <> struct UnitT<2> { typedef uint16_t t; };
template <> struct UnitT<4> { typedef uint32_t t; };
template <> struct UnitT<8> { typedef pu32x2 t; };
template <> struct UnitT<16> { typedef pu32x4 t; };

#define UNITS_LDS 2048   // unit tables this small are read from LDS
#define CHUNK_TAB_MAX 2048   // chunk tables (Type::tabP) up to this many entries

template <bool PACK, int W, int U, bool LDS>
__global__ void __launch_bounds__(256)
k_pack_units(const char *__restrict__ src, char *__restrict__ dst, const int *__restrict__ uoff, long upe,
             long count, long extent, long D, long R)
{
    typedef typename UnitT<W>::t V;
    __shared__ int s_uoff[LDS ? UNITS_LDS : 1];
    if constexpr (LDS) {
        for (int u = threadIdx.x; u < (int)upe; u += 256) s_uoff[u] = uoff[u];
        __syncthreads();
    }
    const long T = (long)gridDim.x * 256;
    const long N = count * upe;
    const long DX = D * extent;                   // the element offset's advance per grid stride
    long q = (long)blockIdx.x * 256 + threadIdx.x;
    long i = q / upe, j = q - i * upe;
    long ix = i * extent;                         // i * extent, carried
    while (q < N) {
        // (a flag per unit, not a null destination: a pointer that may be
        // null was addressed through flat stores, each waiting for every load)
        V v[U];
        long to[U];
        bool ok[U];
#pragma unroll
        for (int k = 0; k < U; ++k) {
            ok[k] = q < N;
            to[k] = 0;
            if (ok[k]) {
                const long e = ix + (LDS ? s_uoff[j] : uoff[j]);
                const char *from = PACK ? src + e : src + q * W;
                to[k] = PACK ? q * W : e;
                v[k] = __builtin_nontemporal_load((const V *)from);
            }
            q += T;
            ix += DX;
            j += R;
            if (j >= upe) { j -= upe; ix += extent; }
        }
#pragma unroll
        for (int k = 0; k < U; ++k)
            if (ok[k]) __builtin_nontemporal_store(v[k], (V *)(dst + to[k]));
    }
}

// LDS bank conflicts of the tile kernels' unit accesses, modelled
// (MI355X_MICROARCH.md LDS: 1-, 2- and 4-byte reads and every write bank
// (a / 4) mod 32 over 32-lane groups, 8-byte reads mod 64): lane l of a group
// takes chunk l, units G l .. G l + G - 1 of the stream, so when an element's
// units repeat every 128 or 256 bytes of the extent layout, lanes a few
// apart hit one bank (struct {char; hole; int}: 7-way, every other float:
// 8-way).  Swizzle candidates s = 7, 8, 9 (tile byte a lives at
// a ^ (((a >> s) & 7) << 4): 16-byte slots permuted within 128-byte rows,
// so whole 16-byte words stay whole) against none, averaged over a few
// group starts and element offsets in the tile; the best if it saves a
// fifth of the extra cycles, else 0.
static int swz_pick(const std::vector<int> &u, long upe, long ext, int W)
{
    const int G = 16 / W, banks = W == 8 ? 64 : 32;
    const int cand[4] = {0, 7, 8, 9};
    const long starts[4] = {0, 13, 32, 77}, offs[3] = {0, 5, 10};
    double cost[4] = {0, 0, 0, 0};
    if (ext <= 0 || ext > 4096 || upe <= 0) return 0;
    for (int ci = 0; ci < 4; ++ci)
        for (long st : starts)
            for (long e0 : offs)
                for (int g = 0; g < G; ++g) {
                    long dw[32];
                    int per[64] = {0}, worst = 1;
                    for (int l = 0; l < 32; ++l) {
                        const long q = (st + l) * G + g, e = q / upe, j = q % upe;
                        long a = e * ext + e0 + u[(size_t)j] + 4096;    // (offsets may be negative)
                        if (cand[ci]) a ^= ((a >> cand[ci]) & 7) << 4;
                        dw[l] = a / 4;
                    }
                    std::sort(dw, dw + 32);                        // distinct dwords per bank
                    for (int l = 0; l < 32; ++l)
                        if (!l || dw[l] != dw[l - 1]) {
                            const int c = ++per[dw[l] % banks];
                            if (c > worst) worst = c;
                        }
                    cost[ci] += worst - 1;
                }
    int best = 0;
    for (int ci = 1; ci < 4; ++ci)
        if (cost[ci] < cost[best]) best = ci;
    return best && cost[best] <= 0.8 * cost[0] ? cand[best] : 0;
}

// the unit table for W (index wi), built once per type; false if the map
// does not split into W-byte units
static bool unit_table(Type &t, int W, int wi)
{
    if (t.units[wi] < 0) return false;
    if (t.dunits[wi]) return true;
    std::vector<int> u;
    bool ok = t.extent > 0 && t.extent % W == 0 && t.size % W == 0 && t.size / W <= (1L << 22);
    for (size_t b = 0; ok && b < t.map.size(); ++b) {
        const Blk &m = t.map[b];
        if (((m.off % W) + W) % W || m.len % W || m.off < INT32_MIN || m.off + m.len > INT32_MAX) { ok = false; break; }
        for (long o = 0; o < m.len; o += W) u.push_back((int)(m.off + o));
    }
    if (!ok || u.empty()) { t.units[wi] = -1; return false; }
    const long upe = (long)u.size();
    t.tabP[wi] = 0;
    if (W <= 8) {
        // chunk c, unit g: unit q = c G + g of the stream; with c = k P + p,
        // its element is k EPP + (p G + g) / upe and its offset in that
        // element u[(p G + g) % upe] (EPP = P G / upe elements per period)
        const long G = 16 / W;
        long g = upe, m = G;
        while (m) { const long r = g % m; g = m; m = r; }
        const long P = upe / g;
        if (P * G <= CHUNK_TAB_MAX && (P * G / upe + 1) * t.extent < INT32_MAX / 2) {
            for (long q = 0; q < P * G; ++q) u.push_back((int)((q / upe) * t.extent + u[(size_t)(q % upe)]));
            t.tabP[wi] = P;
        }
    }
    t.swz[wi] = W <= 8 ? swz_pick(u, upe, t.extent, W) : 0;
    if (hipMalloc(&t.dunits[wi], u.size() * sizeof(int)) != hipSuccess) {
        t.dunits[wi] = nullptr;
        t.units[wi] = -1;
        return false;
    }
    if (hipMemcpy(t.dunits[wi], u.data(), u.size() * sizeof(int), hipMemcpyHostToDevice) != hipSuccess) {
        (void)hipFree(t.dunits[wi]);
        t.dunits[wi] = nullptr;
        t.units[wi] = -1;
        return false;
    }
    t.units[wi] = upe;
    return true;
}

template <bool PACK, int W>
static int launch_units(const Type &t, int wi, const void *src, void *dst, long count, hipStream_t st)
{
    constexpr int U = 4;
    const long upe = t.units[wi], N = count * upe;
    long blocks = (N + 256L * U - 1) / (256L * U);
    if (blocks > 65536) blocks = 65536;
    if (blocks < 1) blocks = 1;
    const long T = blocks * 256;
    if (upe <= UNITS_LDS)
        hipLaunchKernelGGL((k_pack_units<PACK, W, U, true>), dim3((unsigned)blocks), dim3(256), 0, st,
                           (const char *)src, (char *)dst, (const int *)t.dunits[wi], upe, count, t.extent, T / upe,
                           T % upe);
    else
        hipLaunchKernelGGL((k_pack_units<PACK, W, U, false>), dim3((unsigned)blocks), dim3(256), 0, st,
                           (const char *)src, (char *)dst, (const int *)t.dunits[wi], upe, count, t.extent, T / upe,
                           T % upe);
    return hipGetLastError() == hipSuccess ? MPI_SUCCESS : MPI_ERR_OTHER;
}

// ---- unpack by whole words ------------------------------------------------
// The unit kernel's unpack stores W bytes per unit: where the type map
// leaves holes inside a 64-byte DRAM sector, every such store is a partial
// write the memory must merge with the sector's old bytes.  This variant
// merges on the CU instead: a workgroup owns a 16-byte-aligned tile of the
// destination, loads it whole into LDS, writes the tile's units (read from
// the packed stream, contiguous per tile) over it in LDS, and stores the
// tile back whole -- full-line reads and writes only.  The hole bytes go
// back as they were read, so this is for destinations no one else writes
// meanwhile (MVX_UNPACK_MERGE=0 keeps the byte-exact stores).  Words that
// reach outside the hull of the whole buffer's type maps (its first and
// last) are never written whole: their units are stored directly.
#define MERGE_TILE 8192              // destination bytes per workgroup (LDS)
#define MERGE_UNITS_LDS 2048

template <int W> __device__ inline typename UnitT<W>::t unit_of(const pu32x4 &v, int g);
template <> __device__ inline uint32_t unit_of<4>(const pu32x4 &v, int g) { return v[g]; }
template <> __device__ inline pu32x2 unit_of<8>(const pu32x4 &v, int g)
{
    pu32x2 r;
    r.x = v[2 * g];
    r.y = v[2 * g + 1];
    return r;
}
template <> __device__ inline pu32x4 unit_of<16>(const pu32x4 &v, int) { return v; }
template <> __device__ inline uint16_t unit_of<2>(const pu32x4 &v, int g)
{
    return (uint16_t)(v[g >> 1] >> (16 * (g & 1)));
}
template <> __device__ inline uint8_t unit_of<1>(const pu32x4 &v, int g)
{
    return (uint8_t)(v[g >> 2] >> (8 * (g & 3)));
}

// the LDS byte address of tile byte a under the swizzle (Type::swz)
template <bool SWZ> __device__ inline int lds_at(int a, int s) { return SWZ ? a ^ (((a >> s) & 7) << 4) : a; }

// unit g (W bytes) of a 16-byte chunk being assembled
template <int W> __device__ inline void set_unit(pu32x4 &v, int g, typename UnitT<W>::t x);
template <> __device__ inline void set_unit<8>(pu32x4 &v, int g, pu32x2 x)
{
    v[2 * g] = x.x;
    v[2 * g + 1] = x.y;
}
template <> __device__ inline void set_unit<16>(pu32x4 &v, int, pu32x4 x) { v = x; }
template <> __device__ inline void set_unit<4>(pu32x4 &v, int g, uint32_t x) { v[g] = x; }
template <> __device__ inline void set_unit<2>(pu32x4 &v, int g, uint16_t x)
{
    const int s = 16 * (g & 1);
    v[g >> 1] = (v[g >> 1] & ~(0xffffu << s)) | ((uint32_t)x << s);
}
template <> __device__ inline void set_unit<1>(pu32x4 &v, int g, uint8_t x)
{
    const int s = 8 * (g & 3);
    v[g >> 2] = (v[g >> 2] & ~(0xffu << s)) | ((uint32_t)x << s);
}

// The unit offsets come from LDS (LDSU, up to MERGE_UNITS_LDS units per
// element) or from global memory: a template argument, not a run-time
// select -- a select between the two made the compiler address both through
// flat loads and stores in the inner loop.  Units outside the tile go to a
// trash word past its end (a select on the LDS address, no branch), and the
// hull's two edge words are stored byte by byte, so every unit of the tile
// is one LDS store.
template <int W, int TILE, bool LDSU, bool SWZ, bool TAB>
__global__ void __launch_bounds__(256)
k_unpack_merge(const char *__restrict__ packed, char *__restrict__ dst, const int *__restrict__ uoff, long upe,
               long n, long ext, long lo, long hi, uintptr_t a0, uintptr_t h0, uintptr_t h1, int swz, long tabP)
{
    typedef typename UnitT<W>::t V;
    __shared__ pu32x4 s_tile[TILE / 16 + 1];            // + the trash word
    __shared__ __attribute__((aligned(16))) int s_uoff[LDSU || TAB ? MERGE_UNITS_LDS : 1];
    if (TAB)                                            // the chunk table (k_pack_tiles)
        for (int u = threadIdx.x; u < (int)(tabP * (16 / W)); u += 256) s_uoff[u] = uoff[upe + u];
    else if (LDSU)
        for (int u = threadIdx.x; u < (int)upe; u += 256) s_uoff[u] = uoff[u];
    const uintptr_t t0 = a0 + (uintptr_t)blockIdx.x * TILE;                // this tile's first word
    const uintptr_t tend = t0 + TILE < ((h1 + 15) & ~(uintptr_t)15) ? t0 + TILE
                                                                           : ((h1 + 15) & ~(uintptr_t)15);
    const int nw = (int)((tend - t0) / 16);
    for (int w = threadIdx.x; w < nw; w += 256)
        *(pu32x4 *)((char *)s_tile + lds_at<SWZ>(16 * w, swz)) =
            __builtin_nontemporal_load((const pu32x4 *)(t0 + 16 * (uintptr_t)w));
    __syncthreads();
    // the elements whose maps reach into [t0, tend): relative to dst
    const long a = (long)(t0 - (uintptr_t)dst), b = (long)(tend - (uintptr_t)dst);
    long ilo = a - hi >= 0 ? (a - hi) / ext + 1 : 0;
    long ihi = b - lo > 0 ? (b - lo + ext - 1) / ext : 0;
    if (ihi > n) ihi = n;
    // the units of those elements, read 16 bytes of the packed stream (G
    // units) per lane, two chunks in flight; a chunk that runs past the
    // stream's end is read unit by unit.  Offsets from here are 32-bit and
    // relative to the tile (an element's reach and the extent are bounded,
    // merge_ok): unit j of element ilo + ir lands at ir * ext + e0 + uoff[j]
    constexpr int G = 16 / W;
    const int up = (int)upe, ext32 = (int)ext, span = (int)(tend - t0);
    const int e0 = (int)(ilo * ext - a);
    const long q0 = ilo * upe, qn = n * upe, c0 = q0 / G, c1 = (ihi * upe + G - 1) / G;
    // TAB: chunk c0 + d is phase (p0 + d) % P of period k0 + (p0 + d) / P,
    // whose first element is (k0 + ...) EPP; relative to element ilo: b0
    const unsigned P = (unsigned)tabP, p0 = TAB ? (unsigned)(c0 % (long)P) : 0;
    const int epp = TAB ? (int)((long)P * G / upe) : 0;
    const int b0 = TAB ? (int)(c0 / (long)P * epp - ilo) : 0;
    for (long c = c0 + threadIdx.x; c < c1; c += 512) {
        pu32x4 v[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const long cc = c + 256 * u;
            if (cc < c1 && (cc + 1) * G <= qn) v[u] = __builtin_nontemporal_load((const pu32x4 *)(packed + 16 * cc));
        }
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const long cc = c + 256 * u;
            if (cc >= c1) continue;
            const int valid = qn - cc * G < G ? (int)(qn - cc * G) : G;   // units of the chunk in the stream
            if (valid < G) {                       // the stream's last, partial chunk: unit by unit
                v[u] = pu32x4{0, 0, 0, 0};
                for (int g = 0; g < valid; ++g) set_unit<W>(v[u], g, *(const V *)(packed + (cc * G + g) * W));
            }
            int rel[G];
            if constexpr (TAB) {
                const unsigned cr = (unsigned)(cc - c0) + p0, kk = cr / P, p = cr - kk * P;
                const int base = (b0 + (int)kk * epp) * ext32 + e0;
#pragma unroll
                for (int g4 = 0; g4 < G; g4 += 4) {
                    if constexpr (G >= 4) {
                        const pu32x4 t4 = *(const pu32x4 *)&s_uoff[p * G + g4];
#pragma unroll
                        for (int g = 0; g < 4; ++g) rel[g4 + g] = base + (int)t4[g];
                    } else {
#pragma unroll
                        for (int g = 0; g < G; ++g) rel[g] = base + s_uoff[p * G + g];
                    }
                }
            } else {
                // > -G: the first chunk may start in elements before ilo
                // (several when an element has fewer than G units), whose
                // units all land below the tile (ilo is the first element
                // reaching it); ir is the floor of qr / up, so j is a unit
                // index in every case
                const int qr = (int)(cc * G - q0);
                int ir = qr >= 0 ? (int)((unsigned)qr / (unsigned)up) : -(int)((unsigned)(up - 1 - qr) / (unsigned)up);
                int j = qr - ir * up;
#pragma unroll
                for (int g = 0; g < G; ++g) {
                    rel[g] = ir * ext32 + e0 + (LDSU ? s_uoff[j] : uoff[j]);
                    if (++j == up) { j = 0; ++ir; }
                }
            }
#pragma unroll
            for (int g = 0; g < G; ++g) {
                const bool in = (g < valid) & ((unsigned)rel[g] < (unsigned)span);
                *(V *)((char *)s_tile + (in ? lds_at<SWZ>(rel[g], swz) : TILE)) = unit_of<W>(v[u], g);
            }
        }
    }
    __syncthreads();
    for (int w = threadIdx.x; w < nw; w += 256) {
        const uintptr_t at = t0 + 16 * (uintptr_t)w;
        if (at >= h0 && at + 16 <= h1) {
            __builtin_nontemporal_store(*(const pu32x4 *)((const char *)s_tile + lds_at<SWZ>(16 * w, swz)),
                                        (pu32x4 *)at);
        } else {                                   // an edge word of the hull: its hull bytes only
            const uintptr_t b0 = at > h0 ? at : h0, b1 = at + 16 < h1 ? at + 16 : h1;
            const char *word = (const char *)s_tile + lds_at<SWZ>(16 * w, swz);
            for (uintptr_t b = b0; b < b1; ++b) *(char *)b = word[b - at];
        }
    }
}

// MVX_UNPACK_CHUNK_TAB=0: the whole-word unpack steps its unit offsets per
// unit (A/B)
static int merge_tab_on()
{
    static int on = -1;
    if (on < 0) {
        const char *e = getenv("MVX_UNPACK_CHUNK_TAB");
        on = e ? atoi(e) != 0 : 1;
    }
    return on;
}

// MVX_LDS_SWIZZLE=0: the tile kernels keep their LDS layout linear (A/B;
// Type::swz, swz_pick)
static int swz_on()
{
    static int on = -1;
    if (on < 0) {
        const char *e = getenv("MVX_LDS_SWIZZLE");
        on = e ? atoi(e) != 0 : 1;
    }
    return on;
}

// MVX_UNPACK_MERGE: 1 (default) unpack by whole words where the type's map
// qualifies, 0 the unit kernel's byte-exact stores everywhere
static int merge_on()
{
    static int on = -1;
    if (on < 0) {
        const char *e = getenv("MVX_UNPACK_MERGE");
        on = e ? atoi(e) != 0 : 1;
    }
    return on;
}

// The map's reach around the element origin [lo, hi) and whether whole-word
// unpack pays: the maps of neighbouring elements must not interleave (each
// destination byte has one writer), and the map must leave holes inside 64-B
// sectors (partial writes), with no 64-B sector of the hull wholly untouched
// (one that a byte-exact unpack would not touch at all but the merge would
// read and write).
static bool merge_ok(const Type &t, long *lo, long *hi)
{
    if (t.map.empty() || t.extent <= 0 || t.extent > (1L << 30)) return false;   // 32-bit tile offsets
    long l = t.map[0].off, h = t.map[0].off + t.map[0].len;
    for (const Blk &b : t.map) {
        if (b.off < l) l = b.off;
        if (b.off + b.len > h) h = b.off + b.len;
    }
    *lo = l;
    *hi = h;
    if (h - l > t.extent) return false;
    long g = t.extent, m = 64;
    while (m) { const long r = g % m; g = m; m = r; }
    const long reps = 64 / g, span = t.extent * reps;
    if (span > (1L << 20)) return false;
    std::vector<unsigned char> cov((size_t)span + 64, 0);
    for (long r = 0; r < reps; ++r)
        for (const Blk &b : t.map)
            for (long o = 0; o < b.len; ++o) {
                const long x = ((r * t.extent + b.off + o - l) % span + span) % span;
                cov[(size_t)x] = 1;
            }
    bool partial = false;
    for (long s = 0; s < span; s += 64) {
        int c = 0;
        for (long k = s; k < s + 64 && k < span; ++k) c += cov[(size_t)k];
        if (c == 0) return false;
        if (c < 64) partial = true;
    }
    return partial;
}

template <int W>
static int launch_merge(Type &t, int wi, const void *src, void *dst, long count, long lo, long hi, hipStream_t st)
{
    const long upe = t.units[wi];
    const uintptr_t h0 = (uintptr_t)dst + lo, h1 = (uintptr_t)dst + (count - 1) * t.extent + hi;
    const uintptr_t a0 = h0 & ~(uintptr_t)15;
    // 8 KiB tiles (4 KiB ran 30-40 % slower, 16 KiB 0-8 % slower:
    // profiles/r06/pack_tile_sizes.txt, pack_tile_sizes_noflat.txt)
    const long tiles = (long)((((h1 + 15) & ~(uintptr_t)15) - a0 + MERGE_TILE - 1) / MERGE_TILE);
    if (tiles < 1 || tiles > INT32_MAX) return MPI_ERR_OTHER;
    const int sw = swz_on() ? t.swz[wi] : 0;
#define MVX_MERGE_LAUNCH(LU, SW, TB)                                                                               \
    hipLaunchKernelGGL((k_unpack_merge<W, MERGE_TILE, LU, SW, TB>), dim3((unsigned)tiles), dim3(256), 0, st,       \
                       (const char *)src, (char *)dst, (const int *)t.dunits[wi], upe, count, t.extent, lo, hi, a0, \
                       h0, h1, sw, t.tabP[wi])
    // the chunk table for 1- and 2-byte units (as k_pack_tiles; MVX_PACK_CHUNK_TAB)
    const bool tb = merge_tab_on() && W <= 2 && t.tabP[wi] > 0;
    if (tb) {
        if (sw) MVX_MERGE_LAUNCH(false, true, true);
        else MVX_MERGE_LAUNCH(false, false, true);
    } else if (upe > MERGE_UNITS_LDS) {
        if (sw) MVX_MERGE_LAUNCH(false, true, false);
        else MVX_MERGE_LAUNCH(false, false, false);
    } else {
        if (sw) MVX_MERGE_LAUNCH(true, true, false);
        else MVX_MERGE_LAUNCH(true, false, false);
    }
#undef MVX_MERGE_LAUNCH
    return hipGetLastError() == hipSuccess ? MPI_SUCCESS : MPI_ERR_OTHER;
}

// ---- pack by whole words ----------------------------------------------------
// The unit kernel's pack reads 4 or 8 bytes per lane from the extent layout
// and writes as many to the packed stream: four or two times the memory
// instructions of 16-byte accesses, with each read instruction spread over
// several lines.  This variant gives a workgroup a run of whole elements:
// it loads their hull into LDS with 16-byte loads (whole aligned words: a
// word holding one hull byte lies in the same page, so the read is safe),
// then each lane gathers G = 16 / W units from LDS into one 16-byte chunk of
// the packed stream and stores it whole.  A run's packed bytes start on a
// 64-byte boundary (its element count is a multiple of 64 / gcd(size, 64));
// the stream's last, partial chunk is stored unit by unit.  (The kernel
// needs only 16-byte tile starts; pack_ept makes them 64-byte ones.)
#define PACK_TILE 8192               // LDS bytes of extent layout per workgroup

// TAB: the chunk table (Type::tabP phases after the unit offsets) in LDS
// instead of the unit offsets: a chunk's G unit offsets are one vector LDS
// read and one add each, with no per-unit element / unit-index stepping
template <int W, int TILE, bool LDSU, bool TAB, bool SWZ>
__global__ void __launch_bounds__(256)
k_pack_tiles(const char *__restrict__ src, char *__restrict__ dst, const int *__restrict__ uoff, long upe, long n,
             long ext, long lo, long hi, long ept, long tabP, int swz)
{
    typedef typename UnitT<W>::t V;
    constexpr int G = 16 / W;
    __shared__ pu32x4 s_tile[TILE / 16];
    __shared__ __attribute__((aligned(16))) int s_uoff[LDSU || TAB ? MERGE_UNITS_LDS : 1];   // LDSU: as in k_unpack_merge
    if (TAB)
        for (int u = threadIdx.x; u < (int)(tabP * G); u += 256) s_uoff[u] = uoff[upe + u];
    else if (LDSU)
        for (int u = threadIdx.x; u < (int)upe; u += 256) s_uoff[u] = uoff[u];
    const long i0 = (long)blockIdx.x * ept;
    const long i1 = i0 + ept < n ? i0 + ept : n;
    const uintptr_t a0 = ((uintptr_t)src + i0 * ext + lo) & ~(uintptr_t)15;
    const uintptr_t a1 = ((uintptr_t)src + (i1 - 1) * ext + hi + 15) & ~(uintptr_t)15;
    const int nw = (int)((a1 - a0) / 16);
    for (int w = threadIdx.x; w < nw; w += 256)
        *(pu32x4 *)((char *)s_tile + lds_at<SWZ>(16 * w, swz)) =
            __builtin_nontemporal_load((const pu32x4 *)(a0 + 16 * (uintptr_t)w));
    __syncthreads();
    const long qn = n * upe, qlo = i0 * upe, qhi = i1 * upe;
    const long c0 = qlo / G, c1 = (qhi + G - 1) / G;      // qlo is a multiple of G (ept)
    // 32-bit, tile-relative from here (pack_ept bounds the extent): unit j
    // of element i0 + ir sits at ir * ext + e0 + uoff[j] in the tile
    const int up = (int)upe, ext32 = (int)ext;
    const int e0 = (int)(i0 * ext - (long)(a0 - (uintptr_t)src));
    // TAB: chunk c0 + k P + p is phase p of period k, whose first element is
    // i0 + k EPP -- the tile starts a period: i0 is a multiple of pack_ept's
    // step 64 / gcd(size, 64), which EPP = G / gcd(upe, G) divides
    const unsigned P = (unsigned)tabP;
    const int epp = TAB ? (int)((long)P * G / upe) : 0;
    for (long c = c0 + threadIdx.x; c < c1; c += 256) {
        if (TAB && (c + 1) * G <= qn) {
            const unsigned cr = (unsigned)(c - c0), kk = cr / P, p = cr - kk * P;
            const int base = (int)kk * epp * ext32 + e0;
            pu32x4 out = {0, 0, 0, 0};
#pragma unroll
            for (int g4 = 0; g4 < G; g4 += 4) {
                int o[4];
                if constexpr (G >= 4) {
                    const pu32x4 t4 = *(const pu32x4 *)&s_uoff[p * G + g4];
                    o[0] = (int)t4[0]; o[1] = (int)t4[1]; o[2] = (int)t4[2]; o[3] = (int)t4[3];
                } else {
#pragma unroll
                    for (int g = 0; g < G; ++g) o[g] = s_uoff[p * G + g];
                }
#pragma unroll
                for (int g = 0; g < (G < 4 ? G : 4); ++g)
                    set_unit<W>(out, g4 + g, *(const V *)((const char *)s_tile + lds_at<SWZ>(base + o[g], swz)));
            }
            __builtin_nontemporal_store(out, (pu32x4 *)(dst + 16 * c));
            continue;
        }
        const unsigned qr = (unsigned)(c * G - qlo);
        int ir = (int)(qr / (unsigned)up), j = (int)qr - ir * up;
        if ((c + 1) * G <= qn) {
            pu32x4 out = {0, 0, 0, 0};
#pragma unroll
            for (int g = 0; g < G; ++g) {
                const int rel = ir * ext32 + e0 + (LDSU ? s_uoff[j] : uoff[j]);
                set_unit<W>(out, g, *(const V *)((const char *)s_tile + lds_at<SWZ>(rel, swz)));
                if (++j == up) { j = 0; ++ir; }
            }
            __builtin_nontemporal_store(out, (pu32x4 *)(dst + 16 * c));
        } else {
            for (long q = c * G; q < qn; ++q) {
                const int rel = ir * ext32 + e0 + (LDSU ? s_uoff[j] : uoff[j]);
                *(V *)(dst + q * W) = *(const V *)((const char *)s_tile + lds_at<SWZ>(rel, swz));
                if (++j == up) { j = 0; ++ir; }
            }
        }
    }
}

// MVX_PACK_TILES: 1 (default) pack maps of 4- and 8-byte units through LDS
// tiles where an element's hull is small, 0 the unit kernel everywhere
static int tiles_on()
{
    static int on = -1;
    if (on < 0) {
        const char *e = getenv("MVX_PACK_TILES");
        on = e ? atoi(e) != 0 : 1;
    }
    return on;
}

// elements per tile (a multiple of 64 / gcd(size, 64): each tile's packed
// bytes start on a 64-byte sector, so no two workgroups write one sector;
// its hull within the tile with the alignment slack), or 0: no tiling
static long pack_ept(const Type &t, long lo, long hi)
{
    // 8 KiB tiles leave room for 8 resident workgroups per CU; 16 KiB (6 per
    // CU, LDS-bound) and 4 KiB (too little work per tile) ran slower
    // (profiles/r06/pack_tile_sizes.txt, pack_tile_sizes_noflat.txt)
    const long TILE = PACK_TILE;
    if (t.extent <= 0 || t.extent > (1L << 30) || t.size <= 0 || hi - lo > TILE / 4) return 0;
    long g = t.size, m = 64;
    while (m) { const long r = g % m; g = m; m = r; }
    const long step = 64 / g;
    // hull of e elements: (e - 1) * ext + (hi - lo), plus up to 30 bytes of
    // word alignment; spans reaching below the element (lo < 0) included
    long e = (TILE - 32 - (hi - lo)) / t.extent + 1;
    e -= e % step;
    return e >= step ? e : 0;
}

template <int W>
static int launch_tiles(Type &t, int wi, const void *src, void *dst, long count, long lo, long hi, long ept,
                        hipStream_t st)
{
    const long tiles = (count + ept - 1) / ept;
    if (tiles < 1 || tiles > INT32_MAX) return MPI_ERR_OTHER;
#define MVX_PACK_TILES_LAUNCH(LU, TB, SW)                                                                        \
    hipLaunchKernelGGL((k_pack_tiles<W, PACK_TILE, LU, TB, SW>), dim3((unsigned)tiles), dim3(256), 0, st,          \
                       (const char *)src, (char *)dst, (const int *)t.dunits[wi], t.units[wi], count, t.extent, lo,  \
                       hi, ept, t.tabP[wi], sw)
    // MVX_PACK_CHUNK_TAB=0: the unit offsets stepped per unit (A/B)
    static int tab_on = -1;
    if (tab_on < 0) {
        const char *e = getenv("MVX_PACK_CHUNK_TAB");
        tab_on = e ? atoi(e) != 0 : 1;
    }
    // (W = 2 and 1 only: with 2 or 4 units per chunk the table did not pay,
    // profiles/r06/pack_chunk_tab_ab.txt)
    const bool tb = tab_on && W <= 2 && t.tabP[wi] > 0, lu = t.units[wi] <= MERGE_UNITS_LDS;
    // the swizzle for 1- and 2-byte units only: G = 16 / W LDS reads per
    // chunk; at W = 4 it cost its address arithmetic and gained nothing
    // (struct {int; hole; double} 74.5-75.1 -> 75.6-75.9 us, whose unpack it
    // takes 114.8 -> 113.9; profiles/r06/lds_swizzle_ab.txt)
    const int sw = swz_on() && W <= 2 ? t.swz[wi] : 0;
    if (tb) {
        if (sw) MVX_PACK_TILES_LAUNCH(false, true, true);
        else MVX_PACK_TILES_LAUNCH(false, true, false);
    } else if (lu) {
        if (sw) MVX_PACK_TILES_LAUNCH(true, false, true);
        else MVX_PACK_TILES_LAUNCH(true, false, false);
    } else {
        if (sw) MVX_PACK_TILES_LAUNCH(false, false, true);
        else MVX_PACK_TILES_LAUNCH(false, false, false);
    }
#undef MVX_PACK_TILES_LAUNCH
    return hipGetLastError() == hipSuccess ? MPI_SUCCESS : MPI_ERR_OTHER;
}

static int device_map(Type &t)
{
    if (t.dmap) return MPI_SUCCESS;
    std::vector<DBlk> v;
    long poff = 0;
    for (const Blk &b : t.map)
        for (long o = 0; o < b.len; o += 64) {
            const long len = b.len - o < 64 ? b.len - o : 64;
            v.push_back({b.off + o, poff, (int)len, 0});
            poff += len;
        }
    if (v.empty()) return MPI_SUCCESS;
    if (hipMalloc(&t.dmap, v.size() * sizeof(DBlk)) != hipSuccess) { t.dmap = nullptr; return MPI_ERR_OTHER; }
    if (hipMemcpy(t.dmap, v.data(), v.size() * sizeof(DBlk), hipMemcpyHostToDevice) != hipSuccess)
        return MPI_ERR_OTHER;
    t.dmap_n = (long)v.size();
    return MPI_SUCCESS;
}

static int pack(int h, const void *src, void *dst, size_t count, hipStream_t st, bool packing)
{
    Type *t = slot(h);
    Type v;
    if (!t) {
        // a basic type is its own packed form
        if (!basic(h, v)) return MPI_ERR_TYPE;
        if (!count || !v.size) return MPI_SUCCESS;
        if (v.map.size() == 1)
            return hipMemcpyAsync(dst, src, count * (size_t)v.size, hipMemcpyDeviceToDevice, st) == hipSuccess
                   ? MPI_SUCCESS : MPI_ERR_OTHER;
        return MPI_ERR_TYPE;   // the padded pair structs move whole (mvx_dtype.h dense)
    }
    if (!count || !t->size) return MPI_SUCCESS;
    {
        static int units_on = -1;    // MVX_PACK_UNITS=0: the piece kernel only (A/B)
        if (units_on < 0) {
            const char *e = getenv("MVX_PACK_UNITS");
            units_on = e ? atoi(e) != 0 : 1;
        }
        const uintptr_t al = (uintptr_t)src | (uintptr_t)dst;
        const int Ws[3] = {16, 8, 4};
        for (int wi = 0; units_on && wi < 3; ++wi) {
            const int W = Ws[wi];
            if (al % W || !unit_table(*t, W, wi)) continue;
            if (packing && W < 16 && tiles_on() && (uintptr_t)dst % 16 == 0) {
                long lo, hi;
                if (!t->merge) t->merge = merge_ok(*t, &t->mlo, &t->mhi) ? 1 : -1;   // fills the reach too
                lo = t->mlo;
                hi = t->mhi;
                const long ept = pack_ept(*t, lo, hi);
                if (ept > 0) {
                    if (W == 8) return launch_tiles<8>(*t, wi, src, dst, (long)count, lo, hi, ept, st);
                    return launch_tiles<4>(*t, wi, src, dst, (long)count, lo, hi, ept, st);
                }
            }
            if (!packing && merge_on() && (uintptr_t)src % 16 == 0) {
                if (!t->merge) t->merge = merge_ok(*t, &t->mlo, &t->mhi) ? 1 : -1;
                if (t->merge > 0) {
                    if (W == 16) return launch_merge<16>(*t, wi, src, dst, (long)count, t->mlo, t->mhi, st);
                    if (W == 8) return launch_merge<8>(*t, wi, src, dst, (long)count, t->mlo, t->mhi, st);
                    return launch_merge<4>(*t, wi, src, dst, (long)count, t->mlo, t->mhi, st);
                }
            }
            if (W == 16) return packing ? launch_units<true, 16>(*t, wi, src, dst, (long)count, st)
                                        : launch_units<false, 16>(*t, wi, src, dst, (long)count, st);
            if (W == 8) return packing ? launch_units<true, 8>(*t, wi, src, dst, (long)count, st)
                                       : launch_units<false, 8>(*t, wi, src, dst, (long)count, st);
            return packing ? launch_units<true, 4>(*t, wi, src, dst, (long)count, st)
                           : launch_units<false, 4>(*t, wi, src, dst, (long)count, st);
        }
    }
    {
        // maps with 2- or 1-byte pieces: the tile kernels over 2- or 1-byte
        // units where they apply, else the piece kernel below
        static int units_on = -1;
        if (units_on < 0) {
            const char *e = getenv("MVX_PACK_UNITS");
            units_on = e ? atoi(e) != 0 : 1;
        }
        const uintptr_t al = (uintptr_t)src | (uintptr_t)dst;
        for (int wi = 3; units_on && t->size <= 4096 && wi < 5; ++wi) {   // small elements only
            const int W = wi == 3 ? 2 : 1;
            if (al % W || !unit_table(*t, W, wi)) continue;
            if (!t->merge) t->merge = merge_ok(*t, &t->mlo, &t->mhi) ? 1 : -1;
            if (packing && tiles_on() && (uintptr_t)dst % 16 == 0) {
                const long ept = pack_ept(*t, t->mlo, t->mhi);
                if (ept > 0)
                    return W == 2 ? launch_tiles<2>(*t, wi, src, dst, (long)count, t->mlo, t->mhi, ept, st)
                                  : launch_tiles<1>(*t, wi, src, dst, (long)count, t->mlo, t->mhi, ept, st);
            }
            if (!packing && merge_on() && (uintptr_t)src % 16 == 0 && t->merge > 0)
                return W == 2 ? launch_merge<2>(*t, wi, src, dst, (long)count, t->mlo, t->mhi, st)
                              : launch_merge<1>(*t, wi, src, dst, (long)count, t->mlo, t->mhi, st);
            break;
        }
    }
    int rc = device_map(*t);
    if (rc) return rc;
    const long items = (long)count * t->dmap_n;
    long blocks = (items + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    if (packing)
        hipLaunchKernelGGL(k_pack<true>, dim3((unsigned)blocks), dim3(256), 0, st, (const char *)src, (char *)dst,
                           (const DBlk *)t->dmap, t->dmap_n, (long)count, t->extent, t->size);
    else
        hipLaunchKernelGGL(k_pack<false>, dim3((unsigned)blocks), dim3(256), 0, st, (const char *)src, (char *)dst,
                           (const DBlk *)t->dmap, t->dmap_n, (long)count, t->extent, t->size);
    return hipGetLastError() == hipSuccess ? MPI_SUCCESS : MPI_ERR_OTHER;
}

}  // namespace dt
}  // namespace mvx

using namespace mvx::dt;

extern "C" int mvx_type_describe(int type, int *oldtype, int *count, long *extent, long *size)
{
    Info in;
    if (!info(type, &in) || in.kind == K_UB || in.kind == K_LB) return MPI_ERR_TYPE;
    if (oldtype) *oldtype = in.old;
    if (count) *count = in.count;
    if (extent) *extent = in.extent;
    if (size) *size = in.size;
    return MPI_SUCCESS;
}

extern "C" int mvx_type_layout(int type, int *kind, int *dense, long *lb, long *ub, long *span_lo,
                               long *span_hi)
{
    Info in;
    if (!info(type, &in)) return MPI_ERR_TYPE;
    if (kind) *kind = in.kind;
    if (dense) *dense = in.dense;
    if (lb) *lb = in.lb;
    if (ub) *ub = in.ub;
    if (span_lo) *span_lo = in.span_lo;
    if (span_hi) *span_hi = in.span_hi;
    return MPI_SUCCESS;
}

extern "C" int mvx_type_contiguous(int count, int oldtype, int *newtype)
{
    return contiguous(count, oldtype, newtype);
}

extern "C" int mvx_type_vector(int count, int blocklen, int stride, int oldtype, int *newtype)
{
    if (!newtype) return MPI_ERR_ARG;
    return vector(count, blocklen, stride, oldtype, newtype);
}

extern "C" int mvx_type_hvector(int count, int blocklen, long stride, int oldtype, int *newtype)
{
    if (!newtype) return MPI_ERR_ARG;
    return hvector(count, blocklen, stride, oldtype, newtype);
}

extern "C" int mvx_type_indexed(int count, const int *blocklens, const int *indices, int oldtype,
                                int *newtype)
{
    if (!newtype || (count > 0 && (!blocklens || !indices))) return MPI_ERR_ARG;
    return indexed(count, blocklens, indices, oldtype, newtype);
}

extern "C" int mvx_type_hindexed(int count, const int *blocklens, const long *indices, int oldtype,
                                 int *newtype)
{
    if (!newtype || (count > 0 && (!blocklens || !indices))) return MPI_ERR_ARG;
    return hindexed(count, blocklens, indices, oldtype, newtype);
}

extern "C" int mvx_type_struct(int count, const int *blocklens, const long *indices, const int *types,
                               int *newtype)
{
    if (!newtype || (count > 0 && (!blocklens || !indices || !types))) return MPI_ERR_ARG;
    return structure(count, blocklens, indices, types, newtype);
}

extern "C" int mvx_type_commit(int type) { return commit(type); }

// type_free.c:60-105
extern "C" int mvx_type_free(int *type)
{
    Type v;
    if (!type) return MPI_ERR_ARG;
    Type *t = slot(*type);
    if (!t) {
        if (*type != MPI_DATATYPE_NULL && basic(*type, v)) return MVX_ERR_PERM_TYPE;
        return MVX_ERR_TYPE_NULL;
    }
    release(*type);
    *type = MPI_DATATYPE_NULL;
    return MPI_SUCCESS;
}

extern "C" int mvx_dtype_extent(int dtype)
{
    long e;
    return mvx_type_describe(dtype, nullptr, nullptr, &e, nullptr) ? 0 : (int)e;
}

extern "C" int mvx_type_pack(int type, const void *origin, void *packed, size_t count, void *stream)
{
    return pack(type, origin, packed, count, (hipStream_t)stream, true);
}

extern "C" int mvx_type_unpack(int type, const void *packed, void *origin, size_t count, void *stream)
{
    return pack(type, packed, origin, count, (hipStream_t)stream, false);
}
