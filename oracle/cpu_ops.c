/*
 * cpu_ops.c -- TEST INFRASTRUCTURE: CPU restatement of the reference's
 * predefined MPI_Op kernels (reference src/coll/global_ops.c).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use
 * this file (via oracle/liboracle.so).  It is the checker, never the product.
 *
 * Semantics restated (a = inoutvec element, b = invec element):
 *   MAX  a = (b > a) ? b : a          coll.h:17-18 via global_ops.c:56-163
 *   MIN  a = (a > b) ? b : a          coll.h:14-15 via global_ops.c:166-273
 *   SUM  a = a + b                    global_ops.c:281-406 (complex 389-403)
 *   PROD a = a * b; complex product   global_ops.c:410-538 (518-519, 528-529)
 *   LAND a = a && b                   global_ops.c:543-661 (float cast 628)
 *   BAND a = a & b                    global_ops.c:666-767
 *   LOR  a = a || b                   global_ops.c:772-890
 *   BOR  a = a | b                    global_ops.c:894-996
 *   LXOR a = (a && !b) || (!a && b)   global_ops.c:1001-1119
 *   BXOR a = a ^ b                    global_ops.c:1124-1226
 *   MAXLOC/MINLOC on struct pair types (global_ops.c:1271-1384,1511-1620)
 *   and on the contiguous MPI_2INT (global_ops.c:1387-1503, 1622-1740).
 *   The Fortran types of a Fortran-enabled build: INTEGER / REAL / DOUBLE
 *   PRECISION as int / float / double, LOGICAL (646-655 and siblings), and
 *   the contiguous pairs 2INTEGER / 2REAL / 2DOUBLE_PRECISION.
 * The C element types are the reference's (char is signed on x86-64, long is
 * 64-bit, long double is x87 80-bit in a 16-byte slot), compiled by the same
 * gcc at -O2; -fwrapv makes the signed wrap the reference gets in practice
 * well-defined here.
 */
#include <stddef.h>
#include <stdint.h>
#include <string.h>
#include "oracle.h"

#define ERR_OP_NOT_DEFINED 329 /* MPIR_ERRCLASS_TO_CODE(MPI_ERR_OP, 5) */
#define ERR_OP 9
#define ERR_TYPE 3

enum { T_CHAR = 1, T_UCHAR, T_BYTE, T_SHORT, T_USHORT, T_INT, T_UINT, T_LONG,
       T_ULONG, T_FLOAT, T_DOUBLE, T_LDOUBLE, T_LLONG, T_PACKED, T_LB, T_UB,
       T_FLOAT_INT, T_DOUBLE_INT, T_LONG_INT, T_SHORT_INT, T_2INT,
       T_LDOUBLE_INT, T_COMPLEX, T_DCOMPLEX,
       /* the Fortran types (mpi.h:104-112; initfutil.c:220-349) */
       T_LOGICAL, T_REAL, T_DPREC, T_INTEGER, T_2INTEGER, T_2COMPLEX,
       T_2DCOMPLEX, T_2REAL, T_2DPREC };

/* MPIR_F_TRUE / MPIR_F_FALSE (initfutil.c:100-102; gfortran's literals) */
static int g_ftrue = 1, g_ffalse = 0;

void orc_set_flog(int true_value, int false_value)
{
    g_ftrue = true_value;
    g_ffalse = false_value;
}

/* the dte_type a Fortran handle shares with a C type (initfutil.c:238-245,
   261, 279; sizeof(int) == sizeof(float) == 4 with gfortran) */
static int fdte(int t)
{
    return t == T_INTEGER ? T_INT : t == T_REAL ? T_FLOAT : t == T_DPREC ? T_DOUBLE : t;
}

typedef struct { float re, im; } s_cplx;
typedef struct { double re, im; } d_cplx;
typedef struct { float v; int l; } p_float_int;   /* initdte.c:74-78 */
typedef struct { double v; int l; } p_double_int; /* initdte.c:80-84 */
typedef struct { long v; int l; } p_long_int;     /* initdte.c:86-90 */
typedef struct { short v; int l; } p_short_int;   /* initdte.c:92-96 */
typedef struct { long double v; int l; } p_ldouble_int;

/* Derived types live in cpu_types.c (handles 256 + slot). */
static int is_derived(int h)
{
    return orc_derived_info(h, NULL, NULL, NULL, NULL, NULL) == 0;
}

int orc_dtype_info(int dtype, int *extent, int *type_size)
{
    int e, s;
    if (is_derived(dtype)) {
        long de, ds;
        orc_derived_info(dtype, NULL, NULL, NULL, &de, &ds);
        if (extent) *extent = (int)de;
        if (type_size) *type_size = (int)ds;
        return 0;
    }
    switch (dtype) {
    case T_CHAR: case T_UCHAR: case T_BYTE: case T_PACKED: e = s = 1; break;
    case T_SHORT: case T_USHORT: e = s = 2; break;
    case T_INT: case T_UINT: case T_FLOAT: e = s = 4; break;
    case T_LONG: case T_ULONG: case T_DOUBLE: case T_LLONG: e = s = 8; break;
    case T_LDOUBLE: e = s = (int)sizeof(long double); break;
    /* pair types: extent includes the MPI_UB padding, size does not
       (initdte.c:169-222) */
    case T_FLOAT_INT: e = sizeof(p_float_int); s = 8; break;
    case T_DOUBLE_INT: e = sizeof(p_double_int); s = 12; break;
    case T_LONG_INT: e = sizeof(p_long_int); s = 12; break;
    case T_SHORT_INT: e = sizeof(p_short_int); s = 6; break;
    case T_2INT: e = s = 8; break;
    case T_LDOUBLE_INT: e = sizeof(p_ldouble_int);
        s = (int)sizeof(long double) + 4; break;
    /* Fortran complex types: handled by the op kernels; registered only in
       Fortran-enabled builds.  We accept them. */
    case T_COMPLEX: e = s = 8; break;
    case T_DCOMPLEX: e = s = 16; break;
    case T_LOGICAL: case T_REAL: case T_INTEGER: e = s = 4; break;
    case T_DPREC: case T_2INTEGER: case T_2REAL: e = s = 8; break;
    case T_2DPREC: case T_2COMPLEX: e = s = 16; break;
    case T_2DCOMPLEX: e = s = 32; break;
    default: return ERR_TYPE;
    }
    if (extent) *extent = e;
    if (type_size) *type_size = s;
    return 0;
}

/* element-wise loop over one C type */
#define LOOP(T, EXPR)                                                        \
    do {                                                                     \
        T *a = (T *)inout; const T *b = (const T *)in;                       \
        for (i = 0; i < len; i++) a[i] = (T)(EXPR);                          \
    } while (0)

/* the integer types every arithmetic / logical op accepts */
#define INT_CASES(EXPR)                                                      \
    case T_INT:    LOOP(int, EXPR); break;                                   \
    case T_UINT:   LOOP(unsigned int, EXPR); break;                          \
    case T_LONG:   LOOP(long, EXPR); break;                                  \
    case T_LLONG:  LOOP(long long, EXPR); break;                             \
    case T_ULONG:  LOOP(unsigned long, EXPR); break;                         \
    case T_SHORT:  LOOP(short, EXPR); break;                                 \
    case T_USHORT: LOOP(unsigned short, EXPR); break;                        \
    case T_CHAR:   LOOP(char, EXPR); break;                                  \
    case T_UCHAR:  LOOP(unsigned char, EXPR); break;

#define FLT_CASES(EXPR)                                                      \
    case T_FLOAT:   LOOP(float, EXPR); break;                                \
    case T_DOUBLE:  LOOP(double, EXPR); break;                               \
    case T_LDOUBLE: LOOP(long double, EXPR); break;

#define E_MAX  ((b[i] > a[i]) ? b[i] : a[i])
#define E_MIN  ((a[i] > b[i]) ? b[i] : a[i])
#define E_SUM  (a[i] + b[i])
#define E_PROD (a[i] * b[i])
#define E_LAND (a[i] && b[i])
#define E_LOR  (a[i] || b[i])
#define E_LXOR ((a[i] && !b[i]) || (!a[i] && b[i]))
#define E_BAND (a[i] & b[i])
#define E_BOR  (a[i] | b[i])
#define E_BXOR (a[i] ^ b[i])

/* MAXLOC (gt = 0) / MINLOC (gt = 1) on one pair layout */
#define PAIR_LOOP(P)                                                         \
    do {                                                                     \
        P *a = (P *)inout; const P *b = (const P *)in;                       \
        for (i = 0; i < len; i++) {                                          \
            if (a[i].v == b[i].v)                                            \
                a[i].l = (a[i].l > b[i].l) ? b[i].l : a[i].l;                \
            else if (is_min ? (a[i].v > b[i].v) : (a[i].v < b[i].v)) {       \
                a[i].v = b[i].v;                                             \
                a[i].l = b[i].l;                                             \
            }                                                                \
        }                                                                    \
    } while (0)

/* MAXLOC / MINLOC on a derived contiguous type with count == 2: stride-2
 * scalars of the old type (global_ops.c:1387-1503, 1625-1740); len is
 * doubled (1392).  Any other derived type: 329 (1504-1507, 1741-1744). */
#define CONTIG2_LOOP(T)                                                      \
    do {                                                                     \
        T *a = (T *)inout; const T *b = (const T *)in;                       \
        for (i = 0; i < n2; i += 2) {                                        \
            if (a[i] == b[i])                                                \
                a[i + 1] = (a[i + 1] > b[i + 1]) ? b[i + 1] : a[i + 1];      \
            else if (is_min ? (a[i] > b[i]) : (a[i] < b[i])) {               \
                a[i] = b[i];                                                 \
                a[i + 1] = b[i + 1];                                         \
            }                                                                \
        }                                                                    \
    } while (0)

static int loc_op(int is_min, int dtype, const void *in, void *inout, int len)
{
    int i, n2 = len * 2;
    switch (dtype) {
    case T_FLOAT_INT:   PAIR_LOOP(p_float_int); return 0;
    case T_DOUBLE_INT:  PAIR_LOOP(p_double_int); return 0;
    case T_LONG_INT:    PAIR_LOOP(p_long_int); return 0;
    case T_SHORT_INT:   PAIR_LOOP(p_short_int); return 0;
    case T_LDOUBLE_INT: PAIR_LOOP(p_ldouble_int); return 0;
    /* the Fortran pairs: contiguous(2, REAL / DOUBLE PRECISION) run the
       stride-2 case of their old type's dte_type (1459-1482) */
    case T_2REAL:  CONTIG2_LOOP(float); return 0;
    case T_2DPREC: CONTIG2_LOOP(double); return 0;
    case T_2INT: case T_2INTEGER: {
        /* contiguous count-2 type: stride-2 scalars (global_ops.c:1387-1403) */
        int *a = (int *)inout; const int *b = (const int *)in;
        int n2 = len * 2;
        for (i = 0; i < n2; i += 2) {
            if (a[i] == b[i])
                a[i + 1] = (a[i + 1] > b[i + 1]) ? b[i + 1] : a[i + 1];
            else if (is_min ? (a[i] > b[i]) : (a[i] < b[i])) {
                a[i] = b[i];
                a[i + 1] = b[i + 1];
            }
        }
        return 0;
    }
    default:
        return ERR_OP_NOT_DEFINED;
    }
}

static int derived_loc_op(int is_min, int dtype, const void *in, void *inout, int len)
{
    int old, count, i, n2, kind;
    orc_derived_info(dtype, &kind, &old, &count, NULL, NULL);
    if (kind == 4) {
        /* MPIR_STRUCT: the C pair struct of old_types[0]'s dte_type
         * (global_ops.c:1280-1384, 1520-1620) */
        switch (fdte(old)) {
        case T_INT: return loc_op(is_min, T_2INT, in, inout, len);    /* MPIR_2int_loctype */
        case T_FLOAT: return loc_op(is_min, T_FLOAT_INT, in, inout, len);
        case T_LONG: case T_LLONG: return loc_op(is_min, T_LONG_INT, in, inout, len);
        case T_SHORT: return loc_op(is_min, T_SHORT_INT, in, inout, len);
        case T_DOUBLE: return loc_op(is_min, T_DOUBLE_INT, in, inout, len);
        case T_LDOUBLE: return loc_op(is_min, T_LDOUBLE_INT, in, inout, len);
        default: return ERR_OP_NOT_DEFINED;
        }
    }
    if (kind != 1 || count != 2) return ERR_OP_NOT_DEFINED;
    n2 = len * count;
    switch (fdte(old)) {
    case T_INT:     CONTIG2_LOOP(int); return 0;
    case T_LONG:    CONTIG2_LOOP(long); return 0;
    case T_LLONG:   CONTIG2_LOOP(long long); return 0;
    case T_SHORT:   CONTIG2_LOOP(short); return 0;
    case T_CHAR:    CONTIG2_LOOP(char); return 0;
    case T_FLOAT:   CONTIG2_LOOP(float); return 0;
    case T_DOUBLE:  CONTIG2_LOOP(double); return 0;
    case T_LDOUBLE: CONTIG2_LOOP(long double); return 0;
    default: return ERR_OP_NOT_DEFINED;
    }
}

int orc_op(int op, int dtype, const void *in, void *inout, int len)
{
    int i;
    if (is_derived(dtype)) {
        if (op < 100 || op > 111) return ERR_OP;
        if (op == 111 || op == 110) return derived_loc_op(op == 110, dtype, in, inout, len);
        return ERR_OP_NOT_DEFINED;   /* no MPIR_CONTIG case in any other op */
    }
    if (dtype == T_LOGICAL) {
        /* MPIR_LOGICAL, one MPI_Fint: the logical ops through FROM_FLOG /
           TO_FLOG (global_ops.c:646-655, 875-884, 1104-1113; mpi_fort.h:11-19),
           the bitwise ops on the word (678-684, 906-912, 1136-1142) */
#define FROM_FLOG(x) ((x) == g_ftrue ? 1 : 0)
#define TO_FLOG(v) ((v) ? g_ftrue : g_ffalse)
        int *a = (int *)inout; const int *b = (const int *)in;
        switch (op) {
        case 104: for (i = 0; i < len; i++) a[i] = TO_FLOG(FROM_FLOG(a[i]) && FROM_FLOG(b[i])); return 0;
        case 106: for (i = 0; i < len; i++) a[i] = TO_FLOG(FROM_FLOG(a[i]) || FROM_FLOG(b[i])); return 0;
        case 108: for (i = 0; i < len; i++) {
                      int x = FROM_FLOG(a[i]), y = FROM_FLOG(b[i]);
                      a[i] = TO_FLOG((x && !y) || (!x && y));
                  }
                  return 0;
        case 105: for (i = 0; i < len; i++) a[i] = a[i] & b[i]; return 0;
        case 107: for (i = 0; i < len; i++) a[i] = a[i] | b[i]; return 0;
        case 109: for (i = 0; i < len; i++) a[i] = a[i] ^ b[i]; return 0;
        default: return (op < 100 || op > 111) ? ERR_OP : ERR_OP_NOT_DEFINED;
        }
#undef FROM_FLOG
#undef TO_FLOG
    }
    if (op != 111 && op != 110) dtype = fdte(dtype);
    switch (op) {
    case 100: /* MPI_MAX */
        switch (dtype) { INT_CASES(E_MAX) FLT_CASES(E_MAX)
        default: return ERR_OP_NOT_DEFINED; }
        return 0;
    case 101: /* MPI_MIN */
        switch (dtype) { INT_CASES(E_MIN) FLT_CASES(E_MIN)
        default: return ERR_OP_NOT_DEFINED; }
        return 0;
    case 102: /* MPI_SUM */
        switch (dtype) { INT_CASES(E_SUM) FLT_CASES(E_SUM)
        case T_COMPLEX: {
            s_cplx *a = (s_cplx *)inout; const s_cplx *b = (const s_cplx *)in;
            for (i = 0; i < len; i++) { a[i].re = a[i].re + b[i].re;
                                        a[i].im = a[i].im + b[i].im; }
            break; }
        case T_DCOMPLEX: {
            d_cplx *a = (d_cplx *)inout; const d_cplx *b = (const d_cplx *)in;
            for (i = 0; i < len; i++) { a[i].re = a[i].re + b[i].re;
                                        a[i].im = a[i].im + b[i].im; }
            break; }
        default: return ERR_OP_NOT_DEFINED; }
        return 0;
    case 103: /* MPI_PROD */
        switch (dtype) { INT_CASES(E_PROD) FLT_CASES(E_PROD)
        case T_COMPLEX: {
            s_cplx *a = (s_cplx *)inout; const s_cplx *b = (const s_cplx *)in;
            for (i = 0; i < len; i++) {
                s_cplx c = a[i];
                a[i].re = c.re * b[i].re - c.im * b[i].im;
                a[i].im = c.im * b[i].re + c.re * b[i].im;
            }
            break; }
        case T_DCOMPLEX: {
            d_cplx *a = (d_cplx *)inout; const d_cplx *b = (const d_cplx *)in;
            for (i = 0; i < len; i++) {
                d_cplx c = a[i];
                a[i].re = c.re * b[i].re - c.im * b[i].im;
                a[i].im = c.im * b[i].re + c.re * b[i].im;
            }
            break; }
        default: return ERR_OP_NOT_DEFINED; }
        return 0;
    case 104: /* MPI_LAND */
        switch (dtype) { INT_CASES(E_LAND) FLT_CASES(E_LAND)
        default: return ERR_OP_NOT_DEFINED; }
        return 0;
    case 106: /* MPI_LOR */
        switch (dtype) { INT_CASES(E_LOR) FLT_CASES(E_LOR)
        default: return ERR_OP_NOT_DEFINED; }
        return 0;
    case 108: /* MPI_LXOR */
        switch (dtype) { INT_CASES(E_LXOR) FLT_CASES(E_LXOR)
        default: return ERR_OP_NOT_DEFINED; }
        return 0;
    case 105: /* MPI_BAND */
        switch (dtype) { INT_CASES(E_BAND)
        case T_BYTE: LOOP(unsigned char, E_BAND); break;
        default: return ERR_OP_NOT_DEFINED; }
        return 0;
    case 107: /* MPI_BOR */
        switch (dtype) { INT_CASES(E_BOR)
        case T_BYTE: LOOP(unsigned char, E_BOR); break;
        default: return ERR_OP_NOT_DEFINED; }
        return 0;
    case 109: /* MPI_BXOR */
        switch (dtype) { INT_CASES(E_BXOR)
        case T_BYTE: LOOP(unsigned char, E_BXOR); break;
        default: return ERR_OP_NOT_DEFINED; }
        return 0;
    case 111: /* MPI_MAXLOC */
        return loc_op(0, dtype, in, inout, len);
    case 110: /* MPI_MINLOC */
        return loc_op(1, dtype, in, inout, len);
    default:
        return ERR_OP;
    }
}

/* ---------------------------------------------------------------------- */
/* synthetic inputs, SURVEY.md 8(d)                                       */

static inline uint64_t xs64(uint64_t *s)
{
    uint64_t x = *s;
    x ^= x << 13; x ^= x >> 7; x ^= x << 17;
    *s = x;
    return x;
}

void orc_fill(void *buf, long n, int dist, int rank)
{
    uint64_t s = 0x9E3779B97F4A7C15ULL ^ ((uint64_t)rank * 1000003ULL + 1ULL);
    long i;
    switch (dist) {
    case 0: { /* mixed sign, exponent spread */
        float *f = (float *)buf;
        for (i = 0; i < n; i++) {
            uint64_t u = xs64(&s), u2 = xs64(&s);
            int m = (int)(u % 2000001ULL) - 1000000;
            f[i] = (float)((double)m * 1e-3 * (double)(1 + u2 % 1000ULL));
        }
        break; }
    case 1: { /* U[0,1) */
        float *f = (float *)buf;
        for (i = 0; i < n; i++)
            f[i] = (float)((xs64(&s) >> 40) * (1.0 / 16777216.0));
        break; }
    case 2: { /* int64 words, P(bit = 1) = 1 - (1/16)(1/4) = 0.953 (six draws) */
        uint64_t *w = (uint64_t *)buf;
        for (i = 0; i < n; i++) {
            uint64_t a = xs64(&s), b = xs64(&s), c = xs64(&s), d = xs64(&s);
            uint64_t e = xs64(&s), f = xs64(&s);
            w[i] = a | b | c | d | (e & f);
        }
        break; }
    case 3: case 4: { /* FLOAT_INT pairs with many ties */
        p_float_int *p = (p_float_int *)buf;
        for (i = 0; i < n; i++) {
            p[i].v = (float)(xs64(&s) % 1024ULL);
            p[i].l = dist == 3 ? rank : (int)((long)rank * n + i);
        }
        break; }
    default: { /* raw words */
        uint64_t *w = (uint64_t *)buf;
        for (i = 0; i < n; i++) w[i] = xs64(&s);
        break; }
    }
}
