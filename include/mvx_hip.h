/*
 * mvx_hip.h -- C-ABI of libmvx_hip.so, the thin device layer of the
 * reduction path (hand-written HIP for gfx950).
 *
 * Every entry point takes plain device pointers and element counts, is
 * stream-ordered (nothing synchronises unless stated), allocates nothing,
 * takes no ownership, and returns an MPI error code instead of setting a
 * global errno (the reference's MPIR_Op_errno, coll.h:61-68, is replaced by
 * the return value).
 *
 * Reference interfaces replaced:
 *   mvx_op_apply     the predefined op kernels MPIR_MAXF ... MPIR_MINLOC,
 *                    src/coll/global_ops.c:56-1745, called through
 *                    MPI_User_function (include/mpi.h:206) as
 *                    (*uop)(invec, inoutvec, &len, &type), e.g.
 *                    src/coll/intra_fns_new.c:5697.
 *   mvx_op_combine   a whole chain of (*uop) calls of one collective in one
 *                    HBM pass: the Rabenseifner / recursive-doubling tree
 *                    (intra_fns_new.c:5592-5710, 4697-4751), the binomial
 *                    tree (4907-4954), the recursive-halving tree
 *                    (6341-6407) and the pairwise chain (6473-6500), with the
 *                    operand order fixed by the caller's leaf permutation.
 *   mvx_op_supported the (op, type) validity switch of each op function
 *                    (e.g. global_ops.c:158-161).
 */
#ifndef MVX_HIP_H
#define MVX_HIP_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Combine shapes over leaves y[0..k-1] (a = left operand = inout role):
 *  MVX_SHAPE_TREE : S(q,0)=y[q]; S(q,l)=op(S(q,l-1), S(q+2^(l-1),l-1)) when
 *                   q+2^(l-1) < k, else S(q,l-1); result S(0, ceil(log2 k)).
 *                   For k = 2^L this is ((y0 y1)(y2 y3))...; for other k it is
 *                   the binomial tree truncated at k.
 *  MVX_SHAPE_CHAIN: (((y0 y1) y2) ... y(k-1)). */
#define MVX_SHAPE_TREE  0
#define MVX_SHAPE_CHAIN 1

/* Largest k one combine launch takes. */
#define MVX_COMBINE_KMAX 8

/* 1 if a device kernel exists for (op, dtype); 0 otherwise. */
int mvx_op_supported(int op, int dtype);
/* Bytes of one element as the (op, dtype) kernel reads it (the C pair
 * struct for MAXLOC / MINLOC on a struct type), or 0 if undefined. */
int mvx_op_element_size(int op, int dtype);

/* Bytes per element (the datatype extent) on the device path, or 0. */
int mvx_dtype_extent(int dtype);

/* Derived datatypes (the reference's src/pt2pt type constructors, with its
 * bounds rules: MPI_LB / MPI_UB markers, struct alignment to the largest
 * member, vector -> hvector and indexed -> hindexed reductions, the empty
 * type for count 0):
 *   mvx_type_contiguous  type_contig.c:52-187 (MPI_2INT and contiguous old
 *                        types flattened, :139-146)
 *   mvx_type_vector      type_vec.c:44-110
 *   mvx_type_hvector     type_hvec.c:55-175
 *   mvx_type_indexed     type_ind.c:74-134
 *   mvx_type_hindexed    type_hind.c:57-200
 *   mvx_type_struct      type_struct.c:106-330
 *   mvx_type_commit      type_commit.c:41-143
 *   mvx_type_free        type_free.c:60-105
 * The ops follow global_ops.c: MAXLOC / MINLOC are defined on a count-2
 * contiguous type over INT, LONG, LONG_LONG_INT, SHORT, CHAR, FLOAT, DOUBLE
 * or LONG_DOUBLE (stride-2 {value, loc}, 1387-1503 / 1625-1740) and on a
 * struct type by the type of its first member (read as that type's C pair
 * struct, 1280-1384 / 1520-1620); every other (op, derived type) is 329.
 * Handles are MVX_TYPE_DERIVED_BASE + slot.
 * Return codes: 0, MPI_ERR_COUNT, MPI_ERR_ARG, MPI_ERR_TYPE, 323 (null or
 * unknown old type), MPI_ERR_INTERN (table full); a negative value
 * MVX_SETMSG(class, kind) is a code the reference creates with
 * MPIR_Err_setmsg (the MPI_Type_* wrappers of libmvx.so add the error-ring
 * position). */
#define MVX_TYPE_DERIVED_BASE 256
#define MVX_TYPE_DERIVED_MAX  256
#define MVX_SETMSG(cls, kind) (-((cls) | ((kind) << 6)))
#define MVX_ERR_KIND_TYPE_ARRAY_NULL 13   /* mpi_error.h:143 */
#define MVX_ERR_KIND_ARG_ARRAY_VAL   31   /* mpi_error.h:212 */
int mvx_type_contiguous(int count, int oldtype, int *newtype);
int mvx_type_vector(int count, int blocklen, int stride, int oldtype, int *newtype);
int mvx_type_hvector(int count, int blocklen, long stride, int oldtype, int *newtype);
int mvx_type_indexed(int count, const int *blocklens, const int *indices, int oldtype, int *newtype);
int mvx_type_hindexed(int count, const int *blocklens, const long *indices, int oldtype, int *newtype);
int mvx_type_struct(int count, const int *blocklens, const long *indices, const int *types,
                    int *newtype);
/* 0, or 323 for a null / unknown handle */
int mvx_type_commit(int type);
/* 0 (and *type = MPI_DATATYPE_NULL), 323 (null / unknown), 579 (predefined) */
int mvx_type_free(int *type);
/* Any handle, basic or derived: its old type (the handle itself for a basic
 * type; MPI_INT for MPI_2INT; the flattened old type of a contiguous type;
 * the first member's type of a struct), replication count, extent and size
 * in bytes.  0 or MPI_ERR_TYPE. */
int mvx_type_describe(int type, int *oldtype, int *count, long *extent, long *size);
/* The reference's dte_type (MVX_TK_*), whether elements move whole (dense:
 * the type map covers the extent from offset 0 -- basic types, the padded
 * pair structs, contiguous types of them) or packed, the bounds, and the
 * lowest / one-past-highest byte of one element's type map. */
#define MVX_TK_BASIC    0
#define MVX_TK_CONTIG   1
#define MVX_TK_HVECTOR  2
#define MVX_TK_HINDEXED 3
#define MVX_TK_STRUCT   4
#define MVX_TK_UB       5
#define MVX_TK_LB       6
int mvx_type_layout(int type, int *kind, int *dense, long *lb, long *ub, long *span_lo, long *span_hi);
/* count elements between the type's layout at `origin` (element i at
 * origin + i * extent + type-map offsets) and the packed form (type-map
 * bytes only, size bytes per element), on the device, stream-ordered.
 * Unpacking writes type-map bytes only. */
int mvx_type_pack(int type, const void *origin, void *packed, size_t count, void *hip_stream);
int mvx_type_unpack(int type, const void *packed, void *origin, size_t count, void *hip_stream);

/* inout[i] = in[i] op inout[i], i < n.  Returns MPI_SUCCESS, 329 for an
 * undefined (op, type) pair (as MPIR_ERR_OP_NOT_DEFINED), MPI_ERR_OP for an
 * unknown op handle.  MPI_LONG_DOUBLE / MPI_LONG_DOUBLE_INT and the
 * long-double pairs run an integer emulation of the x87 (mvx_xf80.h). */
int mvx_op_apply(int op, int dtype, const void *in, void *inout, size_t n,
                 void *hip_stream);

/* The Fortran .TRUE. / .FALSE. words MPI_LOGICAL's LAND / LOR / LXOR read
 * and write: a = TO_FLOG(FROM_FLOG(a) op FROM_FLOG(b)), with
 * FROM_FLOG(x) = (x == true_value) and TO_FLOG(v) = v ? true_value :
 * false_value (src/fortran/include/mpi_fort.h:10-19, global_ops.c:646-655,
 * 875-884, 1104-1113).  Replaces the reference's globals MPIR_F_TRUE /
 * MPIR_F_FALSE, which mpir_init_flog sets from the Fortran compiler's
 * literals (initfutil.c:100-102, 189).  The default is 1 / 0, gfortran's
 * literals.  The values go to the current device; call this once per
 * device, before launching. */
int mvx_set_fortran_logical(int true_value, int false_value);

/* dst[i] = shape-combine over leaves; leaf q = srcs[q][i] if fold == NULL or
 * fold[q] == NULL, else op(srcs[q][i], fold[q][i]) (srcs[q] is the inout
 * role).  srcs / fold are HOST arrays of k device pointers; 1 <= k <=
 * MVX_COMBINE_KMAX.  dst may alias srcs[0] (only).  Same return codes as
 * mvx_op_apply, plus MPI_ERR_ARG for a bad k / shape. */
int mvx_op_combine(int op, int dtype, const void *const *srcs,
                   const void *const *fold, int k, int shape, void *dst,
                   size_t n, void *hip_stream);

/* The general form: leaves as above, then a combine program over them:
 *   for level l = 0, 1, 2 (h = 2^l), q ascending:
 *       if tree_mask bit (l*8 + q):  y[q] = op(y[q], y[q+h])
 *   for q = 1 .. k-1:
 *       if chain_mask bit q:         y[0] = op(y[0], y[q])
 *   dst = y[0]
 * TREE = mvx_tree_mask(k), CHAIN = mvx_chain_mask(k); MPI_Scan's chain of
 * balanced trees (intra_scan.c:118-147) is a mix.  A step that reaches past
 * leaf k-1 is MPI_ERR_ARG. */
int mvx_op_program(int op, int dtype, const void *const *srcs,
                   const void *const *fold, int k, unsigned tree_mask,
                   unsigned chain_mask, void *dst, size_t n, void *hip_stream);
unsigned mvx_tree_mask(int k);
unsigned mvx_chain_mask(int k);

/* Launch knobs (0 = keep): grid cap in blocks; non-temporal threshold as
 * log2(bytes touched per launch), -1 = never.  Env: MVX_BLOCK_CAP,
 * MVX_NT_MIN_BYTES.  Defaults: one-pass grid, non-temporal from 64 MiB. */
void mvx_hip_set_launch(int block_cap, int nt_min_bytes_log2);

/* Name of the last kernel launched (for profile attribution in bench.py):
 * a short tag ("sum_f32_k2_nt"), and the template as rocprofv3 reports it
 * ("k_combine<2, float, 2, 4, 1>"). */
const char *mvx_hip_last_kernel(void);
const char *mvx_hip_last_kernel_symbol(void);
/* grid blocks, dynamic LDS bytes (the residency cap) and resident blocks per
 * CU (the runtime's occupancy answer) of the last launch */
void mvx_hip_last_launch(unsigned *blocks, size_t *dynamic_lds, int *blocks_per_cu);

#ifdef __cplusplus
}
#endif
#endif /* MVX_HIP_H */
