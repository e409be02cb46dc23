/*
 * mvx_mpi.h -- MPI-1.2 handle values, error classes and callback types for
 * the reduction path.
 *
 * The numeric values are the reference's ABI, so a caller compiled against
 * the reference mpi.h passes the same integers to this library:
 *   datatypes     reference include/mpi.h:64-115
 *   ops           reference include/mpi.h:127-140
 *   error classes reference include/mpi_errno.h:24-49
 *   MPI_User_function  reference include/mpi.h:206
 *   error-code layout (class | kind << 6)  reference include/mpi_error.h:101-102
 *
 * Only the subset that the reduction path uses is declared here; the rest of
 * MPI (pt2pt, groups, topologies, I/O) is out of scope.
 */
#ifndef MVX_MPI_H
#define MVX_MPI_H

#ifdef __cplusplus
extern "C" {
#endif

typedef int MPI_Datatype;
typedef int MPI_Op;
typedef int MPI_Comm;
typedef long MPI_Aint;      /* x86-64 LP64, the reference build's address int */

#define MPI_COMM_WORLD 91   /* reference include/mpi.h:119-120 */
#define MPI_BOTTOM ((void *)0)   /* reference include/mpi.h:179 */
#define MPI_COMM_SELF  92

/* Datatypes: reference include/mpi.h:64-115 (MPI_DATATYPE_NULL :158) */
#define MPI_DATATYPE_NULL      ((MPI_Datatype)0)
#define MPI_CHAR               ((MPI_Datatype)1)
#define MPI_UNSIGNED_CHAR      ((MPI_Datatype)2)
#define MPI_BYTE               ((MPI_Datatype)3)
#define MPI_SHORT              ((MPI_Datatype)4)
#define MPI_UNSIGNED_SHORT     ((MPI_Datatype)5)
#define MPI_INT                ((MPI_Datatype)6)
#define MPI_UNSIGNED           ((MPI_Datatype)7)
#define MPI_LONG               ((MPI_Datatype)8)
#define MPI_UNSIGNED_LONG      ((MPI_Datatype)9)
#define MPI_FLOAT              ((MPI_Datatype)10)
#define MPI_DOUBLE             ((MPI_Datatype)11)
#define MPI_LONG_DOUBLE        ((MPI_Datatype)12)
#define MPI_LONG_LONG_INT      ((MPI_Datatype)13)
#define MPI_LONG_LONG          ((MPI_Datatype)13)
#define MPI_PACKED             ((MPI_Datatype)14)
#define MPI_LB                 ((MPI_Datatype)15)
#define MPI_UB                 ((MPI_Datatype)16)
#define MPI_FLOAT_INT          ((MPI_Datatype)17)
#define MPI_DOUBLE_INT         ((MPI_Datatype)18)
#define MPI_LONG_INT           ((MPI_Datatype)19)
#define MPI_SHORT_INT          ((MPI_Datatype)20)
#define MPI_2INT               ((MPI_Datatype)21)
#define MPI_LONG_DOUBLE_INT    ((MPI_Datatype)22)
/* The Fortran types (mpi.h:101-113).  A Fortran-enabled build registers them
 * in MPI_Init (initutil.c:421-422 -> MPIR_InitFortranDatatypes,
 * src/fortran/src/initfutil.c:220-349), for C callers too.  The layout is
 * x86-64 with gfortran: INTEGER / REAL / LOGICAL are 4 bytes,
 * DOUBLE PRECISION is 8 bytes.
 *   INTEGER, REAL, DOUBLE_PRECISION  the int / float / double kernels
 *                                    (dte_type MPIR_INT / FLOAT / DOUBLE)
 *   LOGICAL                          dte_type MPIR_LOGICAL (global_ops.c:646-655 ...)
 *   2INTEGER / 2REAL / 2DOUBLE_PRECISION / 2COMPLEX / 2DOUBLE_COMPLEX
 *                                    contiguous(2, INTEGER / FLOAT / DOUBLE /
 *                                    COMPLEX / DOUBLE_COMPLEX) */
#define MPI_COMPLEX            ((MPI_Datatype)23)
#define MPI_DOUBLE_COMPLEX     ((MPI_Datatype)24)
#define MPI_LOGICAL            ((MPI_Datatype)25)
#define MPI_REAL               ((MPI_Datatype)26)
#define MPI_DOUBLE_PRECISION   ((MPI_Datatype)27)
#define MPI_INTEGER            ((MPI_Datatype)28)
#define MPI_2INTEGER           ((MPI_Datatype)29)
#define MPI_2COMPLEX           ((MPI_Datatype)30)
#define MPI_2DOUBLE_COMPLEX    ((MPI_Datatype)31)
#define MPI_2REAL              ((MPI_Datatype)32)
#define MPI_2DOUBLE_PRECISION  ((MPI_Datatype)33)
#define MPI_CHARACTER          ((MPI_Datatype)1)
#define MPI_UNSIGNED_LONG_LONG ((MPI_Datatype)35)

/* Ops: reference include/mpi.h:127-140 */
#define MPI_OP_NULL ((MPI_Op)0)
#define MPI_MAX     ((MPI_Op)100)
#define MPI_MIN     ((MPI_Op)101)
#define MPI_SUM     ((MPI_Op)102)
#define MPI_PROD    ((MPI_Op)103)
#define MPI_LAND    ((MPI_Op)104)
#define MPI_BAND    ((MPI_Op)105)
#define MPI_LOR     ((MPI_Op)106)
#define MPI_BOR     ((MPI_Op)107)
#define MPI_LXOR    ((MPI_Op)108)
#define MPI_BXOR    ((MPI_Op)109)
#define MPI_MINLOC  ((MPI_Op)110)
#define MPI_MAXLOC  ((MPI_Op)111)

/* Error classes: reference include/mpi_errno.h:24-49 */
#define MPI_SUCCESS      0
#define MPI_ERR_BUFFER   1
#define MPI_ERR_COUNT    2
#define MPI_ERR_TYPE     3
#define MPI_ERR_COMM     5
#define MPI_ERR_ROOT     7
#define MPI_ERR_OP       9
#define MPI_ERR_ARG     12
#define MPI_ERR_UNKNOWN 13
#define MPI_ERR_OTHER   15
#define MPI_ERR_INTERN  16

/* Error codes = class | kind << MVX_ERR_CLASS_BITS (mpi_error.h:101-102). */
#define MVX_ERR_CLASS_BITS 6
#define MVX_ERRCLASS_TO_CODE(cls, kind) ((cls) | ((kind) << MVX_ERR_CLASS_BITS))
/* MPIR_ERR_OP_NOT_DEFINED, global_ops.c:54 -> 329 */
#define MVX_ERR_OP_NOT_DEFINED MVX_ERRCLASS_TO_CODE(MPI_ERR_OP, 5)
/* Buffer alias as returned by the reference build -> 8641 */
#define MVX_ERR_BUFFER_ALIAS   8641
/* Op free of MPI_OP_NULL (opfree.c:64) and of a permanent op (opfree.c:72);
 * kinds from mpi_error.h:176,199 */
#define MVX_ERR_OP_NULL        MVX_ERRCLASS_TO_CODE(MPI_ERR_OP, 3)
#define MVX_ERR_PERM_OP        MVX_ERRCLASS_TO_CODE(MPI_ERR_ARG, 13)
/* MPIR_TEST_DTYPE of a null / unknown handle (mpid/ch2/datatype.h:64-65) and
 * MPI_Type_free of a predefined type (type_free.c:93-96); mpi_error.h:137-139 */
#define MVX_ERR_TYPE_NULL      MVX_ERRCLASS_TO_CODE(MPI_ERR_TYPE, 5)
#define MVX_ERR_PERM_TYPE      MVX_ERRCLASS_TO_CODE(MPI_ERR_TYPE, 9)

/* User combination function: inoutvec[i] = invec[i] op inoutvec[i]
 * (reference include/mpi.h:206, opcreate.c:47). */
typedef void (MPI_User_function)(void *invec, void *inoutvec, int *len,
                                 MPI_Datatype *datatype);

#ifdef __cplusplus
}
#endif
#endif /* MVX_MPI_H */
