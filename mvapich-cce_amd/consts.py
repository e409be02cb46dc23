"""Handle values of the reference ABI (include/mpi.h:64-140, mpi_errno.h:24-49).

Mirrors include/mvx_mpi.h; numpy dtypes give the element layout of each
datatype on x86-64 (the reference's C types; pair structs per initdte.c:74-104).
"""
import numpy as np

MPI_CHAR, MPI_UNSIGNED_CHAR, MPI_BYTE, MPI_SHORT, MPI_UNSIGNED_SHORT = 1, 2, 3, 4, 5
MPI_INT, MPI_UNSIGNED, MPI_LONG, MPI_UNSIGNED_LONG = 6, 7, 8, 9
MPI_FLOAT, MPI_DOUBLE, MPI_LONG_DOUBLE, MPI_LONG_LONG_INT = 10, 11, 12, 13
MPI_LONG_LONG = 13
MPI_FLOAT_INT, MPI_DOUBLE_INT, MPI_LONG_INT, MPI_SHORT_INT, MPI_2INT, MPI_LONG_DOUBLE_INT = 17, 18, 19, 20, 21, 22
MPI_COMPLEX, MPI_DOUBLE_COMPLEX = 23, 24
MPI_UNSIGNED_LONG_LONG = 35

MPI_OP_NULL = 0
MPI_MAX, MPI_MIN, MPI_SUM, MPI_PROD, MPI_LAND, MPI_BAND = 100, 101, 102, 103, 104, 105
MPI_LOR, MPI_BOR, MPI_LXOR, MPI_BXOR, MPI_MINLOC, MPI_MAXLOC = 106, 107, 108, 109, 110, 111

MPI_COMM_WORLD, MPI_COMM_SELF = 91, 92

MPI_SUCCESS, MPI_ERR_BUFFER, MPI_ERR_COUNT, MPI_ERR_TYPE = 0, 1, 2, 3
MPI_ERR_COMM, MPI_ERR_ROOT, MPI_ERR_OP, MPI_ERR_ARG, MPI_ERR_OTHER, MPI_ERR_INTERN = 5, 7, 9, 12, 15, 16
ERR_OP_NOT_DEFINED = 329   # MPIR_ERRCLASS_TO_CODE(MPI_ERR_OP, MPIR_ERR_NOT_DEFINED)

SHAPE_TREE, SHAPE_CHAIN = 0, 1
COLL_ALLREDUCE, COLL_REDUCE, COLL_REDUCE_SCATTER, COLL_SCAN = 1, 2, 3, 4
ALG_NONE, ALG_RECDBL, ALG_RABENSEIFNER, ALG_BINOMIAL, ALG_RS_HALVING, ALG_RS_PAIRWISE, ALG_SCAN_RECDBL = range(7)

PAIR_FLOAT_INT = np.dtype([("v", np.float32), ("l", np.int32)])
PAIR_DOUBLE_INT = np.dtype({"names": ["v", "l"], "formats": [np.float64, np.int32], "offsets": [0, 8], "itemsize": 16})
PAIR_LONG_INT = np.dtype({"names": ["v", "l"], "formats": [np.int64, np.int32], "offsets": [0, 8], "itemsize": 16})
PAIR_SHORT_INT = np.dtype({"names": ["v", "l"], "formats": [np.int16, np.int32], "offsets": [0, 4], "itemsize": 8})
PAIR_2INT = np.dtype([("v", np.int32), ("l", np.int32)])
# x87 80-bit long double in a 16-byte slot (x86-64 numpy longdouble)
PAIR_LONG_DOUBLE_INT = np.dtype({"names": ["v", "l"], "formats": [np.longdouble, np.int32], "offsets": [0, 16],
                                 "itemsize": 32})

NP_DTYPE = {
    MPI_CHAR: np.dtype(np.int8), MPI_UNSIGNED_CHAR: np.dtype(np.uint8), MPI_BYTE: np.dtype(np.uint8),
    MPI_SHORT: np.dtype(np.int16), MPI_UNSIGNED_SHORT: np.dtype(np.uint16),
    MPI_INT: np.dtype(np.int32), MPI_UNSIGNED: np.dtype(np.uint32),
    MPI_LONG: np.dtype(np.int64), MPI_UNSIGNED_LONG: np.dtype(np.uint64), MPI_LONG_LONG_INT: np.dtype(np.int64),
    MPI_FLOAT: np.dtype(np.float32), MPI_DOUBLE: np.dtype(np.float64),
    MPI_COMPLEX: np.dtype(np.complex64), MPI_DOUBLE_COMPLEX: np.dtype(np.complex128),
    MPI_FLOAT_INT: PAIR_FLOAT_INT, MPI_DOUBLE_INT: PAIR_DOUBLE_INT, MPI_LONG_INT: PAIR_LONG_INT,
    MPI_SHORT_INT: PAIR_SHORT_INT, MPI_2INT: PAIR_2INT,
    MPI_LONG_DOUBLE: np.dtype(np.longdouble), MPI_LONG_DOUBLE_INT: PAIR_LONG_DOUBLE_INT,
}

OP_NAMES = {MPI_MAX: "MPI_MAX", MPI_MIN: "MPI_MIN", MPI_SUM: "MPI_SUM", MPI_PROD: "MPI_PROD",
            MPI_LAND: "MPI_LAND", MPI_BAND: "MPI_BAND", MPI_LOR: "MPI_LOR", MPI_BOR: "MPI_BOR",
            MPI_LXOR: "MPI_LXOR", MPI_BXOR: "MPI_BXOR", MPI_MINLOC: "MPI_MINLOC", MPI_MAXLOC: "MPI_MAXLOC"}
TYPE_NAMES = {MPI_CHAR: "MPI_CHAR", MPI_UNSIGNED_CHAR: "MPI_UNSIGNED_CHAR", MPI_BYTE: "MPI_BYTE",
              MPI_SHORT: "MPI_SHORT", MPI_UNSIGNED_SHORT: "MPI_UNSIGNED_SHORT", MPI_INT: "MPI_INT",
              MPI_UNSIGNED: "MPI_UNSIGNED", MPI_LONG: "MPI_LONG", MPI_UNSIGNED_LONG: "MPI_UNSIGNED_LONG",
              MPI_FLOAT: "MPI_FLOAT", MPI_DOUBLE: "MPI_DOUBLE", MPI_LONG_DOUBLE: "MPI_LONG_DOUBLE",
              MPI_LONG_LONG_INT: "MPI_LONG_LONG_INT", MPI_FLOAT_INT: "MPI_FLOAT_INT",
              MPI_DOUBLE_INT: "MPI_DOUBLE_INT", MPI_LONG_INT: "MPI_LONG_INT", MPI_SHORT_INT: "MPI_SHORT_INT",
              MPI_2INT: "MPI_2INT", MPI_LONG_DOUBLE_INT: "MPI_LONG_DOUBLE_INT", MPI_COMPLEX: "MPI_COMPLEX",
              MPI_DOUBLE_COMPLEX: "MPI_DOUBLE_COMPLEX"}

# (op, type) pairs the reference defines (global_ops.c)
_INTS = [MPI_CHAR, MPI_UNSIGNED_CHAR, MPI_SHORT, MPI_UNSIGNED_SHORT, MPI_INT, MPI_UNSIGNED, MPI_LONG,
         MPI_UNSIGNED_LONG, MPI_LONG_LONG_INT]
_FLTS = [MPI_FLOAT, MPI_DOUBLE, MPI_LONG_DOUBLE]
_PAIRS = [MPI_FLOAT_INT, MPI_DOUBLE_INT, MPI_LONG_INT, MPI_SHORT_INT, MPI_2INT, MPI_LONG_DOUBLE_INT]
DEFINED = {
    MPI_MAX: _INTS + _FLTS, MPI_MIN: _INTS + _FLTS,
    MPI_SUM: _INTS + _FLTS + [MPI_COMPLEX, MPI_DOUBLE_COMPLEX],
    MPI_PROD: _INTS + _FLTS + [MPI_COMPLEX, MPI_DOUBLE_COMPLEX],
    MPI_LAND: _INTS + _FLTS, MPI_LOR: _INTS + _FLTS, MPI_LXOR: _INTS + _FLTS,
    MPI_BAND: _INTS + [MPI_BYTE], MPI_BOR: _INTS + [MPI_BYTE], MPI_BXOR: _INTS + [MPI_BYTE],
    MPI_MAXLOC: _PAIRS, MPI_MINLOC: _PAIRS,
}
DEVICE_TYPES = sorted(NP_DTYPE)
