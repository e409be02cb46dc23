"""GPU parity: libmvx_hip.so's op / combine kernels against the CPU oracle.

The oracle (oracle/cpu_ops.c) restates src/coll/global_ops.c; every case
here is bit-exact except NaN payloads of float SUM/PROD results, which the
reference does not pin either (x86 and gfx950 both return a quiet NaN; the
payload is compared as "is NaN" -- the 1-ulp-class tolerance of the north
star, written here as: identical bits, or both NaN).
"""
import numpy as np
import pytest

import mvxtest as T

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("op", T.ALL_OPS)
@pytest.mark.parametrize("dtype", T.ALL_TYPES)
def test_op_apply_every_pair(mvx, oracle, op, dtype):
    """MPIR_<OP> on every datatype: defined pairs bit-exact, undefined -> 329."""
    n = 4099
    rc_ref = T.oracle_rc(oracle, op, dtype)
    a, b = T.rand_vec(dtype, n, 11), T.rand_vec(dtype, n, 12)
    da, db = T.to_dev(a), T.to_dev(b)
    rc = mvx.op_apply(op, dtype, da, db, n)
    assert rc == rc_ref, (rc, rc_ref)
    if rc:
        assert T.bytes_equal(T.from_dev(db), b), "undefined op must leave inout alone"
        return
    ref = T.clone(b)
    oracle.op(op, dtype, a.view(np.uint8), ref.view(np.uint8), n)
    T.assert_same(op, dtype, T.from_dev(db), ref)


@pytest.mark.parametrize("dtype", [10, 11, 6, 8, 1, 4, 17, 18, 19, 20, 21, 23, 24, 12, 22])
@pytest.mark.parametrize("n", [0, 1, 2, 3, 5, 17, 255, 256, 1023, 65537])
@pytest.mark.parametrize("shift", [(0, 0), (1, 1), (3, 3), (1, 2), (0, 5)])
def test_op_apply_sizes_and_alignment(mvx, oracle, dtype, n, shift):
    """Head/tail elements around the 16-byte body, and operands whose
    alignments differ (scalar path)."""
    op = mvx.MPI_MAXLOC if dtype in T.PAIRS else mvx.MPI_SUM
    a, b = T.rand_vec(dtype, n + 8, 21), T.rand_vec(dtype, n + 8, 22)
    da, db = T.to_dev(a), T.to_dev(b)
    E = a.dtype.itemsize
    rc = mvx.op_apply(op, dtype, da.data_ptr() + shift[0] * E, db.data_ptr() + shift[1] * E, n)
    assert rc == 0
    ref = T.clone(b)
    oracle.op(op, dtype, a[shift[0]:].view(np.uint8), ref[shift[1]:].view(np.uint8), n)
    T.assert_same(op, dtype, T.from_dev(db), ref)


@pytest.mark.parametrize("op,dtype", [(102, 10), (100, 10), (101, 11), (103, 6), (111, 17), (110, 18),
                                      (105, 8), (108, 4), (102, 24), (103, 23), (111, 20), (110, 21),
                                      (102, 12), (100, 12), (111, 22)])
@pytest.mark.parametrize("k", [1, 2, 3, 4, 5, 6, 7, 8])
@pytest.mark.parametrize("shape", [0, 1])
@pytest.mark.parametrize("folded", [False, True])
def test_combine_tree_chain(mvx, oracle, op, dtype, k, shape, folded):
    """k-leaf combine (with and without pre-folded leaves) = the same
    sequence of oracle op calls."""
    from plan_exec import combine_cpu
    n = 3001
    leaves = [T.rand_vec(dtype, n, 100 + q) for q in range(k)]
    folds = [T.rand_vec(dtype, n, 200 + q) if (folded and q % 2 == 0) else None for q in range(k)]
    dl = [T.to_dev(x) for x in leaves]
    dfo = [T.to_dev(x) if x is not None else None for x in folds]
    dst = T.to_dev(np.zeros_like(leaves[0]))
    rc = mvx.op_combine(op, dtype, dl, dst, n, shape=shape, folds=dfo)
    assert rc == 0
    E = leaves[0].dtype.itemsize
    ref = combine_cpu(op, dtype, E, [x.view(np.uint8) for x in leaves],
                      [x.view(np.uint8) if x is not None else None for x in folds], shape, n)
    T.assert_same(op, dtype, T.from_dev(dst), ref.view(leaves[0].dtype))


def test_combine_dst_aliases_leaf0(mvx, oracle):
    from plan_exec import combine_cpu
    n = 10007
    leaves = [T.rand_vec(10, n, q) for q in range(8)]
    dl = [T.to_dev(x) for x in leaves]
    rc = mvx.op_combine(102, 10, dl, dl[0], n, shape=0)
    assert rc == 0
    ref = combine_cpu(102, 10, 4, [x.view(np.uint8) for x in leaves], None, 0, n)
    T.assert_same(102, 10, T.from_dev(dl[0]), ref.view(np.float32))


def test_combine_bad_args(mvx):
    import torch
    x = torch.zeros(16, device="cuda")
    assert mvx.op_combine(102, 10, [x] * 9, x, 16) == mvx.MPI_ERR_ARG
    assert mvx.op_combine(102, 10, [x, x], x, 16, shape=7) == mvx.MPI_ERR_ARG
    assert mvx.op_combine(99, 10, [x, x], x, 16) == mvx.MPI_ERR_OP
    assert mvx.op_combine(105, 10, [x, x], x, 16) == 329


@pytest.mark.parametrize("name,op", [("MPIR_SUM", 102), ("MPIR_MAXF", 100), ("MPIR_MINLOC", 110),
                                     ("MPIR_BXOR", 109), ("MPIR_LAND", 104)])
def test_mpir_user_function_symbols(mvx, oracle, name, op):
    """The predefined ops keep their MPI_User_function ABI (global_ops.c)."""
    dtype = mvx.MPI_DOUBLE_INT if op == 110 else (mvx.MPI_INT if op == 109 else mvx.MPI_DOUBLE)
    n = 777
    a, b = T.rand_vec(dtype, n, 1), T.rand_vec(dtype, n, 2)
    da, db = T.to_dev(a), T.to_dev(b)
    mvx.op_errno()
    mvx.MPIR_call(name, da, db, n, dtype)
    assert mvx.op_errno() == 0
    ref = T.clone(b)
    oracle.op(op, dtype, a.view(np.uint8), ref.view(np.uint8), n)
    T.assert_same(op, dtype, T.from_dev(db), ref)
    # an undefined pair sets the op errno and leaves the data alone
    mvx.MPIR_call("MPIR_BAND", da, db, n, mvx.MPI_DOUBLE)
    assert mvx.op_errno() == 329


LDI = 22   # MPI_LONG_DOUBLE_INT, 32-byte elements


def _place(x, kind):
    """host (pageable numpy), pin (page-locked torch tensor) or dev"""
    import torch
    if kind == "dev":
        return T.to_dev(x)
    if kind == "pin":
        return torch.from_numpy(x.view(np.uint8).copy()).pin_memory()
    return T.clone(x)


def _back(y, kind):
    if kind == "dev":
        return T.from_dev(y)
    if kind == "pin":
        return y.numpy()
    return np.asarray(y)


@pytest.mark.parametrize("n", [1, 1000, 9 * 1024 * 1024 + 5, 17 * 1024 * 1024 + 3, 16 * 1024 * 1024 + 262145])
@pytest.mark.parametrize("where", ["host-host", "dev-host", "host-dev", "pin-pin", "pin-host", "host-pin",
                                   "dev-pin"])
def test_mpir_host_buffers(mvx, oracle, n, where):
    """MPI user buffers live in host memory: pageable operands stream
    through HBM (chunked, through pinned bounce slots; H2D / kernel / D2H
    overlapped), page-locked ones are read and written in place by the same
    kernel when no operand is pageable (zero copy), DMA'd directly otherwise."""
    a, b = T.rand_vec(10, n, 5), T.rand_vec(10, n, 6)
    ref = T.clone(b)
    oracle.op(102, 10, a.view(np.uint8), ref.view(np.uint8), n)
    ki, ko = where.split("-")
    ia, io = _place(a, ki), _place(b, ko)
    mvx.op_errno()
    mvx.MPIR_call("MPIR_SUM", ia, io, n, mvx.MPI_FLOAT)
    assert mvx.op_errno() == 0
    T.assert_same(102, 10, _back(io, ko).view(np.uint8), ref)


@pytest.mark.parametrize("where", ["host-host", "pin-host", "host-pin"])
@pytest.mark.parametrize("dtype,op", [(13, 109), (18, 111), (12, 100), (8, 105), (LDI, 110)])
def test_mpir_host_buffers_types(mvx, oracle, where, dtype, op):
    """Other element sizes (8, 16 and 32-byte elements; the padding of the
    pair structs is carried from inout) over several chunks, operands offset
    by one element from their allocation (misaligned against the bounce)."""
    name = {100: "MPIR_MAXF", 105: "MPIR_BAND", 109: "MPIR_BXOR", 110: "MPIR_MINLOC", 111: "MPIR_MAXLOC"}
    E = mvx.dtype_info(dtype)[0]
    n = (80 << 20) // E + 7          # over HOP_BOUNCE_MIN: the bounce pipeline for pageable operands
    a8 = T.rand_vec(dtype, n + 1, 7).view(np.uint8)[E:]
    b8 = T.rand_vec(dtype, n + 1, 8).view(np.uint8)[E:]
    ref = b8.copy()
    oracle.op(op, dtype, a8.copy(), ref, n)
    ki, ko = where.split("-")
    ia, io = _place(a8, ki), _place(b8, ko)
    mvx.op_errno()
    mvx.MPIR_call(name[op], ia, io, n, dtype)
    assert mvx.op_errno() == 0
    assert np.array_equal(_back(io, ko).view(np.uint8), ref)


@pytest.mark.parametrize("shift", [0, 4, 12])
@pytest.mark.parametrize("dtype,op", [(10, 102), (13, 109), (LDI, 110), (12, 100)])
def test_mpir_pinned_zero_copy(mvx, oracle, dtype, op, shift):
    """Page-locked operands on both sides (or one device operand): the op
    kernel reads and writes them in place over PCIe (csrc/mvx_hostop.c,
    zero copy).  Interior pointers of pinned allocations, shifted by 0 / 4 /
    12 bytes against each other's 16-byte alignment (the kernel's element
    path), ragged counts, bytes outside the vector untouched."""
    import torch
    name = {100: "MPIR_MAXF", 102: "MPIR_SUM", 109: "MPIR_BXOR", 110: "MPIR_MINLOC"}
    E = mvx.dtype_info(dtype)[0]
    n = (3 << 20) // E + 5
    a8 = T.rand_vec(dtype, n + 2, 17).view(np.uint8)
    b8 = T.rand_vec(dtype, n + 2, 18).view(np.uint8)
    pa = torch.from_numpy(np.concatenate([np.zeros(64, np.uint8), a8])).pin_memory()
    pb = torch.from_numpy(np.concatenate([np.zeros(64, np.uint8), b8])).pin_memory()
    before = pb.numpy().copy()
    ia = pa[64 + E:64 + E + n * E]                        # one element in
    io = pb[64 + E + shift:64 + E + shift + n * E]        # and shifted
    ref = io.numpy().copy()
    oracle.op(op, dtype, ia.numpy().copy(), ref, n)
    mvx.op_errno()
    mvx.MPIR_call(name[op], ia, io, n, dtype)
    assert mvx.op_errno() == 0
    assert np.array_equal(io.numpy(), ref)
    whole = pb.numpy()
    lo, hi = 64 + E + shift, 64 + E + shift + n * E
    assert np.array_equal(whole[:lo], before[:lo]) and np.array_equal(whole[hi:], before[hi:])
    # device `in`, page-locked `inout`
    io2 = torch.from_numpy(b8[:n * E].copy()).pin_memory()
    ref2 = io2.numpy().copy()
    oracle.op(op, dtype, a8[:n * E].copy(), ref2, n)
    mvx.MPIR_call(name[op], T.to_dev(a8[:n * E]), io2, n, dtype)
    assert mvx.op_errno() == 0
    assert np.array_equal(io2.numpy(), ref2)


def test_special_values_float(mvx, oracle):
    """NaN stickiness of MAX/MIN (coll.h:14-19), signed zeros, infinities,
    denormals and NaN-vs-value in MAXLOC, elementwise against the oracle."""
    sp = np.array([np.nan, -np.nan, np.inf, -np.inf, 0.0, -0.0, 1.0, -1.0, 1e-45, -1e-45, 1e-40,
                   3.4e38, -3.4e38, 1.17549435e-38], np.float32)
    a = np.repeat(sp, len(sp)).astype(np.float32)
    b = np.tile(sp, len(sp)).astype(np.float32)
    n = a.size
    for op in (100, 101, 102, 103, 104, 106, 108):
        da, db = T.to_dev(a), T.to_dev(b)
        assert mvx.op_apply(op, 10, da, db, n) == 0
        ref = T.clone(b)
        oracle.op(op, 10, a.view(np.uint8), ref.view(np.uint8), n)
        T.assert_same(op, 10, T.from_dev(db), ref)
    pa = np.zeros(n, mvx.PAIR_FLOAT_INT)
    pb = np.zeros(n, mvx.PAIR_FLOAT_INT)
    pa["v"], pb["v"] = a, b
    pa["l"], pb["l"] = np.arange(n), np.arange(n)[::-1]
    for op in (110, 111):
        da, db = T.to_dev(pa), T.to_dev(pb)
        assert mvx.op_apply(op, 17, da, db, n) == 0
        ref = T.clone(pb)
        oracle.op(op, 17, pa.view(np.uint8), ref.view(np.uint8), n)
        T.assert_same(op, 17, T.from_dev(db), ref)


def test_integer_wrap(mvx, oracle):
    """Signed overflow wraps exactly as the reference's x86 build."""
    for dtype, npt in ((6, np.int32), (4, np.int16), (1, np.int8), (8, np.int64)):
        info = np.iinfo(npt)
        a = np.array([info.max, info.min, info.max, -1, info.min], npt)
        b = np.array([1, -1, info.max, info.min, info.min], npt)
        for op in (102, 103):
            da, db = T.to_dev(a), T.to_dev(b)
            assert mvx.op_apply(op, dtype, da, db, a.size) == 0
            ref = T.clone(b)
            oracle.op(op, dtype, a.view(np.uint8), ref.view(np.uint8), a.size)
            assert T.bytes_equal(T.from_dev(db), ref)


@pytest.mark.parametrize("dist", [0, 1])
def test_c2_headline_256mib_sum_f32(mvx, oracle, dist):
    """Config 2 at full size: 256 MiB MPI_SUM on MPI_FLOAT, bit-exact, on
    both SURVEY.md 8(d) inputs: mixed sign with an exponent spread (0) and
    U[0,1) (1)."""
    n = 64 * 1024 * 1024
    a = np.empty(n, np.float32)
    b = np.empty(n, np.float32)
    oracle.fill(a, n, dist, 0)
    oracle.fill(b, n, dist, 1)
    da, db = T.to_dev(a), T.to_dev(b)
    assert mvx.op_apply(102, 10, da, db, n) == 0
    oracle.op(102, 10, a.view(np.uint8), b.view(np.uint8), n)
    got = T.from_dev(db)
    assert np.array_equal(got.view(np.uint32), b.view(np.uint32))


@pytest.mark.parametrize("op,dtype", [(100, 12), (101, 12), (102, 12), (103, 12), (104, 12), (106, 12), (108, 12),
                                      (110, 22), (111, 22)])
def test_x87_long_double_fuzz(mvx, oracle, op, dtype):
    """MPI_LONG_DOUBLE / MPI_LONG_DOUBLE_INT: the device's x87 emulation
    (mvx_xf80.h) against the oracle's x87 unit on every operand class --
    denormals, pseudo-denormals, unnormals, pseudo-NaNs, NaN significand
    ties, round-to-even ties, underflow and overflow -- byte-exact
    including NaN payloads and the untouched slot padding."""
    n = 1 << 20
    if dtype == 12:
        b, a = T.xf_operands(n, op)
    else:
        b, a = T.xfi_operands(n, op)
    da, db = T.to_dev(b), T.to_dev(a)
    assert mvx.op_apply(op, dtype, da, db, n) == 0
    ref = T.clone(a)
    assert oracle.op(op, dtype, b.view(np.uint8), ref.view(np.uint8), n) == 0
    got = T.from_dev(db)
    w = ref.dtype.itemsize
    g, r = got.view(np.uint8).reshape(n, w), ref.view(np.uint8).reshape(n, w)
    bad = np.nonzero((g != r).any(1))[0]
    assert bad.size == 0, "%d differ; first %d: got %s ref %s" % (bad.size, bad[0], g[bad[0]].tobytes().hex(),
                                                                 r[bad[0]].tobytes().hex())


@pytest.mark.parametrize("flog", [(-1, 0), (7, 3)])
def test_logical_with_other_fortran_literals(mvx, oracle, flog):
    """MPI_LOGICAL under another compiler's .TRUE. / .FALSE. words
    (mvx_set_fortran_logical, the reference's MPIR_F_TRUE / MPIR_F_FALSE):
    the op and an 8-leaf combine against the oracle with the same words."""
    from plan_exec import combine_cpu
    n = 70001
    words = np.array([flog[0], flog[1], 0, 1, -1, 2], np.int32)
    rng = np.random.default_rng(3)
    try:
        assert mvx.set_fortran_logical(*flog) == 0
        oracle.set_fortran_logical(*flog)
        for op in (104, 106, 108):
            a, b = rng.choice(words, n), rng.choice(words, n)
            db = T.to_dev(b)
            assert mvx.op_apply(op, 25, T.to_dev(a), db, n) == 0
            ref = T.clone(b)
            oracle.op(op, 25, a.view(np.uint8), ref.view(np.uint8), n)
            assert T.bytes_equal(T.from_dev(db), ref), op
            leaves = [rng.choice(words, n) for _ in range(8)]
            dst = T.to_dev(np.zeros(n, np.int32))
            assert mvx.op_combine(op, 25, [T.to_dev(x) for x in leaves], dst, n, shape=0) == 0
            ref = combine_cpu(op, 25, 4, [x.view(np.uint8) for x in leaves], [None] * 8, 0, n)
            assert T.bytes_equal(T.from_dev(dst), ref), op
    finally:
        mvx.set_fortran_logical(1, 0)
        oracle.set_fortran_logical(1, 0)
