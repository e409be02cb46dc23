"""The body kernels (k_tree_body / k_chain_body, mvx_ops_kern.h): large aligned
full trees and chains over 4 or 8 unfolded leaves run a lean loop at 2
resident blocks per CU; everything else (a head or tail outside the 16-byte
body, misaligned leaves, folded leaves, small launches, MVX_NO_BODY) runs
k_combine.  Both must give the oracle's bits, and the dispatch must pick the
kernel it claims to (mvx_hip_last_kernel_symbol)."""
import numpy as np
import pytest

import mvxtest as T
from plan_exec import SHAPE_CHAIN, SHAPE_TREE, combine_cpu

pytestmark = pytest.mark.gpu

NT_ELEMS = 4 << 20          # 16 MiB of f32 per leaf: a non-temporal launch at k >= 4


def _run(mvx, op, dtype, k, shape, n, offset=0, folded=False, seed=0, ties=0.0):
    import torch
    E = mvx.dtype_info(dtype)[0]
    S = [T.rand_vec(dtype, n, 100 * seed + q) for q in range(k)]
    if ties:
        # equal values across leaves (x87 fields: the loc = min rule), a
        # fraction `ties` of the elements of each leaf copied from the last
        rng = np.random.default_rng(seed + 77)
        for q in range(1, k):
            sel = rng.random(n) < ties
            cur, prev = S[q].view(np.uint8).reshape(n, -1), S[q - 1].view(np.uint8).reshape(n, -1)
            cur[sel, :10] = prev[sel, :10]          # significand + sign / exponent
    F = [T.rand_vec(dtype, n, 100 * seed + 50 + q) if folded and q % 2 else None for q in range(k)]
    # device leaves at byte `offset` into their allocation (offset 4 breaks the
    # 16-byte body for 4-byte types: head elements, k_combine)
    def dev(x):
        b = torch.zeros(x.nbytes + 64, dtype=torch.uint8, device="cuda")
        b[offset:offset + x.nbytes] = torch.from_numpy(x.view(np.uint8).copy()).cuda()
        return b[offset:offset + x.nbytes]
    dS = [dev(x) for x in S]
    dF = [dev(x) if x is not None else None for x in F]
    dst = dev(np.zeros(n, S[0].dtype))
    folds = dF if folded else None
    rc = mvx.op_combine(op, dtype, dS, dst, n, shape=shape, folds=folds)
    torch.cuda.synchronize()
    assert rc == 0
    sym = mvx.last_kernel_symbol()
    ref = combine_cpu(op, dtype, E, [x.view(np.uint8) for x in S],
                      [x.view(np.uint8) if x is not None else None for x in F], shape, n)
    return sym, T.from_dev(dst).view(np.uint8), ref


@pytest.mark.parametrize("k", [4, 8])
@pytest.mark.parametrize("shape", [SHAPE_TREE, SHAPE_CHAIN])
@pytest.mark.parametrize("op,dtype", [(102, 10), (111, 17), (105, 8), (100, 11)])
def test_body_dispatch_and_bits(mvx, op, dtype, k, shape):
    E = mvx.dtype_info(dtype)[0]
    n = NT_ELEMS * 4 // E
    want = "k_tree_body<" if shape == SHAPE_TREE else "k_chain_body<"
    sym, got, ref = _run(mvx, op, dtype, k, shape, n)
    assert sym.startswith(want), sym
    assert np.array_equal(got, ref)
    # a ragged tail (not a whole number of 16-byte chunks) or a shifted
    # start: the general kernel
    for n2, off in ((n + 1 if E < 16 else n, 0), (n, 4 if E == 4 else 8)):
        if (n2, off) == (n, 0):
            continue
        sym, got, ref = _run(mvx, op, dtype, k, shape, n2, offset=off, seed=1)
        assert sym.startswith("k_combine<"), sym
        assert np.array_equal(got, ref)


def test_body_not_used_for_folds_small_or_disabled(mvx, monkeypatch):
    n = NT_ELEMS
    sym, got, ref = _run(mvx, 102, 10, 8, SHAPE_TREE, n, folded=True)
    assert sym.startswith("k_combine<") and np.array_equal(got, ref)
    sym, got, ref = _run(mvx, 102, 10, 8, SHAPE_TREE, 4096)      # cached launch
    assert sym.startswith("k_combine<") and np.array_equal(got, ref)


def test_launch_residency_reported(mvx):
    """mvx_hip_last_launch: the body kernels hold 2 blocks per CU; the plain
    op is uncapped (8)."""
    _run(mvx, 102, 10, 8, SHAPE_TREE, NT_ELEMS)
    blocks, lds, occ = mvx.last_launch()
    assert occ == 2 and blocks == NT_ELEMS // 4 // 512
    _run(mvx, 102, 10, 2, SHAPE_TREE, NT_ELEMS * 8)
    blocks, lds, occ = mvx.last_launch()
    assert occ == 8 and lds == 0


@pytest.mark.parametrize("k", [4, 8])
@pytest.mark.parametrize("op", [110, 111])
def test_long_double_int_loc_pair_body(mvx, op, k):
    """MAXLOC / MINLOC trees on MPI_LONG_DOUBLE_INT (32-byte elements): large
    aligned launches run the lane-pair body (k_pxi_loc_body: lane 2j the x87
    value half, lane 2j+1 the loc half, the compare handed over by DPP) --
    bit for bit against the oracle's x87, ties, NaNs, invalid encodings and
    slot padding included; a start off the 16-byte grid runs k_combine."""
    n = 1 << 19                          # 16 MiB per leaf: a non-temporal launch
    for seed in (0, 1):
        sym, got, ref = _run(mvx, op, 22, k, SHAPE_TREE, n + seed * 4096, seed=seed, ties=0.3)
        assert sym.startswith("k_pxi_loc_body<"), sym
        assert np.array_equal(got, ref)
        # 4 resident blocks per CU (the dynamic LDS reservation)
        assert mvx.last_launch()[2] == 4
    sym, got, ref = _run(mvx, op, 22, k, SHAPE_TREE, n, offset=8, seed=2)
    assert sym.startswith("k_combine<"), sym
    assert np.array_equal(got, ref)


@pytest.mark.parametrize("op", [110, 111])
def test_long_double_int_loc_pair_apply(mvx, oracle, op):
    """The plain op (MPIR_MAXLOC / MINLOC, k = 2) on MPI_LONG_DOUBLE_INT runs
    the lane-pair body too when large and aligned (k_pxi_loc_body<O, 2, 1>):
    bit for bit against the oracle's x87, 30 % tied values (the loc = min
    rule), in place on inout; misaligned operands run k_combine."""
    import torch
    n = 1 << 20                          # 32 MiB per operand: a non-temporal launch
    for seed, off in ((3, 0), (4, 16), (5, 8)):
        a, b = T.rand_vec(22, n, 300 + seed), T.rand_vec(22, n, 400 + seed)
        rng = np.random.default_rng(seed)
        sel = rng.random(n) < 0.3
        a.view(np.uint8).reshape(n, -1)[sel, :10] = b.view(np.uint8).reshape(n, -1)[sel, :10]
        ref = T.clone(b)
        oracle.op(op, 22, a.view(np.uint8), ref.view(np.uint8), n)
        buf_a = torch.zeros(n * 32 + 64, dtype=torch.uint8, device="cuda")
        buf_b = torch.zeros(n * 32 + 64, dtype=torch.uint8, device="cuda")
        da, db = buf_a[off:off + n * 32], buf_b[off:off + n * 32]
        da.copy_(torch.from_numpy(a.view(np.uint8).copy()))
        db.copy_(torch.from_numpy(b.view(np.uint8).copy()))
        assert mvx.op_apply(op, 22, da, db, n) == 0
        torch.cuda.synchronize()
        sym = mvx.last_kernel_symbol()
        # 16-byte aligned (offset 0 or 16): the pair body; offset 8: no whole
        # element starts on the 16-byte grid, the element path
        assert sym.startswith("k_pxi_loc_body<%d, 2, " % (11 if op == 111 else 10)) if off % 16 == 0 else \
            sym.startswith("k_combine<"), sym
        assert np.array_equal(db.cpu().numpy(), ref.view(np.uint8))


@pytest.mark.parametrize("k", [2, 4, 8])
@pytest.mark.parametrize("shape", [SHAPE_TREE, SHAPE_CHAIN])
@pytest.mark.parametrize("op,dtype", [(102, 1), (103, 2), (100, 1), (101, 1), (100, 2), (101, 2), (104, 1),
                                      (106, 2), (108, 1), (105, 3), (107, 3), (109, 3)])
def test_one_byte_types_swar(mvx, op, dtype, k, shape):
    """1-byte elements run the SWAR chunk op (four bytes per 32-bit word:
    wrapping SUM / PROD, signed and unsigned MAX / MIN, the logical ops'
    0 / 1 bytes, the bitwise ops) in every kernel family -- the plain op,
    the masked program, the tree and chain bodies -- bit for bit against the
    oracle, at a non-temporal size and at a small one with head / tail
    elements around the 16-byte body."""
    E = mvx.dtype_info(dtype)[0]
    assert E == 1
    for n, off in ((NT_ELEMS * 4 + 3, 0), (4099, 5)):
        sym, got, ref = _run(mvx, op, dtype, k, shape, n, offset=off, seed=k)
        assert np.array_equal(got, ref), (sym, n)


@pytest.mark.parametrize("shape", [SHAPE_TREE, SHAPE_CHAIN])
@pytest.mark.parametrize("folded", [False, True])
@pytest.mark.parametrize("op,dtype", [(102, 10), (105, 8), (111, 17)])
def test_three_leaf_programs_on_four_leaf_kernel(mvx, op, dtype, shape, folded):
    """Programs over three leaves (and four with folded leaves) run the
    4-leaf program kernel at U = 2 (KSet::prog4), non-temporal size: the
    launched template names KMAX 4, and the bits are the oracle's."""
    E = mvx.dtype_info(dtype)[0]
    n = NT_ELEMS * 4 // E
    for k in (3, 4):
        if k == 4 and not folded:
            continue                      # the plain 4-leaf tree / chain runs its body kernel
        sym, got, ref = _run(mvx, op, dtype, k, shape, n, folded=folded)
        assert sym.startswith("k_combine<") and ", 4, 2, 1, 0>" in sym, sym
        assert np.array_equal(got, ref)


@pytest.mark.parametrize("k", [5, 6, 7])
@pytest.mark.parametrize("op,dtype", [(102, 10), (111, 17), (105, 8), (100, 11), (103, 11)])
def test_five_to_seven_leaf_chains_on_the_eight_leaf_body(mvx, op, dtype, k):
    """Chains of 5-7 leaves (the pairwise Reduce_scatter at p = 5..7) run the
    8-leaf chain body with a run-time leaf count (k_chain_body<..., 8, 2>,
    P.k) where the launch is large and aligned, and its masked program
    otherwise -- bit for bit against the CPU replay either way; trees of 5-7
    leaves keep the masked program."""
    E = mvx.dtype_info(dtype)[0]
    n = NT_ELEMS * 4 // E
    sym, got, ref = _run(mvx, op, dtype, k, SHAPE_CHAIN, n, seed=k)
    assert sym.startswith("k_chain_body<") and ", 8, 2>" in sym, sym
    assert np.array_equal(got, ref)
    sym, got, ref = _run(mvx, op, dtype, k, SHAPE_CHAIN, n, offset=4 if E == 4 else 8, seed=k + 1)
    assert sym.startswith("k_combine<"), sym
    assert np.array_equal(got, ref)
    sym, got, ref = _run(mvx, op, dtype, k, SHAPE_TREE, n, seed=k + 2)
    assert sym.startswith("k_combine<"), sym
    assert np.array_equal(got, ref)
