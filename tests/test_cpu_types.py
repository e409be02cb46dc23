"""CPU: the derived-datatype engine (vector / hvector / indexed / hindexed /
struct, commit, lb / ub / extent / size).

Pinning: every bound the reference's own datatype tests assert
(examples/test/pt2pt typeub.c, typeub2.c, typeub3.c, typelb.c, structlb.c,
dataalign.c; tests/golden/type_known_answers.json) is reproduced by the
product's engine (libmvx_hip.so, through libmvx.so's MPI_Type_* entry
points) and by the oracle's restatement (oracle/cpu_types.c).  Beyond those,
the two agree on random constructor trees (bounds, size, handles, error
codes); the GPU tests check the type maps through pack / unpack and the
collectives.
"""
import json
import os

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
CASES = json.load(open(os.path.join(HERE, "golden", "type_known_answers.json")))["cases"]


def _make(lib, step, names, mvx):
    """Run one constructor step on the product ('mvx') or oracle ('orc')."""
    def h(x):
        return names[x] if x in names else getattr(mvx, x)
    c = step["ctor"]
    if lib == "mvx":
        if c == "vector":
            return mvx.MPI_Type_vector(step["count"], step["blocklen"], step["stride"], h(step["old"]))
        if c == "hvector":
            return mvx.MPI_Type_hvector(step["count"], step["blocklen"], step["stride"], h(step["old"]))
        if c == "indexed":
            return mvx.MPI_Type_indexed(step["count"], step["blocklens"], step["indices"], h(step["old"]))
        if c == "hindexed":
            return mvx.MPI_Type_hindexed(step["count"], step["blocklens"], step["indices"], h(step["old"]))
        if c == "contiguous":
            return mvx.MPI_Type_contiguous(step["count"], h(step["old"]))
        return mvx.MPI_Type_struct(step["count"], step["blocklens"], step["indices"], [h(t) for t in step["types"]])
    from oracle import oracle as O
    if c == "vector":
        return O.type_vector(step["count"], step["blocklen"], step["stride"], h(step["old"]))
    if c == "hvector":
        return O.type_hvector(step["count"], step["blocklen"], step["stride"], h(step["old"]))
    if c == "indexed":
        return O.type_indexed(step["count"], step["blocklens"], step["indices"], h(step["old"]))
    if c == "hindexed":
        return O.type_hindexed(step["count"], step["blocklens"], step["indices"], h(step["old"]))
    if c == "contiguous":
        return O.type_contiguous(step["count"], h(step["old"]))
    return O.type_struct(step["count"], step["blocklens"], step["indices"], [h(t) for t in step["types"]])


def _bounds_mvx(mvx, h):
    return dict(lb=mvx.MPI_Type_lb(h)[1], ub=mvx.MPI_Type_ub(h)[1], extent=mvx.MPI_Type_extent(h)[1],
                size=mvx.MPI_Type_size(h)[1])


def _bounds_orc(oracle, h):
    rc, lb, ub, ext, size = oracle.type_bounds(h)
    assert rc == 0
    return dict(lb=lb, ub=ub, extent=ext, size=size)


@pytest.mark.parametrize("case", CASES, ids=lambda c: c["test"])
def test_reference_type_known_answers(mvx, oracle, case):
    for lib in ("mvx", "orc"):
        names = {}
        for step in case["steps"]:
            rc, h = _make(lib, step, names, mvx)
            assert rc == 0, (lib, step)
            names[step["name"]] = h
            if lib == "mvx":
                assert mvx.MPI_Type_commit(h) == 0
            else:
                assert oracle.type_commit(h) == 0
        for name, exp in case["expect"].items():
            got = _bounds_mvx(mvx, names[name]) if lib == "mvx" else _bounds_orc(oracle, names[name])
            for k, v in exp.items():
                assert got[k] == v, (lib, case["test"], name, k, got)
        for h in names.values():
            if lib == "mvx":
                assert mvx.MPI_Type_free(h)[0] == 0
            else:
                assert oracle.type_free(h) == 0


BASICS = ["MPI_INT", "MPI_CHAR", "MPI_DOUBLE", "MPI_FLOAT", "MPI_SHORT", "MPI_LONG", "MPI_DOUBLE_INT",
          "MPI_FLOAT_INT", "MPI_SHORT_INT", "MPI_2INT", "MPI_BYTE", "MPI_LONG_DOUBLE",
          "MPI_REAL", "MPI_LOGICAL", "MPI_2INTEGER", "MPI_2REAL", "MPI_2DOUBLE_COMPLEX"]


def _random_step(rng, pool):
    c = rng.choice(["vector", "hvector", "indexed", "hindexed", "struct", "contiguous"])
    old = rng.choice(pool)
    n = int(rng.integers(0, 4))
    if c == "vector":
        return {"ctor": c, "count": n, "blocklen": int(rng.integers(0, 3)), "stride": int(rng.integers(-3, 5)),
                "old": old}
    if c == "hvector":
        return {"ctor": c, "count": n, "blocklen": int(rng.integers(0, 3)), "stride": int(rng.integers(-24, 40)),
                "old": old}
    if c == "contiguous":
        return {"ctor": c, "count": n, "old": old}
    bl = [int(x) for x in rng.integers(0, 3, n)]
    if c == "indexed":
        return {"ctor": c, "count": n, "blocklens": bl, "indices": [int(x) for x in rng.integers(-3, 6, n)],
                "old": old}
    if c == "hindexed":
        return {"ctor": c, "count": n, "blocklens": bl, "indices": [int(x) for x in rng.integers(-16, 48, n)],
                "old": old}
    types = [rng.choice(pool + ["MPI_UB", "MPI_LB"]) for _ in range(n)]
    return {"ctor": "struct", "count": n, "blocklens": bl, "indices": [int(x) for x in rng.integers(-8, 40, n)],
            "types": types}


@pytest.mark.parametrize("seed", range(12))
def test_product_and_oracle_agree_on_random_types(mvx, oracle, seed):
    """Random constructor trees, built on both sides: same codes, handles,
    bounds and sizes at every step, committed or not."""
    rng = np.random.default_rng(seed)
    names_m, names_o, pool, made = {}, {}, list(BASICS), []
    for i in range(40):
        step = _random_step(rng, pool)
        rm, hm = _make("mvx", step, names_m, mvx)
        ro, ho = _make("orc", step, names_o, mvx)
        # the oracle returns -(class | kind << 6) where the reference calls
        # MPIR_Err_setmsg; the product's code adds the error-ring position
        assert (rm & 0x1fff == -ro) if ro < 0 else (rm == ro), (step, rm, ro)
        if rm == 0:
            assert ro == 0 and hm == ho, step
            nm = "t%d" % i
            names_m[nm], names_o[nm] = hm, ho
            pool.append(nm)
            made.append(nm)
            if rng.random() < 0.5:
                assert mvx.MPI_Type_commit(hm) == 0 and oracle.type_commit(ho) == 0
            assert _bounds_mvx(mvx, hm) == _bounds_orc(oracle, ho), step
    for nm in made:
        assert mvx.MPI_Type_free(names_m[nm])[0] == 0
        assert oracle.type_free(names_o[nm]) == 0


def test_constructor_error_codes(mvx, oracle):
    """Argument checks in the reference's order and codes: plain classes for
    vector / hvector / hindexed, MPIR_Err_setmsg codes (class | kind << 6 |
    ring << 13) for indexed blocklens and every struct check."""
    I = mvx.MPI_INT
    assert mvx.MPI_Type_vector(-1, 1, 2, I)[0] == 2
    assert mvx.MPI_Type_vector(2, -1, 2, I)[0] == 12
    assert mvx.MPI_Type_vector(2, 1, 2, mvx.MPI_UB)[0] == 3
    assert mvx.MPI_Type_vector(2, 1, 2, 99)[0] == 323
    assert mvx.MPI_Type_hvector(2, -1, 8, I)[0] == 12
    assert mvx.MPI_Type_hindexed(2, [1, -1], [0, 8], I)[0] == 12
    rc = mvx.MPI_Type_indexed(2, [1, -1], [0, 8], I)[0]
    assert rc & 63 == 12 and (rc >> 6) & 0x7f == 31 and rc >> 13 > 0
    rc = mvx.MPI_Type_struct(-1, [], [], [])[0]
    assert rc & 63 == 2 and (rc >> 6) & 0x7f == 1
    rc = mvx.MPI_Type_struct(2, [1, 1], [0, 4], [I, 0])[0]
    assert rc & 63 == 3 and (rc >> 6) & 0x7f == 13
    assert mvx.MPI_Type_struct(2, [1, 1], [0, 4], [I, 99])[0] == 323
    # the empty type: count or blocks zero -> contiguous(0, MPI_INT)
    for rc, h in (mvx.MPI_Type_vector(0, 3, 4, I), mvx.MPI_Type_struct(2, [0, 0], [0, 4], [I, I]),
                  mvx.MPI_Type_hindexed(1, [0], [8], I)):
        assert rc == 0 and mvx.MPI_Type_extent(h) == (0, 0) and mvx.MPI_Type_size(h) == (0, 0)
        mvx.MPI_Type_free(h)
    # vector with stride == blocklen, or count 1, is contiguous
    rc, h = mvx.MPI_Type_vector(3, 2, 2, I)
    assert mvx.type_layout(h)["kind"] == 1 and mvx.type_layout(h)["dense"] == 1
    mvx.MPI_Type_free(h)


def test_layout_and_density(mvx):
    """What moves whole and what moves packed (include/mvx_hip.h)."""
    I, D = mvx.MPI_INT, mvx.MPI_DOUBLE
    rc, v = mvx.MPI_Type_vector(3, 1, 2, I)           # {0, 8, 16}, extent 20
    L = mvx.type_layout(v)
    assert L["kind"] == 2 and not L["dense"] and (L["span_lo"], L["span_hi"]) == (0, 20)
    rc, s = mvx.MPI_Type_struct(2, [1, 1], [0, 8], [D, I])   # {double; int}: extent 16, size 12
    L = mvx.type_layout(s)
    assert L["kind"] == 4 and not L["dense"] and mvx.MPI_Type_extent(s)[1] == 16
    rc, f = mvx.MPI_Type_struct(2, [1, 1], [0, 4], [mvx.MPI_FLOAT, I])   # {float; int}: dense
    assert mvx.type_layout(f)["dense"] == 1
    assert mvx.hip().mvx_op_element_size(mvx.MPI_MAXLOC, f) == 8
    assert mvx.hip().mvx_op_element_size(mvx.MPI_MAXLOC, s) == 16
    assert mvx.hip().mvx_op_element_size(mvx.MPI_SUM, s) == 0
    # ops on derived types: MAXLOC / MINLOC on a struct by its first member,
    # 329 for everything else (global_ops.c)
    assert mvx.hip().mvx_op_apply(mvx.MPI_MAXLOC, s, None, None, 0, None) == 0
    assert mvx.hip().mvx_op_apply(mvx.MPI_SUM, s, None, None, 0, None) == 329
    assert mvx.hip().mvx_op_apply(mvx.MPI_MAXLOC, v, None, None, 0, None) == 329
    rc, c = mvx.MPI_Type_struct(2, [1, 1], [0, 4], [mvx.MPI_CHAR, I])
    assert mvx.hip().mvx_op_apply(mvx.MPI_MINLOC, c, None, None, 0, None) == 329
    for h in (v, s, f, c):
        mvx.MPI_Type_free(h)


def _describe(mvx, h):
    return (mvx.MPI_Type_extent(h)[1], mvx.MPI_Type_size(h)[1], mvx.MPI_Type_lb(h)[1], mvx.MPI_Type_ub(h)[1])


def _describe_orc(oracle, h):
    rc, lb, ub, ext, size = oracle.type_bounds(h)
    assert rc == 0
    return (ext, size, lb, ub)


def test_free_keeps_types_others_were_built_from(mvx, oracle):
    """MPI_Type_free on a type another type was built from only drops a
    reference (MPIR_Type_dup / MPIR_Type_free, type_util.c:29-130): the
    member stays in place until its last user is freed, so (1) committing a
    struct after freeing a member, and (2) building over a contiguous type
    whose old type was freed -- with another type created in between --
    both see the original layout.  Product and oracle hand out the same
    handles throughout."""
    I, D = mvx.MPI_INT, mvx.MPI_DOUBLE

    def both(ctor, *a):
        r1 = getattr(mvx, "MPI_Type_" + ctor)(*a)
        r2 = getattr(oracle, "type_" + ctor)(*a)
        assert r1 == r2, (ctor, a, r1, r2)
        assert r1[0] == 0
        return r1[1]

    def free(h):
        assert mvx.MPI_Type_free(h) == (0, 0)
        assert oracle.type_free(h) == 0

    # (1) struct([contig(2, INT), INT]) -> free the member -> commit
    c = both("contiguous", 2, I)
    s = both("struct", 2, [1, 1], [0, 8], [c, I])
    free(c)
    other = both("contiguous", 5, D)            # must not reuse c's slot
    assert other != c
    assert mvx.MPI_Type_commit(s) == 0 and oracle.type_commit(s) == 0
    assert _describe(mvx, s) == _describe_orc(oracle, s) == (12, 12, 0, 12)
    assert mvx.type_layout(s)["dense"] == 1
    # (2) contig(2, contig(3, dense struct)) after the struct is freed
    ds = both("struct", 2, [1, 1], [0, 4], [I, mvx.MPI_FLOAT])
    assert mvx.MPI_Type_commit(ds) == 0 and oracle.type_commit(ds) == 0
    t3 = both("contiguous", 3, ds)
    free(ds)
    other2 = both("vector", 2, 1, 3, D)
    assert other2 != ds
    t6 = both("contiguous", 2, t3)
    assert _describe(mvx, t6) == _describe_orc(oracle, t6) == (48, 48, 0, 48)
    # the last reference frees the chain: every slot is reusable afterwards
    for h in (t6, t3, s, other, other2):
        free(h)
    again = [both("contiguous", 1, I) for _ in range(3)]
    assert sorted(again)[0] == min(c, s, ds, t3)
    for h in again:
        free(h)
