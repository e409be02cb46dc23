"""The algorithm-choice constants, pinned to the reference's own source.

The oracle (oracle/coll_sim.c) and the product (csrc/mvx_plan.c) each carry
a typed copy of intra_fns_new.c's `coll_table`, its row indices, the
Reduce_scatter switch points and the power-of-two / lgn loop.  A misreading
copied into both would agree with itself, and the reference's known-answer
tests (count 10 at p = 2 / 4) reach only some table cells.  This test reads
the values out of /root/reference/src/coll/intra_fns_new.c itself
(:30-40, :123-132, and the lgn loops of intra_Reduce :4539-4612 and
intra_Allreduce :5472-5538) and checks both copies against them.  It ships
nothing from the reference and skips where the reference tree is absent.
"""
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference/src/coll/intra_fns_new.c"
COPIES = [os.path.join(ROOT, "oracle", "coll_sim.c"), os.path.join(ROOT, "mvapich-cce_amd", "csrc", "mvx_plan.c")]


def _strip_comments(text):
    return re.sub(r"//[^\n]*", "", re.sub(r"/\*.*?\*/", "", text, flags=re.S))


def _defines(text):
    return {m.group(1): int(m.group(2)) for m in re.finditer(r"#define\s+(\w+)\s+(-?\d+)\b", text)}


def _ints(body):
    return [int(x) for x in re.findall(r"-?\d+", body)]


@pytest.fixture(scope="module")
def ref():
    if not os.path.exists(REF):
        pytest.skip("reference tree not present")
    with open(REF, errors="replace") as f:
        return _strip_comments(f.read())


def test_coll_table_matches_reference(ref):
    d = _defines(ref)
    m = re.search(r"int\s+coll_table\s*\[\s*COLL_COUNT\s*\]\s*\[\s*COLL_SIZE\s*\+\s*1\s*\]\s*=\s*\{(.*?)\};", ref, re.S)
    assert m, "coll_table not found"
    table = _ints(m.group(1))
    assert len(table) == d["COLL_COUNT"] * (d["COLL_SIZE"] + 1)
    for path in COPIES:
        src = _strip_comments(open(path).read())
        c = re.search(r"coll_table_flat\s*\[[^\]]*\]\s*=\s*\{(.*?)\};", src, re.S)
        assert c, path
        assert _ints(c.group(1)) == table, path
        ours = _defines(src)
        assert ours["ALLREDUCE_IDX"] == d["ALLREDUCE_IDX"] and ours["REDUCE_IDX"] == d["REDUCE_IDX"], path
        # the lgn cap of pof2_lgn is COLL_SIZE
        cap = re.search(r"if\s*\(\s*lgn\s*>\s*(\d+)\s*\)\s*lgn\s*=\s*(\d+)\s*;", src)
        assert cap and int(cap.group(1)) == int(cap.group(2)) == d["COLL_SIZE"], path


def test_reduce_scatter_switch_points_match_reference(ref):
    d = _defines(ref)
    for path in COPIES:
        ours = _defines(_strip_comments(open(path).read()))
        assert ours["REDSCAT_COMMUTATIVE_LONG_MSG"] == d["MPIR_REDSCAT_COMMUTATIVE_LONG_MSG"], path
        assert ours["REDSCAT_NONCOMMUTATIVE_SHORT_MSG"] == d["MPIR_REDSCAT_NONCOMMUTATIVE_SHORT_MSG"], path
    # ... and the reference compares them as the copies assume: the
    # commutative long-message switch on nbytes (:6248), the
    # noncommutative short switch on nbytes too (:6451-6453, 6506)
    assert re.search(r"\(\s*op_ptr->commute\s*\)\s*&&\s*\(\s*nbytes\s*<\s*MPIR_REDSCAT_COMMUTATIVE_LONG_MSG\s*\)", ref)
    assert re.search(r"nbytes\s*<=?\s*MPIR_REDSCAT_NONCOMMUTATIVE_SHORT_MSG", ref.replace("\n", " "))


def test_lgn_loop_is_the_one_restated(ref):
    """intra_Reduce and intra_Allreduce start lgn at -1 and walk pof2 the
    way pof2_lgn does; the loop text is found at both sites"""
    flat = re.sub(r"\s+", " ", ref)
    loop = (r"pof2 = 1; while \(pof2 <= (size|comm_size)\) \{ pof2 <<= 1; lgn\+\+; \} pof2 >>= ?1; lgn--; "
            r"if \(lgn > COLL_SIZE\) lgn = COLL_SIZE;")
    assert len(re.findall(loop, flat)) >= 2, "the pof2 / lgn loop changed shape"
    assert flat.count("int lgn = -1;") >= 2
    for path in COPIES:
        src = re.sub(r"\s+", " ", _strip_comments(open(path).read()))
        assert re.search(r"int pof2 = 1, lgn = -1; while \(pof2 <= size\) \{ pof2 <<= 1; lgn\+\+; \} "
                         r"pof2 >>= 1; lgn--;", src), path
