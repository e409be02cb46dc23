"""GPU: derived datatypes with holes on the device path.

* pack / unpack (mvx_type_pack / mvx_type_unpack): unpack(pack(x)) into a
  patterned buffer equals the oracle's type-map copy (oracle/cpu_types.c)
  -- type-map bytes moved, every other byte untouched -- for vector,
  hvector, indexed, hindexed, struct and nested types.
* collectives: MAXLOC / MINLOC on struct types (by the first member,
  global_ops.c:1280-1384; {double, int} moves packed, {float, int} whole), a
  user op on a struct with a hole, and the reference's 329 for other ops, on
  virtual communicators p = 1..8, device and host buffers, against the
  oracle's replay -- whole recv buffers compared, so bytes outside the type
  map must keep the caller's pattern as in the reference.
"""
import os

import numpy as np
import pytest

import mvxtest as T
import uops

pytestmark = pytest.mark.gpu

I, D, F, C, B = 6, 11, 10, 1, 3


def _both(mvx, oracle, ctor, *args):
    rm, hm = getattr(mvx, "MPI_Type_" + ctor)(*args)
    ro, ho = getattr(oracle, "type_" + ctor)(*args)
    assert rm == ro == 0 and hm == ho, (ctor, args, rm, ro)
    assert mvx.MPI_Type_commit(hm) == 0 and oracle.type_commit(ho) == 0
    return hm


def _types(mvx, oracle):
    """name -> handle, built identically on both sides (handles agree)."""
    t = {}
    t["vec_int"] = _both(mvx, oracle, "vector", 3, 2, 5, I)             # 3 x 2 ints, stride 5
    t["hvec_dbl"] = _both(mvx, oracle, "hvector", 4, 1, 24, D)          # doubles 24 bytes apart
    t["idx_int"] = _both(mvx, oracle, "indexed", 3, [2, 1, 3], [0, 4, 7], I)
    t["hidx_chr"] = _both(mvx, oracle, "hindexed", 3, [3, 1, 2], [1, 9, 13], C)
    t["st_di"] = _both(mvx, oracle, "struct", 2, [1, 1], [0, 8], [D, I])   # {double; int}: 16 / 12
    t["st_id"] = _both(mvx, oracle, "struct", 2, [1, 1], [0, 8], [I, D])   # {int; hole; double}
    t["st_fi"] = _both(mvx, oracle, "struct", 2, [1, 1], [0, 4], [F, I])   # {float; int}: dense
    t["st_ci"] = _both(mvx, oracle, "struct", 3, [1, 2, 1], [0, 4, 14], [C, I, B])
    t["nest"] = _both(mvx, oracle, "contiguous", 3, t["vec_int"])
    t["vec_st"] = _both(mvx, oracle, "vector", 2, 1, 3, t["st_di"])
    return t


@pytest.fixture(scope="module")
def types(mvx, oracle):
    t = _types(mvx, oracle)
    yield t
    for h in t.values():
        mvx.MPI_Type_free(h)
        oracle.type_free(h)


def test_pack_unpack_match_the_type_map(mvx, oracle, types):
    import torch
    for name, h in types.items():
        ext = mvx.MPI_Type_extent(h)[1]
        size = mvx.MPI_Type_size(h)[1]
        L = mvx.type_layout(h)
        assert L["span_lo"] >= 0
        for n in (1, 7, 1000, 65537):
            nb = (n - 1) * ext + L["span_hi"]
            rng = np.random.default_rng(n + h)
            x = rng.integers(0, 256, nb, dtype=np.uint8)
            y0 = np.full(nb, 0xAB, np.uint8)
            dx = torch.from_numpy(x).cuda()
            dp = torch.zeros(max(n * size, 1), dtype=torch.uint8, device="cuda")
            dy = torch.from_numpy(y0).cuda()
            assert mvx.type_pack(h, dx, dp, n) == 0
            assert mvx.type_unpack(h, dp, dy, n) == 0
            ref = y0.copy()
            assert oracle.type_copy(ref, x, n, h) == 0
            assert np.array_equal(T.from_dev(dy), ref), (name, n)
            if L["dense"]:
                assert size == ext


def _coll(comm, coll, sends, recvs, n, dt, op, root=0, cnts=None):
    if coll == "ar":
        return comm.allreduce_multi(sends, recvs, n, dt, op)
    if coll == "red":
        return comm.reduce_multi(sends, recvs, n, dt, op, root)
    if coll == "scan":
        return comm.scan_multi(sends, recvs, n, dt, op)
    return comm.reduce_scatter_multi(sends, recvs, cnts, dt, op)


def _oracle(oracle, coll, S, R, n, dt, op, root=0, cnts=None):
    if coll == "ar":
        return oracle.allreduce(S, R, n, dt, op)
    if coll == "red":
        return oracle.reduce(S, R, n, dt, op, root)
    if coll == "scan":
        return oracle.scan(S, R, n, dt, op)
    return oracle.reduce_scatter(S, R, cnts, dt, op)


def _pairs_bytes(h, n, ext, seed, kind):
    """n elements of a struct {value, int loc} laid out by extent, ties
    included; the bytes outside the type map random too."""
    rng = np.random.default_rng(seed)
    b = rng.integers(0, 256, n * ext, dtype=np.uint8)
    v = b.reshape(n, ext)
    if kind == "di":
        vals = rng.integers(-3, 4, n).astype(np.float64)
        vals[rng.random(n) < 0.05] = np.nan
        v[:, 0:8] = vals.view(np.uint8).reshape(n, 8)
        v[:, 8:12] = rng.integers(-9, 9, n).astype(np.int32).view(np.uint8).reshape(n, 4)
    elif kind == "fi":
        v[:, 0:4] = rng.integers(-3, 4, n).astype(np.float32).view(np.uint8).reshape(n, 4)
        v[:, 4:8] = rng.integers(-9, 9, n).astype(np.int32).view(np.uint8).reshape(n, 4)
    else:   # id: {int a; hole; double b}
        v[:, 0:4] = rng.integers(-1000, 1000, n).astype(np.int32).view(np.uint8).reshape(n, 4)
        v[:, 8:16] = (rng.standard_normal(n) * 100).astype(np.float64).view(np.uint8).reshape(n, 8)
    return b


CASES = [("st_di", 111, "di"), ("st_di", 110, "di"), ("st_fi", 111, "fi"), ("st_id", "idsum", "id")]


@pytest.mark.parametrize("where", ["device", "host"])
@pytest.mark.parametrize("p", [1, 2, 3, 4, 8])
@pytest.mark.parametrize("tname,op,kind", CASES)
def test_struct_collectives_match_reference(mvx, oracle, types, where, p, tname, op, kind):
    import torch
    h = types[tname]
    ext = mvx.MPI_Type_extent(h)[1]
    comm = mvx.Comm.local_ranks(p, 0)
    uop = None
    if op == "idsum":
        rc, uop = (mvx.op_create_device(uops.dev_fn("idsum"), 1) if where == "device"
                   else mvx.MPI_Op_create(uops.host_fn("idsum"), 1))
        assert rc == 0
        assert oracle.user_op_set(250, uops.host_fn("idsum"), 1) == 0
    try:
        for coll, n in (("ar", 3), ("ar", 70001), ("red", 5000), ("rs", 1500), ("scan", 800)):
            cnts = [n // p + (r % 2) for r in range(p)] if coll == "rs" else None
            tot = sum(cnts) if cnts else n
            S = [_pairs_bytes(h, tot, ext, 17 * p + r + tot, kind) for r in range(p)]
            nrecv = [(cnts[r] if cnts else tot) for r in range(p)]
            R0 = [np.full(max(k, 1) * ext, 0x5C, np.uint8) for k in nrecv]      # caller's pattern
            if where == "device":
                sends = [torch.from_numpy(s).cuda() for s in S]
                recvs = [torch.from_numpy(r.copy()).cuda() for r in R0]
            else:
                sends = [s.copy() for s in S]
                recvs = [r.copy() for r in R0]
            root = p - 1
            r, rcs = _coll(comm, coll, sends, recvs, tot, h, uop if uop else op, root, cnts)
            assert r == 0, (coll, n, r)
            ref = [x.copy() for x in R0]
            rref = _oracle(oracle, coll, S, ref, tot, h, 250 if uop else op, root, cnts)
            assert rcs == rref, (coll, n)
            for q in range(p):
                got = recvs[q] if isinstance(recvs[q], np.ndarray) else T.from_dev(recvs[q])
                assert np.array_equal(got, ref[q]), (tname, op, coll, n, q)
    finally:
        comm.free()
        if uop:
            mvx.MPI_Op_free(uop)


def test_undefined_ops_and_refused_layouts(mvx, oracle, types):
    """329 for SUM on a struct and MAXLOC on a vector (every rank that calls
    the op); MAXLOC on a struct whose extent is not its first member's pair
    struct is refused (MPI_ERR_TYPE, a documented deviation: the reference's
    element-overlapping reads have no reorderable equivalent)."""
    import torch
    comm = mvx.Comm.local_ranks(4, 0)
    x = [torch.zeros(64 * 64, dtype=torch.uint8, device="cuda") for _ in range(4)]
    y = [torch.zeros(64 * 64, dtype=torch.uint8, device="cuda") for _ in range(4)]
    for h, op in ((types["st_di"], 102), (types["vec_int"], 111), (types["nest"], 110)):
        r, rcs = comm.allreduce_multi(x, y, 16, h, op)
        assert r == 0 and rcs == [329] * 4
    r, rcs = comm.allreduce_multi(x, y, 16, types["st_ci"], 111)      # CHAR first: 329
    assert rcs == [329] * 4
    # {float; int; hole} (extent 12) -> the FLOAT_INT kernel reads 8-byte pairs
    rm, odd = mvx.MPI_Type_struct(3, [1, 1, 1], [0, 4, 12], [F, I, mvx.MPI_UB])
    assert rm == 0 and mvx.MPI_Type_extent(odd)[1] == 12
    r, rcs = comm.allreduce_multi(x, y, 16, odd, 111)
    assert r == mvx.MPI_ERR_TYPE
    mvx.MPI_Type_free(odd)
    comm.free()


@pytest.mark.parametrize("where", ["device", "host"])
@pytest.mark.parametrize("p", [2, 3, 5, 8])
@pytest.mark.parametrize("tname,op,kind", CASES)
def test_struct_collectives_smp_flavour(mvx, oracle, types, where, p, tname, op, kind):
    """The _SMP_ collops on derived types: below the shmem thresholds (int
    count * extent < 32 KiB Allreduce, 1 KiB Reduce) the node leader's
    rank-order fold, above them the intra_* algorithms -- against the
    oracle's replay of intra_shmem_* (smp = 1)."""
    import torch
    h = types[tname]
    ext = mvx.MPI_Type_extent(h)[1]
    comm = mvx.Comm.local_ranks(p, 0)
    assert comm.set_tuning(mvx.smp_tuning()) == 0
    oracle.smp_set(1)
    uop = None
    if op == "idsum":
        rc, uop = (mvx.op_create_device(uops.dev_fn("idsum"), 1) if where == "device"
                   else mvx.MPI_Op_create(uops.host_fn("idsum"), 1))
        assert rc == 0
        assert oracle.user_op_set(250, uops.host_fn("idsum"), 1) == 0
    try:
        for coll in ("ar", "red"):
            for n in (3, (1 << 10) // ext - 1, (1 << 10) // ext + 1, (1 << 15) // ext - 1, (1 << 15) // ext + 1):
                S = [_pairs_bytes(h, n, ext, 29 * p + r + n, kind) for r in range(p)]
                R0 = [np.full(n * ext, 0x5C, np.uint8) for _ in range(p)]
                if where == "device":
                    sends = [torch.from_numpy(s).cuda() for s in S]
                    recvs = [torch.from_numpy(r.copy()).cuda() for r in R0]
                else:
                    sends = [s.copy() for s in S]
                    recvs = [r.copy() for r in R0]
                root = p - 1
                r, rcs = _coll(comm, coll, sends, recvs, n, h, uop if uop else op, root)
                assert r == 0, (coll, n, r)
                ref = [x.copy() for x in R0]
                rref = _oracle(oracle, coll, S, ref, n, h, 250 if uop else op, root)
                assert rcs == rref, (coll, n, rcs, rref)
                for q in range(p):
                    if coll == "red" and q != root:
                        continue
                    got = recvs[q] if isinstance(recvs[q], np.ndarray) else T.from_dev(recvs[q])
                    assert np.array_equal(got, ref[q]), (tname, op, coll, n, q)
    finally:
        oracle.smp_set(0)
        comm.free()
        if uop:
            mvx.MPI_Op_free(uop)


@pytest.mark.parametrize("batch", range(int(__import__("os").environ.get("MVX_FUZZ_DT_BATCHES", "3"))))
def test_random_derived_sweep(mvx, oracle, types, batch):
    """Seeded random cases over the derived types above: collective, p,
    count, root, ragged recvcnts, exchange variant, device or host buffers,
    and an op that is defined on the type (MAXLOC / MINLOC on the pair
    structs) or not (329 -- the data still moves as the reference moves it,
    packed where the type has holes).  Whole recv buffers compared: bytes
    outside the type map keep the caller's pattern."""
    import torch
    rng = np.random.default_rng(9000 + batch)
    # plus a type whose map starts before its origin (lb -8): buffers get a
    # head margin too, and the calls take origins inside them
    types = dict(types)
    types["hidx_neg"] = _both(mvx, oracle, "hindexed", 2, [1, 1], [-8, 4], I)
    names = sorted(types)
    comms = {}
    checked = undefined = 0
    head = 64
    try:
        for _ in range(30):
            tname = str(rng.choice(names))
            h = types[tname]
            ext = mvx.MPI_Type_extent(h)[1]
            op = int(rng.choice([110, 111, 102, 105, 100]))
            p = int(rng.choice([1, 2, 3, 4, 5, 8]))
            if p not in comms:
                comms[p] = mvx.Comm.local_ranks(p, 0)
            comm = comms[p]
            mode = int(rng.choice([mvx.EXCH_P2P, mvx.EXCH_PIPE, mvx.EXCH_COLL]))
            assert comm.set_exchange(mode, int(rng.integers(2, 5))) == 0
            coll = str(rng.choice(["ar", "ar", "red", "rs", "scan"]))
            n = int(rng.choice([1, 3, 100, 2049, 30001]))
            cnts = [max(0, n // p + int(rng.integers(-1, 2))) for _ in range(p)] if coll == "rs" else None
            tot = sum(cnts) if cnts else n
            kind = {"st_di": "di", "st_fi": "fi", "vec_st": None}.get(tname)
            # buffers cover the type map's span: a type whose map reaches past
            # its extent (hidx_chr: lb 1, extent 14, map up to byte 15) touches
            # bytes past count * extent -- the caller's to provide, as in MPI
            tail = 64
            S = [np.concatenate([rng.integers(0, 256, head, dtype=np.uint8),
                                 (_pairs_bytes(h, tot, ext, int(rng.integers(1 << 30)), kind) if kind
                                  else rng.integers(0, 256, tot * ext, dtype=np.uint8)),
                                 rng.integers(0, 256, tail, dtype=np.uint8)]) for _ in range(p)]
            nrecv = [(cnts[r] if cnts else tot) for r in range(p)]
            R0 = [np.full(head + k * ext + tail, 0x5C, np.uint8) for k in nrecv]
            where = str(rng.choice(["device", "host"]))
            if where == "device":
                sends = [torch.from_numpy(s).cuda() for s in S]
                recvs = [torch.from_numpy(r.copy()).cuda() for r in R0]
            else:
                sends = [s.copy() for s in S]
                recvs = [r.copy() for r in R0]
            root = int(rng.integers(0, p))
            r, rcs = _coll(comm, coll, [x[head:] for x in sends], [x[head:] for x in recvs], tot, h, op, root,
                           cnts)
            ref = [x.copy() for x in R0]
            rref = _oracle(oracle, coll, [x[head:] for x in S], [x[head:] for x in ref], tot, h, op, root, cnts)
            case = (tname, op, p, coll, n, cnts, mode, where, root)
            if r == mvx.MPI_ERR_TYPE:        # the documented refusal (MAXLOC, extent != pair struct)
                continue
            assert r == 0, (r, case)
            assert rcs == rref, (rcs, rref, case)
            for q in range(p):
                got = recvs[q] if isinstance(recvs[q], np.ndarray) else T.from_dev(recvs[q])
                assert np.array_equal(got, ref[q]), (q, case)
            checked += 1
            undefined += 329 in rcs
        assert checked >= 20 and undefined >= 1, (checked, undefined)
    finally:
        for c in comms.values():
            c.free()
        assert mvx.MPI_Type_free(types["hidx_neg"])[0] == 0 and oracle.type_free(types["hidx_neg"]) == 0


def test_whole_word_unpack_keeps_every_other_byte(mvx, oracle):
    """Pack through LDS tiles (k_pack_tiles, into a 16-byte-aligned packed
    buffer) gives the unit kernel's stream (into a buffer 4 bytes off).
    Unpack of types whose maps leave holes inside 64-byte sectors runs by
    whole 16-byte words (mvx_dtype.hip k_unpack_merge: each tile read into
    LDS, the units merged in, written back whole).  Against the oracle's
    type-map copy over a patterned buffer with guard bands: type-map bytes
    land, holes and guards keep their pattern -- at counts 1, 2, 3, 1000
    and 100003, with the origin at every 4-byte phase of a 16-byte word (the
    first and last words of the hull are partial there and take unit stores
    instead), for a type reaching below its origin (negative stride), and
    for maps of 1- and 2-byte pieces (the tile kernels over 1- and 2-byte
    units)."""
    import torch
    made = [
        _both(mvx, oracle, "vector", 8, 1, 4, D),              # 8 B of every 32
        _both(mvx, oracle, "vector", 2, 1, 2, F),              # every other float
        _both(mvx, oracle, "struct", 2, [1, 1], [0, 8], [I, D]),  # {int; hole; double}
        _both(mvx, oracle, "hvector", 3, 1, -20, I),           # reaches below the origin
        _both(mvx, oracle, "hindexed", 3, [1, 2, 1], [0, 12, 40], F),
        _both(mvx, oracle, "vector", 2, 1, 2, C),              # every other byte (1-byte units)
        _both(mvx, oracle, "struct", 2, [1, 1], [0, 4], [C, I]),  # {char; hole; int}
        _both(mvx, oracle, "hvector", 3, 1, 6, 4),             # shorts 6 bytes apart (2-byte units)
        _both(mvx, oracle, "hindexed", 3, [3, 1, 2], [1, 9, 13], C),   # bytes from 1, odd spans
    ]
    try:
        for h in made:
            ext = mvx.MPI_Type_extent(h)[1]
            size = mvx.MPI_Type_size(h)[1]
            L = mvx.type_layout(h)
            for n in (1, 2, 3, 1000, 100003):
                for phase in (0, 4, 8, 12):
                    guard = 256
                    off = guard + phase - min(0, L["span_lo"])
                    nb = off + (n - 1) * ext + L["span_hi"] + guard
                    rng = np.random.default_rng(n * 7 + phase + h)
                    x = np.zeros(nb, np.uint8)
                    x[off + min(0, L["span_lo"]):nb - guard] = rng.integers(
                        0, 256, nb - guard - off - min(0, L["span_lo"]), dtype=np.uint8)
                    y0 = rng.integers(0, 256, nb, dtype=np.uint8)
                    dx = torch.from_numpy(x).cuda()
                    dy = torch.from_numpy(y0).cuda()
                    dp = torch.zeros(max(n * size, 16), dtype=torch.uint8, device="cuda")
                    assert mvx.type_pack(h, dx.data_ptr() + off, dp, n) == 0
                    # the same pack into a packed buffer 4 bytes off a 16-byte
                    # boundary (no tiled pack there: the unit kernel) -- the
                    # same stream
                    dq = torch.zeros(max(n * size, 16) + 16, dtype=torch.uint8, device="cuda")
                    assert mvx.type_pack(h, dx.data_ptr() + off, dq.data_ptr() + 4, n) == 0
                    assert torch.equal(dq[4:4 + n * size], dp[:n * size]), (h, n, phase)
                    assert mvx.type_unpack(h, dp, dy.data_ptr() + off, n) == 0
                    ref = y0.copy()
                    assert oracle.type_copy(ref[off:], x[off:], n, h) == 0
                    got = T.from_dev(dy)
                    assert np.array_equal(got, ref), (h, n, phase, np.flatnonzero(got != ref)[:8])
    finally:
        for h in made:
            mvx.MPI_Type_free(h)
            oracle.type_free(h)


def _random_type(mvx, oracle, rng):
    """A random hindexed / struct type of 1-, 2-, 4- and 8-byte pieces:
    blocks in random order (the type map's order is the packed order),
    gaps, sometimes reaching below the origin, sometimes nested in an
    hvector whose stride leaves a gap.  Returns the handles to free."""
    base = [(C, 1), (B, 1), (4, 2), (I, 4), (F, 4), (D, 8)]
    nb = int(rng.integers(1, 6))
    kind = "struct" if rng.random() < 0.4 else "hindexed"
    if kind == "hindexed":
        bt, bs = base[int(rng.integers(len(base)))]
        types = [bt] * nb
        sizes = [bs] * nb
    else:
        pick = [base[int(i)] for i in rng.integers(len(base), size=nb)]
        types = [p[0] for p in pick]
        sizes = [p[1] for p in pick]
    lens = [int(x) for x in rng.integers(1, 5, size=nb)]
    displs, cur = [], 0
    for s, ln in zip(sizes, lens):
        cur += int(rng.integers(0, 4)) * s          # a gap of whole pieces
        cur = (cur + s - 1) // s * s
        displs.append(cur)
        cur += s * ln
    if rng.random() < 0.25:                         # reach below the origin
        shift = 8 * int(rng.integers(1, 4))
        displs = [d - shift for d in displs]
    order = rng.permutation(nb)
    displs = [displs[i] for i in order]
    lens = [lens[i] for i in order]
    types = [types[i] for i in order]
    if kind == "hindexed":
        h = _both(mvx, oracle, "hindexed", nb, lens, displs, types[0])
    else:
        h = _both(mvx, oracle, "struct", nb, lens, displs, types)
    made = [h]
    if rng.random() < 0.3:
        ext = mvx.MPI_Type_extent(h)[1]
        stride = ext + 8 * int(rng.integers(0, 3))
        h = _both(mvx, oracle, "hvector", int(rng.integers(2, 4)), 1, stride, h)
        made.append(h)
    return h, made


@pytest.mark.parametrize("batch", range(int(os.environ.get("MVX_FUZZ_TYPEMAP_BATCHES", "8"))))
def test_random_type_maps_pack_unpack(mvx, oracle, batch):
    """Seeded random type maps (_random_type) through every pack / unpack
    kernel the dispatch picks -- the tiled pack and whole-word unpack
    (16-byte-aligned packed buffer), the unit kernel and the piece kernel
    (packed buffer 4 bytes off) -- at counts 1 to 65537 and a random origin
    phase: the packed streams agree, and unpack(pack(x)) into a patterned
    buffer with guard bands equals the oracle's type-map copy (type-map bytes
    land, holes and guards keep their pattern)."""
    import torch
    rng = np.random.default_rng(4242 + batch)
    for _ in range(15):
        h, made = _random_type(mvx, oracle, rng)
        try:
            ext = mvx.MPI_Type_extent(h)[1]
            size = mvx.MPI_Type_size(h)[1]
            L = mvx.type_layout(h)
            for n in (1, 2, 17, 1000, 65537):
                phase = int(rng.integers(0, 16))
                guard = 256
                off = guard + phase - min(0, L["span_lo"])
                nb = off + (n - 1) * ext + L["span_hi"] + guard
                x = rng.integers(0, 256, nb, dtype=np.uint8)
                y0 = rng.integers(0, 256, nb, dtype=np.uint8)
                dx = torch.from_numpy(x).cuda()
                dy = torch.from_numpy(y0).cuda()
                dp = torch.zeros(max(n * size, 16), dtype=torch.uint8, device="cuda")
                dq = torch.zeros(max(n * size, 16) + 16, dtype=torch.uint8, device="cuda")
                assert mvx.type_pack(h, dx.data_ptr() + off, dp, n) == 0
                assert mvx.type_pack(h, dx.data_ptr() + off, dq.data_ptr() + 4, n) == 0
                assert torch.equal(dq[4:4 + n * size], dp[:n * size]), (h, n, phase)
                assert mvx.type_unpack(h, dp, dy.data_ptr() + off, n) == 0
                ref = y0.copy()
                assert oracle.type_copy(ref[off:], x[off:], n, h) == 0
                got = T.from_dev(dy)
                assert np.array_equal(got, ref), (L, n, phase, np.flatnonzero(got != ref)[:8])
                # and from the misaligned packed copy (unit / piece kernels)
                dz = torch.from_numpy(y0).cuda()
                assert mvx.type_unpack(h, dq.data_ptr() + 4, dz.data_ptr() + off, n) == 0
                assert np.array_equal(T.from_dev(dz), ref), (L, n, phase, "misaligned packed")
        finally:
            for m in reversed(made):
                mvx.MPI_Type_free(m)
                oracle.type_free(m)


def test_whole_word_unpack_of_large_elements(mvx, oracle):
    """Whole-word unpack of types with more than 2048 units per element (the
    unit offsets then come from global memory, k_unpack_merge<..., LDSU =
    false, ...>): 2 chars of every 3, 1100 and 1400 blocks (extents 3299 and
    4199 bytes; the first within the LDS-swizzle model's reach), against the
    oracle's type-map copy with guard bands, at several counts and origin
    phases."""
    import torch
    made = [
        _both(mvx, oracle, "hindexed", 1100, [2] * 1100, [3 * i for i in range(1100)], C),
        _both(mvx, oracle, "hindexed", 1400, [2] * 1400, [3 * i for i in range(1400)], C),
    ]
    try:
        for h in made:
            ext = mvx.MPI_Type_extent(h)[1]
            size = mvx.MPI_Type_size(h)[1]
            L = mvx.type_layout(h)
            for n in (1, 2, 3, 100, 3001):
                for phase in (0, 7):
                    guard = 256
                    off = guard + phase
                    nb = off + (n - 1) * ext + L["span_hi"] + guard
                    rng = np.random.default_rng(n * 11 + phase + h)
                    x = rng.integers(0, 256, nb, dtype=np.uint8)
                    y0 = rng.integers(0, 256, nb, dtype=np.uint8)
                    dx = torch.from_numpy(x).cuda()
                    dy = torch.from_numpy(y0).cuda()
                    dp = torch.zeros(max(n * size, 16), dtype=torch.uint8, device="cuda")
                    assert mvx.type_pack(h, dx.data_ptr() + off, dp, n) == 0
                    assert mvx.type_unpack(h, dp, dy.data_ptr() + off, n) == 0
                    ref = y0.copy()
                    assert oracle.type_copy(ref[off:], x[off:], n, h) == 0
                    got = T.from_dev(dy)
                    assert np.array_equal(got, ref), (ext, n, phase, np.flatnonzero(got != ref)[:8])
    finally:
        for h in made:
            mvx.MPI_Type_free(h)
            oracle.type_free(h)
