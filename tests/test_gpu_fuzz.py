"""Seeded random sweep over the whole device path against the oracle's
replay of the reference schedules (oracle/coll_sim.c): communicator size,
collective, (op, datatype) -- undefined pairs included, whose 329 must come
from exactly the ranks the reference's (*uop) calls would --, count (0,
ragged, across the algorithm thresholds and the staging-slice sizes), root,
ragged recvcnts, exchange variant (p2p / pipe with 2-6 slices / coll),
device flavour (ch_shmem / _SMP_), buffer kind per rank (HBM, pageable,
page-locked, mixed, and offset by one element from the allocation), and
user-defined ops (host MPI_User_functions and device functions, commutative
or not, tests/user_ops.c / user_ops_dev.hip).

Each case is one call on a virtual communicator; every rank's result and
return code must equal the reference's.  MVX_FUZZ_CASES / MVX_FUZZ_SEED
widen or move the sweep."""
import os

import numpy as np
import pytest

import mvxtest as T
import uops

pytestmark = pytest.mark.gpu

N_CASES = int(os.environ.get("MVX_FUZZ_CASES", "600"))
SEED = int(os.environ.get("MVX_FUZZ_SEED", "20261017"))
BATCH = 40
TYPES = [t for t in T.ALL_TYPES]
MAX_BYTES = int(os.environ.get("MVX_FUZZ_MAX_MIB", "24")) << 20     # per rank vector
BIG = os.environ.get("MVX_FUZZ_BIG") == "1"     # sizes 1 Mi - 64 Mi elements (one-off sweeps)
DEVICE_UOPS = ["addem", "affine", "fsum", "mix"]   # the ops tests/user_ops_dev.hip also defines


def _case(rng, mvx):
    p = int(rng.choice([1, 2, 2, 3, 4, 4, 5, 6, 7, 8, 8, 9, 12, 16, 33]))
    coll = str(rng.choice(["ar", "ar", "red", "rs", "scan"]))
    dtype = int(rng.choice(TYPES))
    op = int(rng.integers(100, 112))
    E = mvx.dtype_info(dtype)[0]
    r = rng.random()
    if BIG:
        n = int(np.exp2(rng.uniform(20, 26)))
    elif r < 0.08:
        n = 0
    elif r < 0.45:
        n = int(rng.integers(1, 300))
    elif r < 0.85:
        n = int(np.exp2(rng.uniform(8, 17)))
    else:
        n = int(np.exp2(rng.uniform(17, 21)))
    n = min(n, MAX_BYTES // E // (p if coll == "rs" else 1))
    cnts = None
    if coll == "rs":
        base = max(n // max(p, 1), 0)
        cnts = [int(max(0, base + rng.integers(-3, 4))) if rng.random() < 0.8 else 0 for _ in range(p)]
    exch = str(rng.choice(["p2p", "pipe", "coll"]))
    slices = int(rng.integers(2, 7))
    smp = bool(rng.random() < 0.25)
    kinds = [str(rng.choice(["dev", "dev", "host", "pin"])) for _ in range(2 * p)]
    shift = [int(rng.random() < 0.2) for _ in range(2 * p)]
    root = int(rng.integers(0, p))
    uop = None
    if rng.random() < 0.2:
        device = bool(rng.random() < 0.5)
        names = DEVICE_UOPS if device else sorted(uops.UOPS)
        uop = (str(rng.choice(names)), int(rng.integers(0, 2)), device)
        n = min(n, 1 << 18)
        if cnts:
            cnts = [min(x, (1 << 18) // p) for x in cnts]
    return dict(p=p, coll=coll, dtype=dtype, op=op, n=n, cnts=cnts, exch=exch, slices=slices, smp=smp,
                kinds=kinds, shift=shift, root=root, seed=int(rng.integers(1 << 30)), uop=uop)


def _place(a_u8, kind, shift, E):
    """A buffer of kind `kind` holding bytes a_u8, `shift` elements into its
    allocation; returns (buffer, allocation) -- the allocation keeps it alive."""
    import torch
    off = shift * E
    nb = a_u8.nbytes
    if kind == "host":
        whole = np.zeros(nb + off + 1, np.uint8)
        whole[off:off + nb] = a_u8
        return whole[off:off + max(nb, 1)], whole
    if kind == "pin":
        whole = torch.zeros(nb + off + 1, dtype=torch.uint8, pin_memory=True)
        whole.numpy()[off:off + nb] = a_u8
        return whole[off:off + max(nb, 1)], whole
    whole = torch.zeros(nb + off + 1, dtype=torch.uint8, device="cuda")
    if nb:
        whole[off:off + nb] = torch.from_numpy(np.ascontiguousarray(a_u8)).to("cuda")
    return whole[off:off + max(nb, 1)], whole


def _back(buf):
    import torch
    if isinstance(buf, torch.Tensor):
        if buf.is_cuda:
            torch.cuda.synchronize()
        return buf.cpu().numpy()
    return buf


@pytest.fixture(scope="module")
def comms(mvx):
    cs = {}
    yield cs
    for key, c in cs.items():
        if key == "ops":
            for h in c.values():
                mvx.MPI_Op_free(h)
        else:
            c.free()


def _user_op(mvx, comms, name, commute, device):
    """Product handle of a user op (created once per module); the oracle
    runs the same host function under handle 250."""
    ops = comms.setdefault("ops", {})
    key = (name, commute, device)
    if key not in ops:
        if device:
            rc, h = mvx.op_create_device(uops.dev_fn(name), commute)
        else:
            rc, h = mvx.MPI_Op_create(uops.host_fn(name), commute)
        assert rc == 0
        ops[key] = h
    return ops[key]


def _run_case(mvx, oracle, comms, c):
    p, coll, dtype, op, n = c["p"], c["coll"], c["dtype"], c["op"], c["n"]
    oracle_op = op
    if c["uop"]:
        name, commute, device = c["uop"]
        dtype = uops.UOPS[name][0]
        op = _user_op(mvx, comms, name, commute, device)
        oracle_op = 250
        assert oracle.user_op_set(250, uops.host_fn(name), commute) == 0
    E = mvx.dtype_info(dtype)[0]
    if p not in comms:
        comms[p] = mvx.Comm.local_ranks(p, 0)
    comm = comms[p]
    mode = {"p2p": mvx.EXCH_P2P, "pipe": mvx.EXCH_PIPE, "coll": mvx.EXCH_COLL}[c["exch"]]
    assert comm.set_exchange(mode, c["slices"]) == 0
    assert comm.set_tuning(mvx.smp_tuning() if c["smp"] else mvx.tuning_from_env(smp=False)) == 0
    cnts = c["cnts"]
    tot = sum(cnts) if cnts else n
    if c["uop"]:
        S = [uops.rand_for(c["uop"][0], tot, c["seed"] + q) for q in range(p)]
    else:
        S = [T.rand_vec(dtype, tot, c["seed"] + q) for q in range(p)]
    rcount = [(cnts[q] if cnts else n) for q in range(p)]
    keep, sends, recvs = [], [], []
    for q in range(p):
        b, w = _place(np.ascontiguousarray(S[q]).view(np.uint8), c["kinds"][2 * q], c["shift"][2 * q], E)
        sends.append(b)
        keep.append(w)
        b, w = _place(np.zeros(rcount[q] * E, np.uint8), c["kinds"][2 * q + 1], c["shift"][2 * q + 1], E)
        recvs.append(b)
        keep.append(w)
    if coll == "ar":
        r, rcs = comm.allreduce_multi(sends, recvs, n, dtype, op)
    elif coll == "red":
        r, rcs = comm.reduce_multi(sends, recvs, n, dtype, op, c["root"])
    elif coll == "scan":
        r, rcs = comm.scan_multi(sends, recvs, n, dtype, op)
    else:
        r, rcs = comm.reduce_scatter_multi(sends, recvs, cnts, dtype, op)
    assert r == 0, (r, c)
    R0 = [np.zeros(max(rcount[q], 1), S[0].dtype) for q in range(p)]
    s8 = [s.view(np.uint8) for s in S]
    r8 = [x.view(np.uint8) for x in R0]
    oracle.smp_set(1 if c["smp"] else 0)
    try:
        if coll == "ar":
            rref = oracle.allreduce(s8, r8, n, dtype, oracle_op)
        elif coll == "red":
            rref = oracle.reduce(s8, r8, n, dtype, oracle_op, c["root"])
        elif coll == "scan":
            rref = oracle.scan(s8, r8, n, dtype, oracle_op)
        else:
            rref = oracle.reduce_scatter(s8, r8, cnts, dtype, oracle_op)
    finally:
        oracle.smp_set(0)
    assert list(rcs) == list(rref), (rcs, rref, c)
    for q in range(p):
        got = _back(recvs[q])
        if coll == "red" and q != c["root"]:
            assert not got[: rcount[q] * E].any(), ("non-root recvbuf written", q, c)
            continue
        if rcount[q] == 0:
            continue
        # every rank, 329 or not: an undefined pair moves the data as the
        # reference's algorithm does (ops that keep their inout operand)
        try:
            T.assert_same(0 if c["uop"] else op, dtype, got[: rcount[q] * E], R0[q][: rcount[q]],
                          typemap_only=True)
        except AssertionError as e:
            raise AssertionError("rank %d of %s: %s" % (q, c, e))


@pytest.mark.parametrize("batch", range((N_CASES + BATCH - 1) // BATCH))
def test_random_sweep(mvx, oracle, comms, batch):
    rng = np.random.default_rng(SEED + batch)
    for _ in range(min(BATCH, N_CASES - batch * BATCH)):
        _run_case(mvx, oracle, comms, _case(rng, mvx))


MPIR_NAMES = {100: "MPIR_MAXF", 101: "MPIR_MINF", 102: "MPIR_SUM", 103: "MPIR_PROD", 104: "MPIR_LAND",
              105: "MPIR_BAND", 106: "MPIR_LOR", 107: "MPIR_BOR", 108: "MPIR_LXOR", 109: "MPIR_BXOR",
              110: "MPIR_MINLOC", 111: "MPIR_MAXLOC"}


def _op_case(rng):
    dtype = int(rng.choice(TYPES))
    op = int(rng.integers(100, 112))
    r = rng.random()
    if r < 0.5:
        n = int(rng.integers(0, 5000))
    elif r < 0.9:
        n = int(np.exp2(rng.uniform(12, 22)))
    else:
        n = int(np.exp2(rng.uniform(22, 24.5)))       # past the 64 MiB bounce threshold
    return dict(dtype=dtype, op=op, n=n, kin=str(rng.choice(["dev", "host", "pin"])),
                kio=str(rng.choice(["dev", "host", "pin"])), sin=int(rng.random() < 0.3),
                sio=int(rng.random() < 0.3), seed=int(rng.integers(1 << 30)))


@pytest.mark.parametrize("batch", range(int(os.environ.get("MVX_FUZZ_OP_BATCHES", "4"))))
def test_random_op_functions(mvx, oracle, batch):
    """The predefined ops through their MPI_User_function symbols (MPIR_SUM
    ...) on random sizes (up to ~90 MiB), operand kinds (HBM, pageable,
    page-locked, independently per operand, offset by one element) and
    (op, datatype) pairs -- undefined ones included, which must set the op
    errno to 329 and leave inoutvec untouched -- against the oracle's op."""
    rng = np.random.default_rng(SEED + 1000 + batch)
    for _ in range(25):
        c = _op_case(rng)
        dtype, op, n = c["dtype"], c["op"], c["n"]
        E = mvx.dtype_info(dtype)[0]
        n = min(n, (96 << 20) // E)
        a, b = T.rand_vec(dtype, n, c["seed"]), T.rand_vec(dtype, n, c["seed"] + 1)
        ia, wa = _place(np.ascontiguousarray(a).view(np.uint8), c["kin"], c["sin"], E)
        io, wio = _place(np.ascontiguousarray(b).view(np.uint8), c["kio"], c["sio"], E)
        ref = T.clone(b)
        rc_ref = oracle.op(op, dtype, np.ascontiguousarray(a).view(np.uint8), ref.view(np.uint8), n)
        mvx.op_errno()
        mvx.MPIR_call(MPIR_NAMES[op], ia, io, n, dtype)
        rc = mvx.op_errno()
        assert rc == rc_ref, (rc, rc_ref, c)
        got = _back(io)[: n * E]
        if n:
            try:
                T.assert_same(op, dtype, got, ref)
            except AssertionError as e:
                raise AssertionError("%s: %s" % (c, e))


@pytest.mark.parametrize("batch", range(int(os.environ.get("MVX_FUZZ_REG_BATCHES", "2"))))
def test_random_op_functions_registered(mvx, oracle, batch):
    """The op-function sweep with the registration cache on (mode 2: every
    pageable block is reported with host_invalidate before it is freed), and
    pageable operand pairs that often share pages: carved from one block,
    `inoutvec` starting 0-64 bytes after `invec` ends, or before it -- the
    call-local merge of a call's own operands and the CPU-bounced ranges under
    another registration (mvx_host.c reg_range) against the oracle's op, with
    no registration left held after a call."""
    rng = np.random.default_rng(SEED + 5000 + batch)
    assert mvx.host_register_enable(True) == 0
    try:
        for _ in range(25):
            c = _op_case(rng)
            dtype, op, n = c["dtype"], c["op"], c["n"]
            E = mvx.dtype_info(dtype)[0]
            n = min(n, (64 << 20) // E)
            a, b = T.rand_vec(dtype, n, c["seed"]), T.rand_vec(dtype, n, c["seed"] + 1)
            au8, bu8 = np.ascontiguousarray(a).view(np.uint8), np.ascontiguousarray(b).view(np.uint8)
            blocks = []
            if rng.random() < 0.5 and n:
                # both pageable, from one block: [in][gap][inout] or reversed
                gap = int(rng.choice([0, E, 16, 64]))
                nb = au8.nbytes
                whole = np.zeros(2 * nb + gap + 64, np.uint8)
                first, second = (0, nb + gap) if rng.random() < 0.5 else (nb + gap, 0)
                whole[first:first + nb] = au8
                whole[second:second + nb] = bu8
                ia, io = whole[first:first + nb], whole[second:second + nb]
                blocks.append(whole)
            else:
                ia, wa = _place(au8, c["kin"], c["sin"], E)
                io, wio = _place(bu8, c["kio"], c["sio"], E)
                blocks += [w for w in (wa, wio) if isinstance(w, np.ndarray)]
            ref = T.clone(b)
            rc_ref = oracle.op(op, dtype, au8, ref.view(np.uint8), n)
            mvx.op_errno()
            mvx.MPIR_call(MPIR_NAMES[op], ia, io, n, dtype)
            rc = mvx.op_errno()
            assert rc == rc_ref, (rc, rc_ref, c)
            got = _back(io)[: n * E]
            if n:
                try:
                    T.assert_same(op, dtype, got, ref)
                except AssertionError as e:
                    raise AssertionError("%s: %s" % (c, e))
            assert mvx.host_register_deferred()["held"] == 0, c
            for w in blocks:                          # mode 2: report before the free
                mvx.host_invalidate(w.ctypes.data, w.nbytes)
            del blocks
    finally:
        mvx.host_register_enable(False)
