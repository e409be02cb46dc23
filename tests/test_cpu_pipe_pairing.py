"""CPU: the PIPE exchange's messages pair up across ranks (csrc/mvx_exec.c
run_device_pipe), checked on the ranks' real plans (mvx_plan_build).

Every rank computes its slice length from its own plan; RCCL and the host
transports pair a rank's sends to a peer with that peer's receives in issue
order, so a schedule is only correct if, for every ordered pair of ranks,
the sender's message sizes equal the receiver's, in order.  The model below
restates the schedule: phase A slice by slice (slice t of every range is
[t*cs, (t+1)*cs) from its start, mvxi_plan_slice), phase C unsliced on every
rank.  The round-4 bug it guards against: phase C sliced on the ranks whose
result is a temporary (a non-root Reduce) and whole on the root.
"""
import importlib

import numpy as np
import pytest

mvx = importlib.import_module("mvapich-cce_amd")


def _span(P, p):
    s = P.c_cnt if P.has_combine else 0
    for q in range(p):
        for r in (P.a_send[q], P.a_recv[q], P.b_send[q], P.b_recv[q]):
            s = max(s, r.cnt)
    return s


def _slice_len(cnt, t, cs):
    return max(0, min(cs, cnt - t * cs))


def _schedule(P, p, ns):
    """(sends[peer], recvs[peer]): element counts in issue order"""
    span = _span(P, p)
    cs = -(-span // ns)
    cs = (cs + 255) & ~255
    nsl = -(-span // cs) if cs else 0
    sends = {q: [] for q in range(p)}
    recvs = {q: [] for q in range(p)}
    if nsl <= 1:                      # run_device_plain: A whole, then C whole
        slices = [(0, 1 << 62)]
    else:
        slices = [(t, cs) for t in range(nsl)]
    for t, c in slices:
        for q in range(p):
            n = _slice_len(P.a_send[q].cnt, t, c)
            if n:
                sends[q].append(("A", n))
            n = _slice_len(P.a_recv[q].cnt, t, c)
            if n:
                recvs[q].append(("A", n))
    for q in range(p):
        if P.b_send[q].cnt:
            sends[q].append(("C", P.b_send[q].cnt))
        if P.b_recv[q].cnt:
            recvs[q].append(("C", P.b_recv[q].cnt))
    return cs, sends, recvs


def _cases(n_cases, seed):
    """collective, p, count, recvcnts, op, type, root, slices, and the op
    kind (predefined, or a user op: commutative / not, which the reference
    sends through other algorithms) and the device flavour (ch_shmem or an
    _SMP_ build's knobs, mvx_tuning_from_env)"""
    rng = np.random.default_rng(seed)
    kinds = [mvx.COLL_ALLREDUCE, mvx.COLL_REDUCE, mvx.COLL_REDUCE_SCATTER, mvx.COLL_SCAN]
    smp = mvx.tuning_from_env(True)
    for _ in range(n_cases):
        p = int(rng.integers(2, 17))
        kind = kinds[int(rng.integers(0, len(kinds)))]
        op = int(rng.integers(100, 112))
        dtype = 10
        root = int(rng.integers(0, p))
        ns = int(rng.integers(2, 9))
        opkind = [None, mvx.OPKIND_USER_COMMUTE, mvx.OPKIND_USER_NONCOMMUTE][int(rng.integers(0, 3))]
        tuning = smp if rng.integers(0, 4) == 0 else None
        if kind == mvx.COLL_REDUCE_SCATTER:
            cnts = [int(rng.integers(0, 60000)) for _ in range(p)]
            yield kind, p, sum(cnts), cnts, op, dtype, root, ns, opkind, tuning
        else:
            yield kind, p, int(rng.integers(1, 500000)), None, op, dtype, root, ns, opkind, tuning


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_pipe_messages_pair_up(seed):
    checked = 0
    for kind, p, n, cnts, op, dtype, root, ns, opkind, tuning in _cases(150, seed):
        try:
            plans = [mvx.plan(kind, p, r, n, dtype, op, root=root, recvcnts=cnts, opkind=opkind, tuning=tuning)
                     for r in range(p)]
        except ValueError:
            continue
        sched = [_schedule(P, p, ns) for P in plans]
        # one slice length on every rank: the plans' spans agree
        assert len({s[0] for s in sched}) == 1, (kind, p, n, cnts, root, [s[0] for s in sched])
        for a in range(p):
            for b in range(p):
                assert sched[a][1][b] == sched[b][2][a], (kind, p, n, cnts, root, ns, a, b)
        checked += 1
    assert checked > 100


def test_reduce_root_and_non_roots_pair_in_phase_c():
    """the case the sliced phase C broke: Reduce, p = 4, root 3, whose
    non-root ranks hold their result in a temporary"""
    p, n, root = 4, 70001, 3
    plans = [mvx.plan(mvx.COLL_REDUCE, p, r, n, 10, 102, root=root) for r in range(p)]
    assert [P.c_dst_tmp for P in plans] == [1, 1, 1, 0]
    sched = [_schedule(P, p, 3) for P in plans]
    for a in range(p):
        for b in range(p):
            assert sched[a][1][b] == sched[b][2][a]
