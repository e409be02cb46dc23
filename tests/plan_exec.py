"""TEST HELPER: run libmvx.so's per-rank plans on the CPU.

Phase A/C data movement is done with numpy copies (or, in the gloo tests,
torch.distributed send/recv); phase B's k-leaf combine is evaluated with the
oracle's op (oracle/cpu_ops.c) in the TREE / CHAIN shape of
include/mvx_hip.h.  Comparing the result with oracle/coll_sim.c (the
reference schedule replayed message by message) checks that the plans encode
the reference's combine order and operand roles exactly.
"""
import numpy as np

from oracle import oracle as O

SHAPE_TREE, SHAPE_CHAIN = 0, 1


def tree_mask(k):
    m, l = 0, 0
    while (1 << l) < k and l < 3:
        for q in range(0, k, 2 << l):
            if q + (1 << l) < k:
                m |= 1 << (l * 8 + q)
        l += 1
    return m


def chain_mask(k):
    return ((1 << k) - 1) & ~1 if k >= 2 else 0


def run_program(op, dtype, leaves, folds, tmask, cmask, n, tswap=0, cswap=0):
    """The combine program of include/mvx_hip.h (<= 8 leaves, masks), step by
    step with the oracle op; a swapped step (user ops) is
    y_left = uop(in = y_left, inout = y_right)."""
    y = []
    for q, a in enumerate(leaves):
        v = a.copy()
        if folds is not None and folds[q] is not None:
            O.op(op, dtype, folds[q], v, n)
        y.append(v)
    k = len(y)
    for l in range(3):
        for q in range(8):
            if tmask >> (l * 8 + q) & 1:
                assert q + (1 << l) < k
                if tswap >> (l * 8 + q) & 1:
                    O.op(op, dtype, y[q], y[q + (1 << l)], n)
                    y[q] = y[q + (1 << l)]
                else:
                    O.op(op, dtype, y[q + (1 << l)], y[q], n)
            else:
                assert not tswap >> (l * 8 + q) & 1
    for q in range(1, k):
        if cmask >> q & 1:
            if cswap >> q & 1:
                O.op(op, dtype, y[0], y[q], n)
                y[0] = y[q]
            else:
                O.op(op, dtype, y[q], y[0], n)
    return y[0]


def run_plan_program(P, leaves, folds, n):
    """A plan's chain-of-trees program (include/mvx_coll.h, any k): every
    segment's tree level by level, then the chain over the segment heads."""
    y = []
    for q, a in enumerate(leaves):
        v = a.copy()
        if folds is not None and folds[q] is not None:
            O.op(P.op, P.dtype, folds[q], v, n)
        y.append(v)
    for s, e in P.segments():
        h = 1
        while h < e - s:
            for q in range(s, e - h, 2 * h):
                if P.tree_swap:
                    O.op(P.op, P.dtype, y[q], y[q + h], n)
                    y[q] = y[q + h]
                else:
                    O.op(P.op, P.dtype, y[q + h], y[q], n)
            h *= 2
    for s, _ in P.segments()[1:]:
        if P.chain_swap >> s & 1:
            O.op(P.op, P.dtype, y[0], y[s], n)
            y[0] = y[s]
        else:
            O.op(P.op, P.dtype, y[s], y[0], n)
    return y[0]


def combine_cpu(op, dtype, esize, leaves, folds, shape, n):
    """leaves/folds: lists of uint8 arrays (n*esize bytes) or None."""
    k = len(leaves)
    return run_program(op, dtype, leaves, folds, tree_mask(k) if shape == SHAPE_TREE else 0,
                       chain_mask(k) if shape == SHAPE_CHAIN else 0, n)


def run_plans(plans, sends, recvs):
    """Execute all ranks' plans.  sends/recvs: per-rank uint8 arrays."""
    p = len(plans)
    outs = [None] * p
    for r, P in enumerate(plans):
        if not P.has_combine or P.c_cnt == 0:
            continue
        E = P.esize
        lo, hi = P.c_src_off * E, (P.c_src_off + P.c_cnt) * E
        # phase A: rank r's staging slot s holds sends[s][lo:hi]
        for s in range(p):
            if s != r:
                assert P.a_recv[s].cnt in (0, P.c_cnt), "a_recv must cover the combine range"
                if P.a_recv[s].cnt:
                    assert plans[s].a_send[r].cnt == P.a_recv[s].cnt and plans[s].a_send[r].off == P.a_recv[s].off
        leaves = [sends[P.leaf[q]][lo:hi] for q in range(P.k)]
        folds = [sends[P.leaf_fold[q]][lo:hi] if P.leaf_fold[q] >= 0 else None for q in range(P.k)]
        out = run_plan_program(P, leaves, folds, P.c_cnt)
        outs[r] = out
        if not P.c_dst_tmp:
            d = P.c_dst_off * E
            recvs[r][d:d + out.size] = out
    # phase C
    for r, P in enumerate(plans):
        E = P.esize
        for d in range(p):
            if P.b_send[d].cnt:
                assert plans[d].b_recv[r].cnt == P.b_send[d].cnt and plans[d].b_recv[r].off == P.b_send[d].off
                o = P.b_send[d].off * E
                recvs[d][o:o + P.b_send[d].cnt * E] = outs[r][:P.b_send[d].cnt * E]
    return recvs
