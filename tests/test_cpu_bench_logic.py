"""CPU: bench.py's host-side logic at N > 1 -- which exchange variant is
timed for the line (bench.choose_variant) and what the plan says each rank
moves per phase (bench.plan_bytes, the denominators of the per-link rates)."""
import importlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def test_choose_variant_skips_failed_and_mismatched():
    names = ["p2p", "pipe", "pipe2", "pipe8", "coll"]
    tried = {"p2p": {"ms_per_step": 2.0, "parity": True},
             "pipe": {"ms_per_step": 1.0, "parity": False},          # fastest, wrong: never timed
             "pipe2": {"ms_per_step": None, "parity": None, "error": "x"},
             "pipe8": {"ms_per_step": 1.5, "parity": None},          # no reference: allowed
             "coll": {"ms_per_step": None, "parity": None, "error": "hung"}}
    assert bench.choose_variant(names, tried) == "pipe8"
    tried["pipe8"]["parity"] = False
    assert bench.choose_variant(names, tried) == "p2p"
    tried["p2p"]["ms_per_step"] = None
    assert bench.choose_variant(names, tried) is None
    # ties go to the earlier variant
    tied = {k: {"ms_per_step": 1.0, "parity": True} for k in names}
    assert bench.choose_variant(names, tied) == "p2p"


def test_plan_bytes_match_the_partition():
    mvx = importlib.import_module("mvapich-cce_amd")
    n = 1 << 20
    for p in (2, 4, 8):
        for r in range(p):
            b = bench.plan_bytes(mvx, "allreduce", p, r, n, None, bench.MPI_FLOAT, bench.MPI_SUM)
            blk = n // p * 4
            assert b["A"] == {"sent": (p - 1) * blk, "received": (p - 1) * blk, "max_per_peer": blk,
                              "peers": p - 1}
            assert b["C"] == b["A"]
            cn = [n // p] * p
            b = bench.plan_bytes(mvx, "reduce_scatter", p, r, n, cn, bench.MPI_LONG, bench.MPI_BAND)
            blk = n // p * 8
            assert b["A"]["received"] == (p - 1) * blk and b["A"]["max_per_peer"] == blk
            assert b["C"] == {"sent": 0, "received": 0, "max_per_peer": 0, "peers": 0}
    # MAXLOC at p = 2 is recursive doubling: the whole vector each way, no phase C
    b = bench.plan_bytes(mvx, "allreduce", 2, 0, n, None, bench.MPI_FLOAT_INT, bench.MPI_MAXLOC)
    assert b["A"]["sent"] == n * 8 and b["C"]["sent"] == 0


def test_rccl_net_env_gives_each_rank_its_own_host():
    """--transport rccl-net: distinct NCCL_HOSTID per rank (RCCL's
    duplicate-GPU check keys on host hash + bus id), loopback sockets, and a
    caller's own interface choice left alone."""
    tp = importlib.import_module("mvapich-cce_amd.transport")
    envs = [tp.rccl_net_env(r, {}) for r in range(8)]
    assert len({e["NCCL_HOSTID"] for e in envs}) == 8
    assert all(e["NCCL_SOCKET_IFNAME"] == "lo" and e["NCCL_IB_DISABLE"] == "1" for e in envs)
    assert tp.rccl_net_env(3, {"NCCL_SOCKET_IFNAME": "eth0"})["NCCL_SOCKET_IFNAME"] == "eth0"
