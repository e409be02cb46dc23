"""GPU: the C executor across process boundaries.

* Host transport (mvx_comm_init_transport + mvapich-cce_amd/transport.py):
  p = 2, 3, 4 processes share the test box's one GPU as separate ranks, each
  running exactly the RCCL path's plan / phase / combine code, with the
  bytes between ranks moved by gloo through host memory (RCCL refuses two
  ranks on one GPU).  All collectives, device and host buffers, both device
  exchange variants, against the oracle's replay of the reference schedule.
* RCCL over xGMI (mvx_comm_init): the same suite, plus the BASELINE
  multi-GPU shapes (C3, C4, C5) at full size, on p = 2, 4, 8 GPUs -- skipped
  where the box has fewer GPUs.
* RCCL with ranks sharing the one GPU (rccl-net: each rank its own
  NCCL_HOSTID, so RCCL's socket transport moves the bytes): the suites, the
  bench leg, and the bench's hang path (ncclCommAbort, a fresh communicator).
* bench.py under torchrun with the host transport: the multi-GPU leg
  (exchange tuning, parity against the CPU reference schedule, p-thread CPU
  baseline) end to end on one GPU.

Every worker is a fresh process (tests/mp_worker.py).
"""
import json
import os
import socket
import subprocess
import sys
import tempfile

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _ngpus():
    import torch
    return torch.cuda.device_count()


def _launch(world, transport, suite, timeout, extra_env=None):
    out = tempfile.mkdtemp(prefix="mvx_mp_")
    port = str(_port())
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    env.update(extra_env or {})
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "mp_worker.py"), str(r), str(world), port,
                               os.path.join(out, "r%d.json" % r), transport, suite], env=env)
             for r in range(world)]
    try:
        rcs = [p.wait(timeout=timeout) for p in procs]
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    assert rcs == [0] * world, rcs
    reports = []
    for r in range(world):
        with open(os.path.join(out, "r%d.json" % r)) as f:
            reports.append(json.load(f))
    return reports


@pytest.mark.parametrize("world", [2, 3, 4])
def test_executor_across_processes_host_transport(world):
    """Every exchange variant, COLL included: over the host transport its
    all-to-all / in-place all-gather run as the transport's alltoall /
    allgather hooks (gloo), with the staging layout, leaf pointers and
    gather offsets of the RCCL path."""
    reports = _launch(world, "host", "small", 300)
    for rep in reports:
        assert rep["checked"] > 100
        assert not rep["fails"], rep["fails"][:5]
        assert not rep["transport_errors"], rep["transport_errors"][:3]
        ran = rep["ran"]
        # the COLL variant ran whole on the regular plans (p equal blocks);
        # every other call under it reports the P2P fallback, never COLL
        assert ran["coll"].get("2", 0) > 0, ran
        assert ran["p2p"].get("2", 0) == 0 and ran["pipe"].get("2", 0) == 0, ran
        assert ran["p2p"].get("1", 0) == 0, ran
        if world > 1:
            assert ran["pipe"].get("1", 0) > 0, ran


@pytest.mark.parametrize("world", [2, 3])
def test_executor_random_host_transport(world):
    """A seeded random sweep (collective, op x datatype with the undefined
    pairs, count, root, exchange variant, device or host buffers) through the
    one-rank-per-process path; every rank's code and recvbuf against the
    oracle."""
    reports = _launch(world, "host", "random", 600)
    for rep in reports:
        assert rep["checked"] == int(os.environ.get("MVX_MP_CASES", "120")), rep["checked"]
        assert not rep["fails"], rep["fails"][:5]


@pytest.mark.parametrize("world", [2, 4, 8])
def test_rccl_multirank(world):
    if _ngpus() < world:
        pytest.skip("needs %d GPUs (RCCL refuses two ranks on one GPU)" % world)
    for suite in ("small", "random", "full"):
        for rep in _launch(world, "rccl", suite, 900):
            assert rep["checked"] > 0
            assert not rep["fails"], rep["fails"][:5]


@pytest.mark.parametrize("world", [2, 4])
def test_rccl_multirank_net_transport(world):
    """The RCCL executor itself at p > 1 on one GPU: each rank names itself
    a separate host (NCCL_HOSTID, transport.rccl_net_env), so RCCL accepts
    ranks that share the GPU and moves every byte through its socket
    transport -- the grouped ncclSend / ncclRecv of P2P and PIPE and the
    ncclAllToAll / in-place ncclAllGather of COLL, bit-exact against the
    oracle's replay."""
    for suite in ("small", "random"):
        for rep in _launch(world, "rccl-net", suite, 600):
            assert rep["checked"] > 0
            assert not rep["fails"], rep["fails"][:5]
            if suite == "small":
                ran = rep["ran"]
                assert ran["coll"].get("2", 0) > 0, ran
                assert ran["pipe"].get("1", 0) > 0, ran


@pytest.mark.parametrize("world,transport", [(2, "host"), (3, "host"), (2, "rccl-net"), (4, "rccl-net")])
def test_mixed_buffer_kinds_across_ranks(world, transport):
    """One call, different buffer kinds on different ranks (host on some,
    device on others -- legal MPI): the host ranks run on HBM mirrors and
    their transfers pair with the device ranks' under every exchange
    variant; every rank bit-exact against the oracle's replay."""
    for rep in _launch(world, transport, "mixed", 600):
        assert rep["checked"] > 50
        assert not rep["fails"], rep["fails"][:5]


@pytest.mark.parametrize("world,transport", [(2, "host"), (3, "host"), (2, "rccl-net"), (4, "rccl-net")])
def test_slice_schedule_any_kinds(world, transport):
    """The slice schedule of large blocking calls (a 1 MiB threshold and
    1 MiB slices here): every rank runs the same slices whatever its
    buffers' kind -- host ranks overlapping H2D / collective / D2H, device
    ranks issuing slices back to back -- so mixed kinds pair; all host and
    all device too; every collective, role-sensitive ops included,
    bit-exact against the oracle's replay."""
    for rep in _launch(world, transport, "sliced", 600):
        assert rep["checked"] >= 5 * 3 * 5 + 4
        assert not rep["fails"], rep["fails"][:5]
        assert set(rep["ran"]["sliced"]) <= {"0", "-1"}, rep["ran"]     # P2P slices
        # agreed kinds: all device ran the communicator's variant (PIPE, 1)
        # unsliced; all host the P2P slices; a hint rank 0 contradicts runs the
        # hint's schedule on every rank (checked bit-exact above)
        assert rep["agreed_ran"] == [["device", 1], ["host", 0]] * 2, rep["agreed_ran"]
        assert rep["contradicted"] == [1, 0] * 2, rep["contradicted"]


@pytest.mark.parametrize("world", [2, 4])
def test_graphs_rccl_net(world):
    """HIP graphs of RCCL device calls (mvx_comm_set_graphs) on RCCL
    communicators sharing the GPU: every job eager, then captured, then
    replayed -- on the null stream (fork / join) and on a torch stream --
    under P2P, PIPE and COLL; every result bit-exact against the oracle."""
    for rep in _launch(world, "rccl-net", "graph", 600):
        assert rep["checked"] > 100
        assert not rep["fails"], rep["fails"][:5]
        assert rep["graph_error"] == 0, rep["graph_error"]
        for key, runs in rep["graph_states"].items():
            # eager, captured, replayed -- or all eager once the
            # communicator holds its 32 graphs (none is destroyed before
            # mvx_comm_free, csrc/mvx_exec.c)
            assert all(st in ([0, 2, 1], [0, 0, 0]) for st in runs), (key, runs)
        assert sum(st == [0, 2, 1] for runs in rep["graph_states"].values() for st in runs) >= 16


@pytest.mark.parametrize("world", [2, 4])
def test_graphs_rccl_net_evicting(world):
    """The same with at most 4 graphs per communicator (MVX_GRAPH_CACHE=4),
    so graphs are destroyed mid-life: the least recently used one for each
    new job, and every one captured on a staging pool before the pool is
    reallocated -- on this process's HIP runtime (torch's 7.0) only graphs
    without parallel branches, the forked ones being kept (csrc/mvx_exec.c,
    DESIGN.md section 6: HIP 7.0 crashes in hipGraphLaunch once forked
    graphs were destroyed).  Every result bit-exact, the cap held; a crash
    would print the native stack (MVX_SEGV_BT)."""
    env = {"MVX_GRAPH_CACHE": "4", "MVX_SEGV_BT": "1"}
    for rep in _launch(world, "rccl-net", "graph", 600, env):
        assert rep["checked"] > 100
        assert not rep["fails"], rep["fails"][:5]
        assert rep["graph_error"] == 0, rep["graph_error"]
        for key, runs in rep["graph_states"].items():
            assert all(st in ([0, 2, 1], [0, 0, 0]) for st in runs), (key, runs)
        gs = rep["graph_stats"]
        assert gs["live"] + gs["retired"] <= 4, gs
        if rep["hip_runtime"] >= 70200000:
            assert gs["destroyed"] >= 10, gs
        # on HIP 7.0 the graphs RCCL's socket transport captures have
        # parallel branches (its proxy's host stream), so all are kept:
        # the cap holds and nothing crashes


def test_graphs_host_transport_stay_eager():
    """a caller-supplied transport (host callbacks) is never captured"""
    for rep in _launch(2, "host", "graph", 600):
        assert not rep["fails"], rep["fails"][:5]
        assert all(st == [0, 0, 0] for runs in rep["graph_states"].values() for st in runs)


def _bench_host(cfg, extra_env=None, world=2, transport="host", extra_args=()):
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    env.update(extra_env or {})
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", str(world), "--steps", "3", "--warmup", "1", "--tune-steps", "1", "--mib", "32",
           "--config", cfg, "--transport", transport] + list(extra_args)
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    return p


@pytest.mark.parametrize("cfg", ["c3", "c4", "c5"])
def test_bench_multi_gpu_leg_host_transport(cfg):
    """The N > 1 bench leg under torchrun (2 ranks on one GPU, host
    transport): one JSON line with parity bit-exact for every exchange
    variant tried -- each one reporting the variant that actually ran (COLL
    over the transport's alltoall / allgather hooks) -- a 2-thread CPU
    baseline, and every per-phase field the 8-GPU run prints."""
    p = _bench_host(cfg)
    assert p.returncode == 0, p.stderr[-3000:]
    line = [x for x in p.stdout.splitlines() if x.startswith("{")]
    assert len(line) == 1, p.stdout[-2000:]
    d = json.loads(line[0])
    assert d["n_gpus"] == 2 and d["value"] > 0
    assert d["parity"].startswith("bit-exact"), d
    tuning = d["config"]["exchange_tuning"]
    assert all(v["parity"] for v in tuning.values()), tuning
    # C5 (MAXLOC, role-sensitive) at p = 2 is recursive doubling with every
    # rank combining the whole vector as its own root:
    # not a regular plan, so COLL runs -- and reports -- the P2P fallback
    want_coll = "p2p (fallback)" if cfg == "c5" else "coll"
    assert tuning["p2p"]["ran"] == "p2p" and tuning["coll"]["ran"] == want_coll, tuning
    assert tuning["pipe"]["ran"] == "pipe", tuning
    assert d["config"]["exchange_ran"] == tuning[d["config"]["exchange"]]["ran"]
    assert d["cpu_baseline"]["cores"] == 2
    assert d["config"]["transport"] == "host"
    assert "rccl_native" not in d           # no RCCL handle under the host transport
    ph = d["roofline"]["phases"]
    assert ph["total_ms"] > 0, ph
    S = d["config"]["vector_bytes_per_rank"]
    # C3 / C4: reduce-scatter halves (+ all-gather for the Allreduce); C5 at
    # p = 2: the whole vector each way, every rank combining all of it
    a = S if cfg == "c5" else S // 2
    assert ph["A_bytes"]["received"] == ph["A_bytes"]["sent"] == a, ph
    assert ph["A_bytes"]["peers"] == 1 and ph["A_bytes"]["max_per_peer"] == a
    assert ph["C_bytes"]["received"] == (S // 2 if cfg == "c3" else 0), ph
    if d["config"]["exchange"] != "pipe" and not d["config"]["exchange"].startswith("pipe"):
        assert set(ph["A_GBs_per_rank"]) == {"sent", "received", "per_link", "link_frac"}, ph


@pytest.mark.parametrize("cfg", ["c3", "c4"])
def test_bench_multi_gpu_leg_rccl_net(cfg):
    """bench.py's N > 1 leg on RCCL communicators (2 ranks sharing the GPU,
    RCCL's socket transport): every exchange variant -- COLL as
    ncclAllToAll + ncclAllGather -- ran as itself with parity bit-exact."""
    p = _bench_host(cfg, transport="rccl-net", extra_args=("--graphs",))
    assert p.returncode == 0, p.stderr[-3000:]
    line = [x for x in p.stdout.splitlines() if x.startswith("{")]
    assert len(line) == 1, p.stdout[-2000:]
    d = json.loads(line[0])
    assert d["parity"].startswith("bit-exact"), d
    assert d["config"]["transport"] == "rccl-net"
    tuning = d["config"]["exchange_tuning"]
    assert all(v["parity"] for v in tuning.values()), tuning
    assert tuning["coll"]["ran"] == "coll" and tuning["p2p"]["ran"] == "p2p", tuning
    assert all(v["host_issue_us"] > 0 for v in tuning.values()), tuning
    # the graph variants: RCCL's groups captured into HIP graphs and replayed
    for name in ("p2p+g", "pipe+g", "pipe8+g", "coll+g"):
        assert tuning[name]["graph"] == {"state": "replayed", "capture_error": 0}, (name, tuning[name])
        assert tuning[name]["ran"] == tuning[name.split("+")[0]]["ran"], tuning
    # RCCL's own reduction on the same communicator, timed after the line
    nat = d["rccl_native"]
    assert nat["op"] == ("ncclAllReduce(ncclSum)" if cfg == "c3" else "ncclReduceScatter(ncclSum)"), nat
    assert nat["ms_per_step"] > 0 and nat["line_over_native"] > 0, nat


def test_bench_full_size_eight_ranks_rccl_net():
    """The driver's 8-GPU bench leg at the BASELINE sizes, with RCCL itself
    carrying the bytes between 8 ranks that share the GPU (rccl-net): C3
    (Allreduce SUM f32, 256 MiB per rank) with C5 (Allreduce MAXLOC
    FLOAT_INT, 512 MiB per rank) in other_configs, every exchange variant
    run as itself -- COLL as ncclAllToAll + in-place ncclAllGather at p = 8
    -- and every rank's result bit-exact against the reference schedule."""
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "8",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "8", "--steps", "2", "--warmup", "1", "--tune-steps", "1", "--transport", "rccl-net",
           "--graphs"]
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=420)
    assert p.returncode == 0, p.stderr[-3000:]
    line = [x for x in p.stdout.splitlines() if x.startswith("{")]
    assert len(line) == 1, p.stdout[-2000:]
    d = json.loads(line[0])
    assert d["n_gpus"] == 8 and d["config"]["vector_bytes_per_rank"] == 256 << 20
    assert d["parity"] == "bit-exact vs the reference schedule, all 8 ranks", d["parity"]
    tuning = d["config"]["exchange_tuning"]
    for name, v in tuning.items():
        base = name.split("+")[0]
        assert v["parity"] and v["ran"] == ("coll" if base == "coll" else base[:4]), (name, v)
        if name.endswith("+g"):
            assert v["graph"]["state"] == "replayed", (name, v)
    (o,) = d["other_configs"]
    assert o["config"] == "c5" and o["vector_bytes_per_rank"] == 512 << 20
    assert o["parity"] == "bit-exact vs the reference schedule, all 8 ranks", o


def test_bench_survives_a_hung_variant_rccl_net():
    """A variant whose checked step hangs (rank 1 never issues it: rank 0's
    RCCL transfers wait for a peer that never comes, MVX_BENCH_HANG) is
    detected by the variant timeout, every rank aborts its RCCL communicator
    (ncclCommAbort) and builds a fresh one, and the later variants -- COLL
    included -- still run on it with parity bit-exact."""
    p = _bench_host("c3", {"MVX_BENCH_HANG": "pipe@1"}, transport="rccl-net",
                    extra_args=["--variant-timeout", "15"])
    assert p.returncode == 0, p.stderr[-3000:]
    line = [x for x in p.stdout.splitlines() if x.startswith("{")]
    assert len(line) == 1, p.stdout[-2000:]
    d = json.loads(line[0])
    tuning = d["config"]["exchange_tuning"]
    assert tuning["pipe"]["ms_per_step"] is None and "did not complete" in tuning["pipe"]["error"], tuning
    assert "stayed blocked" not in tuning["pipe"]["error"], tuning
    for v in ("p2p", "pipe2", "pipe8", "coll"):
        assert tuning[v]["parity"] and tuning[v]["ms_per_step"], tuning
    assert tuning["coll"]["ran"] == "coll", tuning
    assert d["parity"].startswith("bit-exact"), d


@pytest.mark.parametrize("bad", ["coll@1", "p2p@0,pipe8@1"])
def test_bench_survives_a_failing_variant(bad):
    """A variant that returns an error on one rank (MVX_BENCH_FAIL) is
    recorded and left out; the line still comes, from the other variants,
    with parity bit-exact."""
    p = _bench_host("c3", {"MVX_BENCH_FAIL": bad})
    assert p.returncode == 0, p.stderr[-3000:]
    line = [x for x in p.stdout.splitlines() if x.startswith("{")]
    assert len(line) == 1, p.stdout[-2000:]
    d = json.loads(line[0])
    tuning = d["config"]["exchange_tuning"]
    failed = [x.split("@")[0] for x in bad.split(",")]
    for v in failed:
        assert tuning[v]["ms_per_step"] is None and "error" in tuning[v], tuning
    assert d["config"]["exchange"] not in failed
    assert d["parity"].startswith("bit-exact"), d


def test_bench_no_clean_variant_exits_nonzero():
    """Every variant failing: no throughput line, a nonzero exit."""
    sys.path.insert(0, ROOT)
    import bench
    p = _bench_host("c3", {"MVX_BENCH_FAIL": ",".join("%s@1" % v for v in bench.EXCH)})
    assert p.returncode != 0
    assert not [x for x in p.stdout.splitlines() if x.startswith("{")]


def test_bench_line_carries_the_other_baseline_configs():
    """At N = 4 the line also carries C4 (Reduce_scatter BAND int64) measured
    after the timed region on the same communicator: its own parity against
    the reference schedule, time and bus bandwidth (host transport, 4 ranks
    on one GPU, small vectors)."""
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "4",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "4", "--steps", "2", "--warmup", "1", "--tune-steps", "1", "--mib", "16",
           "--transport", "host"]
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=400)
    assert p.returncode == 0, p.stderr[-3000:]
    line = [x for x in p.stdout.splitlines() if x.startswith("{")]
    assert len(line) == 1, p.stdout[-2000:]
    d = json.loads(line[0])
    assert d["config"]["workload"].startswith("c3") and d["parity"].startswith("bit-exact")
    (o,) = d["other_configs"]
    assert o["config"] == "c4" and o["parity"].startswith("bit-exact"), o
    assert o["value"] > 0 and o["busbw_GBs"] > 0 and o["exchange"] == d["config"]["exchange"]


def _bench_self(world, transport, extra=(), extra_env=None):
    """bench.py in the driver's own form -- no torchrun, no WORLD_SIZE:
    --gpus N starts its N workers itself (bench.launch)."""
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_PORT")}
    env["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"
    env.update(extra_env or {})
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(world), "--steps", "2", "--warmup", "1",
           "--tune-steps", "1", "--mib", "16", "--transport", transport] + list(extra)
    return subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=400)


def _one_line(p):
    assert p.returncode == 0, p.stderr[-3000:]
    line = [x for x in p.stdout.splitlines() if x.startswith("{")]
    assert len(line) == 1, p.stdout[-2000:]
    return json.loads(line[0])


@pytest.mark.parametrize("transport", ["host", "rccl-net"])
def test_bench_self_launch_driver_form(transport):
    """`python3 bench.py --gpus 2 ...` with no launcher prints ONE 2-rank
    line: n_gpus 2, parity bit-exact on both ranks, the launcher's record,
    RCCL's own rank count (rccl-net: ncclCommCount = 2, one device per rank),
    the env knobs echoed, and per-stage wall times that add up to the run's
    wall clock."""
    d = _one_line(_bench_self(2, transport))
    assert d["n_gpus"] == 2 and d["value"] > 0
    assert d["parity"] == "bit-exact vs the reference schedule, all 2 ranks", d["parity"]
    assert d["launch"]["workers"] == 2 and d["launch"]["worker_rcs"] == [0, 0], d["launch"]
    r = d["rccl"]
    assert r["transport"] == transport and len(r["hip_devices"]) == 2
    if transport == "rccl-net":
        assert r["nranks"] == 2 and len(r["devices"]) == 2 and r["version"] > 0, r
    else:
        assert r["nranks"] is None, r
    assert d["env"].get("HSA_ENABLE_IPC_MODE_LEGACY") == "0"
    w = d["wall"]
    total = sum(w["stage_s"].values()) + w["unaccounted_s"]
    assert abs(total - w["wall_s"]) <= 0.05 * w["wall_s"], w
    assert w["wall_s"] <= d["launch"]["wall_s"] + 1.0, (w, d["launch"])
    assert any(k.startswith("variant ") for k in w["stage_s"]), w


def test_bench_self_launch_worker_failure_exits_nonzero():
    """Workers that end without a line take the job down: the launcher exits
    with their worst code and prints no line (every variant fails on rank 1)."""
    sys.path.insert(0, ROOT)
    import bench
    p = _bench_self(2, "host", extra_env={"MVX_BENCH_FAIL": ",".join("%s@1" % v for v in bench.EXCH)})
    assert p.returncode != 0
    assert not [x for x in p.stdout.splitlines() if x.startswith("{")]


def test_bench_self_launch_rccl_xgmi():
    """The same over RCCL proper when the box has 2 GPUs (on the node: xGMI)."""
    if _ngpus() < 2:
        pytest.skip("needs 2 GPUs")
    d = _one_line(_bench_self(2, "rccl"))
    assert d["n_gpus"] == 2 and d["rccl"]["nranks"] == 2 and d["rccl"]["distinct_gpus"] == 2, d["rccl"]
    assert d["parity"].startswith("bit-exact"), d
