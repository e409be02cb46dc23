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


def test_launch_decision():
    """--gpus N without a launcher starts N workers itself; under a launcher
    --gpus must name the launcher's world size (or be absent)."""
    assert bench.decide_launch(None, {}) == ("single", 1)
    assert bench.decide_launch(1, {}) == ("single", 1)
    assert bench.decide_launch(8, {}) == ("self", 8)
    assert bench.decide_launch(8, {"WORLD_SIZE": "8"}) == ("worker", 8)
    assert bench.decide_launch(None, {"WORLD_SIZE": "4"}) == ("worker", 4)
    assert bench.decide_launch(1, {"WORLD_SIZE": "1"}) == ("single", 1)
    how, msg = bench.decide_launch(8, {"WORLD_SIZE": "2"})
    assert how == "mismatch" and "WORLD_SIZE=2" in msg
    assert bench.decide_launch(0, {})[0] == "mismatch"


def test_worker_env_is_torchrun_shaped():
    env = bench.worker_env({"PATH": "/bin", "HSA_ENABLE_IPC_MODE_LEGACY": "0"}, 3, 8, 29500)
    assert env["RANK"] == env["LOCAL_RANK"] == "3"
    assert env["WORLD_SIZE"] == env["LOCAL_WORLD_SIZE"] == "8"
    assert env["MASTER_ADDR"] == "127.0.0.1" and env["MASTER_PORT"] == "29500"
    assert env["HSA_ENABLE_IPC_MODE_LEGACY"] == "0" and env["PATH"] == "/bin"
    assert bench.decide_launch(8, env) == ("worker", 8)
    assert bench._rc_of(0) == 0 and bench._rc_of(1) == 1 and bench._rc_of(-9) == 137


def test_mismatched_world_exits_nonzero_before_any_gpu_work():
    """WORLD_SIZE from a launcher that disagrees with --gpus: exit 2 at once
    (main() returns before importing torch)."""
    import subprocess
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4"], env=env,
                       capture_output=True, text=True, timeout=60)
    assert p.returncode == 2, (p.returncode, p.stderr)
    assert "WORLD_SIZE=2" in p.stderr and not p.stdout.strip()


def test_self_launch_refuses_more_rccl_ranks_than_gpus(tmp_path):
    """A topology with no GPU node (a CPU-only KFD tree): --gpus 2 over RCCL
    cannot place its ranks, so the launcher says so and exits 2 before
    starting workers."""
    import subprocess
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["MVX_KFD_NODES"] = _fake_kfd(tmp_path, [{"simd_count": 0}])
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 2, (p.returncode, p.stderr[-2000:])
    assert "needs 2 GPUs" in p.stderr


def test_stages_partition_the_wall_clock():
    st = bench.Stages()
    st.mark("a")
    st.mark("b")
    st.mark("a")
    r = st.report()
    assert set(r["stage_s"]) == {"a", "b"}
    assert abs(sum(r["stage_s"].values()) + r["unaccounted_s"] - r["wall_s"]) < 0.01


def test_env_echo_keeps_only_the_knobs():
    e = bench.env_echo({"NCCL_DEBUG": "INFO", "HOME": "/root", "MVX_EXCHANGE": "coll", "RCCL_X": "1",
                        "HSA_ENABLE_IPC_MODE_LEGACY": "0"})
    assert e == {"HSA_ENABLE_IPC_MODE_LEGACY": "0", "MVX_EXCHANGE": "coll", "NCCL_DEBUG": "INFO", "RCCL_X": "1"}


def test_auto_variants_leave_graphs_to_the_flag():
    """--exchange auto tries the eager variants; the HIP-graph ones only with
    --graphs (untested over xGMI), after the eager ones"""
    eager = bench.auto_variants(bench.parse([]))
    assert eager == ["p2p", "pipe", "pipe2", "pipe8", "coll"]
    both = bench.auto_variants(bench.parse(["--graphs"]))
    assert both[:5] == eager and all(n.endswith("+g") for n in both[5:]) and len(both) == 10
    assert bench.parse(["--exchange", "pipe+g"]).exchange == "pipe+g"


def _fake_kfd(tmp, props):
    """a KFD topology tree: one node directory per properties dict"""
    for i, p in enumerate(props):
        d = tmp / "nodes" / str(i)
        d.mkdir(parents=True)
        (d / "properties").write_text("".join("%s %s\n" % kv for kv in p.items()))
    return str(tmp / "nodes")


def test_visible_gpus_from_kfd_topology(tmp_path):
    """GPU nodes are the ones with SIMDs; ROCR_VISIBLE_DEVICES, then
    HIP_VISIBLE_DEVICES (indices or GPU-<unique_id>) narrow them"""
    cpu = {"cpu_cores_count": 64, "simd_count": 0, "unique_id": 0}
    gpus = [{"cpu_cores_count": 0, "simd_count": 1024, "unique_id": 0x1000 + i} for i in range(8)]
    root = _fake_kfd(tmp_path, [cpu, cpu] + gpus)
    assert bench.visible_gpus({}, root) == 8
    assert bench.visible_gpus({"HIP_VISIBLE_DEVICES": "0,3"}, root) == 2
    assert bench.visible_gpus({"ROCR_VISIBLE_DEVICES": "1,2,5", "HIP_VISIBLE_DEVICES": "2"}, root) == 1
    assert bench.visible_gpus({"ROCR_VISIBLE_DEVICES": "GPU-%016x,GPU-%016x" % (0x1003, 0x1004)}, root) == 2
    assert bench.visible_gpus({"CUDA_VISIBLE_DEVICES": "0,9"}, root) == 1      # stops at the invalid one
    assert bench.visible_gpus({}, str(tmp_path / "absent")) is None


def test_launcher_counts_gpus_without_torch(tmp_path, monkeypatch):
    """bench.py --gpus N (no launcher, --transport rccl) decides whether the
    box has N GPUs and starts its workers without importing torch: with torch
    poisoned in sys.modules, 2 fake GPUs lead to 2 Popen calls, 1 fake GPU to
    exit code 2 and none."""
    import subprocess
    import types
    root = _fake_kfd(tmp_path, [{"simd_count": 0}] + [{"simd_count": 1024, "unique_id": i + 1} for i in range(2)])
    monkeypatch.setitem(sys.modules, "torch", None)      # `import torch` raises ImportError
    monkeypatch.setenv("MVX_KFD_NODES", root)
    for var in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(var, raising=False)
    started = []

    class FakeProc:
        def __init__(self, cmd, env=None, stdout=None, preexec_fn=None):
            started.append(env["RANK"])
            self.returncode = 0
            self.stdout = types.SimpleNamespace(read=lambda: b"")

        def poll(self):
            return 0

        def kill(self):
            pass

    monkeypatch.setattr(subprocess, "Popen", FakeProc)
    args = types.SimpleNamespace(transport="rccl", launch_grace=1.0)
    assert bench.launch(args, 2, ["--gpus", "2"]) == 0
    assert started == ["0", "1"]
    started.clear()
    assert bench.launch(args, 3, ["--gpus", "3"]) == 2 and started == []


def test_mix_ceiling_summary():
    """bench.ceiling_summary: the additive bound is 3 vectors over the
    read-both plus write-one times; the mixed line sits two thirds of the way
    from the read-only rate to the copy rate (write share 1/3 of 1/2)."""
    sys.path.insert(0, ROOT)
    import bench
    nb = 1 << 28
    us = {"read2": 80.0, "write1": 40.0, "copy": 90.0}
    d = bench.ceiling_summary(nb, us, 6400.0)
    read, copy = 2 * nb / 80e-6 / 1e9, 2 * nb / 90e-6 / 1e9
    assert abs(d["additive_GBs"] - 3 * nb / 120e-6 / 1e9) < 0.1
    assert abs(d["mixed_line_GBs"] - (read + (copy - read) * 2 / 3)) < 0.1
    assert d["frac_of_additive"] == round(6400.0 / (3 * nb / 120e-6 / 1e9), 4)
    assert copy < d["mixed_line_GBs"] < read


_CHATTER = r'''
import datetime, os, sys
sys.path.insert(0, sys.argv[1])
import torch.distributed as dist
import bench
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
with bench._StdoutToStderr():
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=60))
    dist.barrier()
if rank == 0:
    print('{"metric": "x"}')
dist.destroy_process_group()
'''


def test_gloo_connection_report_stays_off_stdout(tmp_path):
    """gloo prints each rank's connection count on stdout when the process
    group forms; under torchrun every rank's stdout is the driver's, which
    reads rank 0's one JSON line there.  bench.py forms the group inside
    _StdoutToStderr: stdout is the JSON line alone."""
    import socket
    import subprocess
    script = tmp_path / "chatter.py"
    script.write_text(_CHATTER)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "3",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), str(script), repo],
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.strip().splitlines() == ['{"metric": "x"}'], r.stdout
