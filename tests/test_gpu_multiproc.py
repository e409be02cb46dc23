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


def _launch(world, transport, suite, timeout):
    out = tempfile.mkdtemp(prefix="mvx_mp_")
    port = str(_port())
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
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
    reports = _launch(world, "host", "small", 240)
    for rep in reports:
        assert rep["checked"] > 100
        assert not rep["fails"], rep["fails"][:5]
        assert not rep["transport_errors"], rep["transport_errors"][:3]


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


@pytest.mark.parametrize("cfg", ["c3", "c4", "c5"])
def test_bench_multi_gpu_leg_host_transport(cfg):
    """The N > 1 bench leg under torchrun (2 ranks on one GPU, host
    transport): one JSON line with parity bit-exact for every exchange
    variant tried, and a 2-thread CPU baseline."""
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "3", "--warmup", "1", "--tune-steps", "1", "--mib", "32",
           "--config", cfg, "--transport", "host"]
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    line = [x for x in p.stdout.splitlines() if x.startswith("{")]
    assert len(line) == 1, p.stdout[-2000:]
    d = json.loads(line[0])
    assert d["n_gpus"] == 2 and d["value"] > 0
    assert d["parity"].startswith("bit-exact"), d
    assert all(v["parity"] for v in d["config"]["exchange_tuning"].values()), d["config"]["exchange_tuning"]
    assert d["cpu_baseline"]["cores"] == 2
    assert d["config"]["transport"] == "host"
    ph = d["roofline"]["phases"]
    assert ph["total_ms"] > 0, ph
