"""GPU: HIP graphs of the executor from a C application (tools/graph_app.c)
on the image's own ROCm runtime -- two processes sharing the GPU as an RCCL
communicator (socket transport), graphs on, each exchange variant's
Allreduce run eagerly, captured, then replayed, blocking and
stream-ordered, every result checked in the app.
The same library from Python runs on torch's bundled HIP / RCCL instead
(tests/test_gpu_multiproc.py::test_graphs_rccl_net)."""
import os
import re
import subprocess

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
APP = os.path.join(ROOT, "tools", "graph_app")


def test_graphs_of_every_variant_from_c():
    if not os.path.exists(APP):
        pytest.skip("tools/graph_app not built (__graft_entry__.build)")
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    p = subprocess.run([APP], env=env, capture_output=True, text=True, timeout=150)
    assert p.returncode == 0 and "graph_app: ok" in p.stdout, (p.returncode, p.stderr[-3000:])
    # per rank, variant and way of calling: eager, captured, replayed
    states = re.findall(r"rank (\d): +ok, graph state (\d) error (\d)", p.stderr)
    assert len(states) == 36, p.stderr[-2000:]
    for r in "01":
        seq = [int(s) for rank, s, e in states if rank == r]
        assert seq == [0, 2, 1] * 6, (r, seq)
        assert all(e == "0" for rank, s, e in states)


def test_graphs_evicted_from_c_on_rocm72():
    """On the image's ROCm 7.2 runtime every graph may be destroyed
    mid-life: one graph per communicator (MVX_GRAPH_CACHE=1) and 6 job sizes
    x 3 variants x 2 ways of calling, so each new job destroys the previous
    graph -- PIPE's forked ones included -- and every job still goes eager,
    captured, replayed with every result checked (HIP 7.0, torch's runtime,
    crashes on the same sequence: tools/graph_probe2.c churn_fork_norccl)."""
    if not os.path.exists(APP):
        pytest.skip("tools/graph_app not built (__graft_entry__.build)")
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", MVX_GRAPH_CACHE="1", MVX_APP_SIZES="6",
               MVX_GRAPH_TRACE="1")
    env.pop("MVX_GRAPH_EVICT", None)
    p = subprocess.run([APP], env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0 and "graph_app: ok" in p.stdout, (p.returncode, p.stderr[-3000:])
    states = re.findall(r"rank (\d): +ok, graph state (\d) error (\d)", p.stderr)
    assert len(states) == 6 * 36, len(states)
    for r in "01":
        seq = [int(s) for rank, s, e in states if rank == r]
        assert seq == [0, 2, 1] * 36, (r, seq)
    destroys = p.stderr.count("destroy graph of variant")
    forked = p.stderr.count("instantiated graph has parallel branches 1")
    assert destroys >= 2 * 34 and forked > 0, (destroys, forked)
