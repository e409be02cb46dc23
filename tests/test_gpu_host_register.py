"""GPU: the registration cache for pageable host buffers (mvx_host.c;
MVAPICH's dreg, mpid/ch_gen2/dreg.c:774-832).

With the cache on, a pageable range a call uses is page-locked on first use
and found again on later calls (hits), so those DMA directly.

A registration must not outlive its memory: in round 4 a DMA through a
registration whose buffer had been freed and allocated again at the same
address faulted the GPU.  libmvx.so now interposes the calls that release
memory (free, realloc, munmap, mremap, madvise, sbrk) and drops the
registrations inside a released range first (the reference's mem_hooks.c).
test_free_and_reallocate_without_unregister runs that case in a C program
linked with -lmvx (tests/reg_app.c: free and munmap with no unregister call,
the same addresses handed out again), which checks the entries are gone
before it makes the second DMA.  This Python process loads libmvx.so with
ctypes, where the hooks are not the process's (mode 2 of the cache: the test
unregisters before it frees).  Results are checked against numpy or the CPU
(sums of small integers in float32 are exact).
"""
import os
import subprocess
import tempfile

import ctypes
import importlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
MIB = 1 << 20


@pytest.fixture()
def mvx():
    m = importlib.import_module("mvapich-cce_amd")
    m.host_register_enable(True)
    yield m
    m.host_register_enable(False)


def _libc_buffer(nbytes):
    """malloc'd memory (mmap'd at this size: free() unmaps it, the next
    malloc of the same size usually maps the same range again)"""
    libc = ctypes.CDLL("libc.so.6")
    libc.malloc.restype = ctypes.c_void_p
    libc.malloc.argtypes = [ctypes.c_size_t]
    libc.free.argtypes = [ctypes.c_void_p]
    p = libc.malloc(nbytes)
    assert p
    return libc, p


def _as_array(p, n):
    return np.ctypeslib.as_array((ctypes.c_float * n).from_address(p))


def _sum_call(mvx, x, y, n):
    mvx.MPIR_call("MPIR_SUM", x, y, n, mvx.MPI_FLOAT)
    assert mvx.op_errno() == 0


@pytest.mark.parametrize("mib", [2, 80])
def test_repeat_calls_hit_the_cache(mvx, mib):
    """the first call registers both operands, later calls find them"""
    n = mib * MIB // 4
    rng = np.random.default_rng(mib)
    a = rng.integers(-8, 8, n).astype(np.float32)
    b = rng.integers(-8, 8, n).astype(np.float32)
    want = a + b
    s0 = mvx.host_register_stats()
    for rep in range(3):
        y = b.copy() if rep == 0 else y
        if rep:
            np.copyto(y, b)
        _sum_call(mvx, a, y, n)
        assert np.array_equal(y, want), rep
    s1 = mvx.host_register_stats()
    # both operands registered: an entry each, or one union when their
    # allocations share a page (the call's own operands merge)
    assert s1["misses"] - s0["misses"] == 2, (s0, s1)
    assert s1["entries"] - s0["entries"] >= 1 and s1["bytes"] - s0["bytes"] >= 2 * n * 4, (s0, s1)
    assert s1["hits"] - s0["hits"] >= 4, (s0, s1)
    assert mvx.host_unregister(a) == 0
    mvx.host_unregister(y)                      # its own entry, or gone with a's union
    assert mvx.host_unregister(a) != 0          # nothing left at that address


def test_free_and_reallocate_without_unregister():
    """A C program linked with -lmvx (cache mode 1, the release hooks in
    effect): two registered 96 MiB malloc'd buffers freed with no
    mvx_host_unregister, the same size allocated again, reduced again --
    bit-exact, and the hooks dropped the stale registrations before the
    second DMA (the program stops before that DMA otherwise).  The same for
    mmap'd buffers unmapped and mapped again at the same address."""
    here = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(here)
    out = os.path.join(tempfile.mkdtemp(prefix="mvx_reg_"), "reg_app")
    pkg = os.path.join(root, "mvapich-cce_amd")
    subprocess.check_call(["gcc", "-O2", "-std=gnu99", "-Wall", "-Werror", "-D__HIP_PLATFORM_AMD__",
                           "-I/opt/rocm/include", "-I" + os.path.join(root, "include"),
                           os.path.join(here, "reg_app.c"), "-o", out, "-L" + pkg, "-lmvx",
                           "-L/opt/rocm/lib", "-lamdhip64", "-Wl,-rpath," + pkg, "-Wl,-rpath,/opt/rocm/lib"])
    env = {k: v for k, v in os.environ.items() if not k.startswith("MVX_HOST_REGISTER")}
    p = subprocess.run([out, "gpu"], capture_output=True, text=True, timeout=120, env=env)
    assert p.returncode == 0 and "reg_app ok" in p.stdout, p.stdout[-2000:] + p.stderr[-2000:]
    print(p.stdout)


def test_neighbour_frees_and_deferred_release_under_dma():
    """tests/reg_app.c neighbour (cache mode 1, the hooks in effect): two
    registered 64 MiB heap buffers reduced on the device 24 times while a
    second thread frees and reallocates the small blocks that share their
    boundary pages -- no registration is dropped, every result bit-exact, no
    fault (round 5's hooks unregistered the buffer under the DMA).  Then the
    second thread reports a release of an operand while a call holds it: the
    unregistration waits for the call (dreg.c:725-733) and follows it."""
    here = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(here)
    out = os.path.join(tempfile.mkdtemp(prefix="mvx_reg_"), "reg_app")
    pkg = os.path.join(root, "mvapich-cce_amd")
    subprocess.check_call(["gcc", "-O2", "-std=gnu99", "-Wall", "-Werror", "-D__HIP_PLATFORM_AMD__",
                           "-I/opt/rocm/include", "-I" + os.path.join(root, "include"),
                           os.path.join(here, "reg_app.c"), "-o", out, "-L" + pkg, "-lmvx",
                           "-L/opt/rocm/lib", "-lamdhip64", "-lpthread", "-Wl,-rpath," + pkg,
                           "-Wl,-rpath,/opt/rocm/lib"])
    env = {k: v for k, v in os.environ.items() if not k.startswith("MVX_HOST_REGISTER")}
    p = subprocess.run([out, "neighbour"], capture_output=True, text=True, timeout=180, env=env)
    assert p.returncode == 0 and "reg_app ok" in p.stdout, p.stdout[-2000:] + p.stderr[-2000:]
    print(p.stdout)


def test_buffers_under_a_neighbours_registration():
    """tests/reg_app.c shadow: HIP refuses a copy that starts inside a
    registration and runs past it (tools/shadow_probe.c), so a buffer whose
    first page another buffer's registration covers is merged with it (the
    same call's operands: one registration) or, while another call holds that
    registration, copied by the CPU -- a 2-rank Allreduce on a virtual
    communicator beside a thread that keeps reducing the neighbour.  Every
    result bit-exact."""
    here = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(here)
    out = os.path.join(tempfile.mkdtemp(prefix="mvx_reg_"), "reg_app")
    pkg = os.path.join(root, "mvapich-cce_amd")
    subprocess.check_call(["gcc", "-O2", "-std=gnu99", "-Wall", "-Werror", "-D__HIP_PLATFORM_AMD__",
                           "-I/opt/rocm/include", "-I" + os.path.join(root, "include"),
                           os.path.join(here, "reg_app.c"), "-o", out, "-L" + pkg, "-lmvx",
                           "-L/opt/rocm/lib", "-lamdhip64", "-lpthread", "-Wl,-rpath," + pkg,
                           "-Wl,-rpath,/opt/rocm/lib"])
    env = {k: v for k, v in os.environ.items() if not k.startswith("MVX_HOST_REGISTER")}
    p = subprocess.run([out, "shadow"], capture_output=True, text=True, timeout=180, env=env)
    assert p.returncode == 0 and "reg_app ok" in p.stdout, p.stdout[-2000:] + p.stderr[-2000:]
    print(p.stdout)


def test_adjacent_operands_share_a_registration(mvx):
    """Mode 2 (this process): two 8 MiB host operands, the second starting in
    the first's last page (carved from one malloc'd block, as back-to-back
    heap chunks lie), reduced by one op call -- the first's registration (held
    by the call) merges with the second's into one, no HIP copy refused,
    bit-exact; then unregistered before the free."""
    libc = ctypes.CDLL("libc.so.6")
    libc.malloc.restype = ctypes.c_void_p
    libc.malloc.argtypes = [ctypes.c_size_t]
    libc.free.argtypes = [ctypes.c_void_p]
    n = 8 * MIB // 4
    base = libc.malloc(2 * n * 4 + 3 * 4096)
    assert base
    px = (base + 4095) // 4096 * 4096 + 64    # x ends 64 bytes into a page
    py = px + n * 4 + 16                      # y starts 16 bytes later, same page
    assert (px + n * 4 - 1) // 4096 == py // 4096
    x, y = _as_array(px, n), _as_array(py, n)
    rng = np.random.default_rng(3)
    x[:] = rng.integers(-8, 8, n).astype(np.float32)
    y[:] = rng.integers(-8, 8, n).astype(np.float32)
    want = x + y
    st0 = mvx.host_register_stats()
    _sum_call(mvx, px, py, n)
    ok = bool(np.array_equal(y, want))
    st = mvx.host_register_stats()
    mvx.host_unregister(px)
    mvx.host_unregister(py)
    libc.free(base)
    assert ok and st["entries"] - st0["entries"] == 1, (st0, st)


def test_free_and_reallocate_same_size(mvx):
    """Mode 2 (this process's contract): a registered buffer is
    unregistered, freed and the same size allocated again (the same address
    in practice); the call on the new buffer must see its new contents."""
    n = 96 * MIB // 4
    libc, px = _libc_buffer(n * 4)
    _, py = _libc_buffer(n * 4)
    x, y = _as_array(px, n), _as_array(py, n)
    x[:] = 1.0
    y[:] = 2.0
    _sum_call(mvx, px, py, n)
    assert np.all(y == 3.0)
    assert mvx.host_unregister(px) == 0 and mvx.host_unregister(py) == 0
    libc.free(px)
    libc.free(py)
    qx = _libc_buffer(n * 4)[1]
    qy = _libc_buffer(n * 4)[1]
    x2, y2 = _as_array(qx, n), _as_array(qy, n)
    rng = np.random.default_rng(7)
    x2[:] = rng.integers(-8, 8, n).astype(np.float32)
    y2[:] = rng.integers(-8, 8, n).astype(np.float32)
    want = x2 + y2
    _sum_call(mvx, qx, qy, n)
    same = (qx == px, qy == py)
    ok = bool(np.array_equal(y2, want))
    mvx.host_unregister(qx)
    mvx.host_unregister(qy)
    libc.free(qx)
    libc.free(qy)
    assert ok, "reallocated buffers (same address: %s) reduced stale data" % (same,)


def test_cache_off_leaves_pageable_path(mvx):
    """turned off, nothing is registered and results are unchanged"""
    mvx.host_register_enable(False)
    n = 70 * MIB // 4
    a = np.full(n, 1.5, np.float32)
    b = np.full(n, 2.0, np.float32)
    _sum_call(mvx, a, b, n)
    assert np.all(b == 3.5)
    assert mvx.host_register_stats()["entries"] == 0


def test_partial_overlap_is_widened(mvx):
    """a call on a longer range than the one registered replaces the
    registration with the union (no DMA past pinned pages)"""
    n = 64 * MIB // 4
    a = np.ones(2 * n, np.float32)
    b = np.ones(2 * n, np.float32)
    _sum_call(mvx, a[:n], b[:n], n)
    assert np.all(b[:n] == 2.0) and np.all(b[n:] == 1.0)
    _sum_call(mvx, a, b, 2 * n)
    assert np.all(b[:n] == 3.0) and np.all(b[n:] == 2.0)
    st = mvx.host_register_stats()
    assert st["bytes"] >= 2 * (2 * n * 4), st
    mvx.host_unregister(a)
    mvx.host_unregister(b)
