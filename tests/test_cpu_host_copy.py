"""The host copy pool (mvx_pcopy, mvx_host.c) that fills and drains the
pinned bounce slots of host-buffer collectives: every byte of every size is
copied -- ragged sizes included (a split that rounded bytes / n down lost the
last bytes % n bytes whenever bytes / n fell on a 4 KiB boundary)."""
import ctypes

import numpy as np
import pytest


@pytest.mark.parametrize("nbytes", [1, 4095, (1 << 20) - 1, 1 << 20, (1 << 20) + 4, 8 * (1 << 20) + 3,
                                    8 * (1 << 20) + 7, 5_000_001, 3 * (1 << 20) + 5, 32 * (1 << 20) + 1])
def test_pcopy_copies_every_byte(mvx, nbytes):
    lib = mvx.coll()
    lib.mvx_pcopy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
    lib.mvx_pcopy.restype = None
    rng = np.random.default_rng(nbytes)
    src = rng.integers(0, 256, nbytes + 64, dtype=np.uint8)
    dst = np.zeros(nbytes + 64, np.uint8)
    lib.mvx_pcopy(dst.ctypes.data, src.ctypes.data, nbytes)
    assert np.array_equal(dst[:nbytes], src[:nbytes])
    assert not dst[nbytes:].any()          # nothing past the end


@pytest.mark.parametrize("threads", [1, 2, 3, 8])
def test_pcopy_thread_counts(threads, tmp_path):
    """Fresh processes with MVX_COPY_THREADS = 1, 2, 3, 8: ragged sizes
    around every split boundary."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = r'''
import ctypes, numpy as np, sys
lib = ctypes.CDLL(sys.argv[1])
lib.mvx_pcopy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
lib.mvx_pcopy.restype = None
n = lib.mvx_copy_threads()
assert n == int(sys.argv[2]), n
for base in (1 << 20, 4096 * n * 64, 4096 * n * 257):
    for extra in range(-3, 2 * n + 1):
        nb = base + extra
        s = np.random.default_rng(nb).integers(0, 256, nb, dtype=np.uint8)
        d = np.zeros(nb, np.uint8)
        lib.mvx_pcopy(d.ctypes.data, s.ctypes.data, nb)
        assert np.array_equal(d, s), (n, nb)
print("ok")
'''
    env = dict(os.environ, MVX_COPY_THREADS=str(threads))
    lib = os.path.join(root, "mvapich-cce_amd", "libmvx.so")
    ncpu = os.cpu_count() or 1
    p = subprocess.run([sys.executable, "-c", code, lib, str(min(threads, ncpu))], env=env,
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 0 and "ok" in p.stdout, p.stderr[-2000:]


def test_pcopy_concurrent_callers(mvx):
    """Several threads copying at once (ctypes drops the GIL around each
    call): every job completes whole -- callers queue behind one another
    instead of overwriting the pool's one job record."""
    import threading
    lib = mvx.coll()
    lib.mvx_pcopy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
    lib.mvx_pcopy.restype = None
    bad = []

    def worker(t):
        rng = np.random.default_rng(100 + t)
        for i in range(30):
            nb = int(rng.integers(1 << 20, 6 << 20))
            s = rng.integers(0, 256, nb, dtype=np.uint8)
            d = np.zeros(nb, np.uint8)
            lib.mvx_pcopy(d.ctypes.data, s.ctypes.data, nb)
            if not np.array_equal(d, s):
                bad.append((t, i, nb))

    ts = [threading.Thread(target=worker, args=(t,)) for t in range(4)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(120)
    assert not any(t.is_alive() for t in ts)
    assert not bad, bad[:5]
