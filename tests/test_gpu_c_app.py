"""GPU: a C program against libmvx.so alone (tests/c_app.c) -- the MPI calls
a user of the reference compiles when switching: blocking Allreduce /
Reduce / Scan on host and device buffers, the reference's error codes, a
4-rank virtual communicator with known answers, a user op, MAXLOC on
MPI_FLOAT_INT.  Built with gcc here and run as its own process."""
import os
import subprocess
import tempfile

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def test_c_application():
    out = os.path.join(tempfile.mkdtemp(prefix="mvx_capp_"), "c_app")
    pkg = os.path.join(ROOT, "mvapich-cce_amd")
    subprocess.check_call(["gcc", "-O2", "-std=gnu99", "-Wall", "-Werror", "-D__HIP_PLATFORM_AMD__",
                           "-I/opt/rocm/include", "-I" + os.path.join(ROOT, "include"),
                           os.path.join(HERE, "c_app.c"), "-o", out, "-L" + pkg, "-lmvx",
                           "-L/opt/rocm/lib", "-lamdhip64", "-Wl,-rpath," + pkg, "-Wl,-rpath,/opt/rocm/lib"])
    p = subprocess.run([out], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0 and "c_app ok" in p.stdout, p.stdout[-2000:] + p.stderr[-2000:]
