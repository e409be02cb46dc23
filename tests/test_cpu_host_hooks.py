"""The registration cache's release hooks on the CPU (csrc/mvx_host.c; the
reference's mem_hooks.c:97-132 -> dreg.c:1063 find_and_free_dregs_inside).

tests/reg_app.c, linked with -lmvx so libmvx.so's free / realloc / munmap /
mremap / madvise / sbrk are the process's, registers ranges in the cache's
dry mode (MVX_HOST_REGISTER_DRY=1: ranges tracked, nothing page-locked --
no GPU here) and releases them every way: each release drops the entries it
overlaps, an unrelated free keeps them.  In this process (libmvx.so loaded
with ctypes) the hooks are not in effect, so mode 1 is refused and mode 2
(the caller's contract) is what the Python API turns on."""
import os
import subprocess
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _reg_app(stub=False):
    """stub: the counting HIP stubs of reg_app.c in place of the runtime's"""
    out = os.path.join(tempfile.mkdtemp(prefix="mvx_reg_"), "reg_app")
    pkg = os.path.join(ROOT, "mvapich-cce_amd")
    extra = ["-DREG_STUB", "-rdynamic"] if stub else []
    subprocess.check_call(["gcc", "-O2", "-std=gnu99", "-Wall", "-Werror", "-D__HIP_PLATFORM_AMD__"] + extra + [
                           "-I/opt/rocm/include", "-I" + os.path.join(ROOT, "include"),
                           os.path.join(HERE, "reg_app.c"), "-o", out, "-L" + pkg, "-lmvx",
                           "-L/opt/rocm/lib", "-lamdhip64", "-lpthread", "-Wl,-rpath," + pkg, "-Wl,-rpath,/opt/rocm/lib"])
    return out


def test_release_hooks_drop_registrations():
    env = dict(os.environ, MVX_HOST_REGISTER_DRY="1")
    p = subprocess.run([_reg_app(), "dry"], capture_output=True, text=True, timeout=120, env=env)
    assert p.returncode == 0 and "reg_app ok" in p.stdout, p.stdout[-2000:] + p.stderr[-2000:]
    assert '"invalidations": 8' in p.stdout, p.stdout


def test_release_hook_makes_no_hip_call():
    """The real (non-dry) cache against counting stubs of hipHostRegister /
    hipHostUnregister / hipPointerGetAttributes / hipGetLastError defined in
    the program: free() and munmap() of registered memory make no HIP call
    on the releasing thread -- the registration leaves the cache and waits on
    the deferred list (dreg.c:1063-1080) -- and the next libmvx entry
    unregisters it (flush_dereg_mrs_external, dreg.c:678-767)."""
    p = subprocess.run([_reg_app(stub=True), "stub"], capture_output=True, text=True, timeout=120,
                       env={k: v for k, v in os.environ.items() if not k.startswith("MVX_HOST_REGISTER")})
    assert p.returncode == 0 and "reg_app ok" in p.stdout, p.stdout[-2000:] + p.stderr[-2000:]
    assert '"hip_in_release": 0' in p.stdout and '"unregisters": 2' in p.stdout, p.stdout


def test_release_hooks_under_threads():
    """8 threads register and free their own blocks while others churn small
    blocks and unrelated mappings: each registration is dropped once, by its
    own free, and nothing is left (no deadlock: the run is bounded)"""
    env = dict(os.environ, MVX_HOST_REGISTER_DRY="1")
    p = subprocess.run([_reg_app(), "stress"], capture_output=True, text=True, timeout=120, env=env)
    assert p.returncode == 0 and "reg_app ok" in p.stdout, p.stdout[-2000:] + p.stderr[-2000:]
    assert '"registered": 3200' in p.stdout, p.stdout


def test_hooks_inactive_under_ctypes(mvx):
    """dlopen'ed: the process's free is libc's, mode 1 is refused, the API
    falls back to mode 2 and mvx_host_invalidate with nothing registered
    drops nothing"""
    c = mvx.coll()
    assert not mvx.host_hooks_active()
    assert c.mvx_host_register_enable(1, 0) == 15
    assert mvx.host_register_enable(True) == 0
    assert mvx.host_invalidate(4096, 1 << 20) == 0
    assert mvx.host_register_enable(False) == 0
    assert mvx.host_register_stats()["entries"] == 0


def test_embed_library_has_no_hooks():
    """libmvx_embed.so (linked into a host MPI with its own malloc and hooks)
    exports mvx_host_invalidate and defines no free / munmap of its own"""
    out = subprocess.check_output(["nm", "-D", "--defined-only",
                                   os.path.join(ROOT, "mvapich-cce_amd", "libmvx_embed.so")], text=True)
    names = {line.split()[-1] for line in out.splitlines() if line.strip()}
    assert "mvx_host_invalidate" in names
    assert not names & {"free", "realloc", "munmap", "mremap", "madvise", "sbrk"}
    out = subprocess.check_output(["nm", "-D", "--defined-only",
                                   os.path.join(ROOT, "mvapich-cce_amd", "libmvx.so")], text=True)
    names = {line.split()[-1] for line in out.splitlines() if line.strip()}
    assert {"free", "realloc", "munmap", "mremap", "madvise", "sbrk"} <= names
