#!/usr/bin/env python3
"""Benchmark of the MI355X MPI reduction path (BASELINE.json metric).

  N = 1  config 2 (default): device-resident pairwise MPI_SUM on MPI_FLOAT,
         256 MiB vectors -- one step = one local MPI_Op kernel
         (inout = in + inout).
  N > 1  one process per GPU (torchrun), RCCL over xGMI for the exchanges +
         the reference-order combine kernel, one step = one collective:
           c3 (default)  MPI_Allreduce(MPI_SUM, MPI_FLOAT), 256 MiB per rank
           c4            MPI_Reduce_scatter(MPI_BAND, MPI_LONG), 1 GiB per rank
           c5            MPI_Allreduce(MPI_MAXLOC, MPI_FLOAT_INT), 64 Mi pairs

value = bytes of input vectors reduced per second over the whole job
(N x bytes per rank per step / step time), GiB/s.  Inputs are resident in HBM
before the timed region.  Every run checks one untimed step against the
reference computed on the host by the cpu_baseline leg ("parity"): at N = 1
the oracle's MPIR_SUM of the same inputs, at N > 1 the reference schedule
on p host threads (one per rank), which is also the timed cpu_baseline.  The
exchange variant (mvx_comm_set_exchange) is chosen by time alone (--exchange
auto); every variant tried reports its parity.  See DESIGN.md sections 5-6.
"""
import argparse
import hashlib
import importlib
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

MIB = 1 << 20
GIB = 1 << 30
HBM_PEAK_GBS = 8000.0           # MI355X_MICROARCH.md, chip-level parameters
XGMI_LINK_GBS = 153.0           # BASELINE.md section 3 (per link, per direction)
MPI_SUM, MPI_FLOAT, MPI_LONG, MPI_FLOAT_INT, MPI_BAND, MPI_MAXLOC = 102, 10, 8, 17, 105, 111

CONFIGS = {
    # name: (collective, datatype, op, element bytes, default MiB per rank, description)
    "c3": ("allreduce", MPI_FLOAT, MPI_SUM, 4, 256, "MPI_Allreduce MPI_SUM MPI_FLOAT"),
    "c4": ("reduce_scatter", MPI_LONG, MPI_BAND, 8, 1024, "MPI_Reduce_scatter MPI_BAND MPI_LONG"),
    "c5": ("allreduce", MPI_FLOAT_INT, MPI_MAXLOC, 8, 512, "MPI_Allreduce MPI_MAXLOC MPI_FLOAT_INT"),
}
# exchange variants: (mvx_comm_set_exchange mode, slices, mvx_comm_set_graphs).
# The "+g" ones capture each call into a HIP graph once and replay it (one
# hipGraphLaunch per step in place of the host issue of every RCCL group and
# kernel); tried last, after every eager variant has had its turn, and only
# with --graphs: they have run over RCCL's socket transport on one GPU, never
# over xGMI, and a fault there would take the whole line with it (DESIGN.md
# section 6).
EXCH = {"p2p": (0, 0, 0), "pipe": (1, 4, 0), "pipe2": (1, 2, 0), "pipe8": (1, 8, 0), "coll": (2, 0, 0),
        "p2p+g": (0, 0, 1), "pipe+g": (1, 4, 1), "pipe2+g": (1, 2, 1), "pipe8+g": (1, 8, 1), "coll+g": (2, 0, 1)}


def auto_variants(args):
    """--exchange auto: the eager variants, then the graph ones if --graphs"""
    return [k for k, v in EXCH.items() if args.graphs or not v[2]]


def apply_variant(comm, name):
    """set the communicator's exchange variant and graph mode: 0 or an MPI code"""
    mode, slices, graphs = EXCH[name]
    return comm.set_exchange(mode, slices) or comm.set_graphs(graphs)


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one per GPU).  Under torchrun it must equal WORLD_SIZE; without a launcher "
                         "(no WORLD_SIZE) N > 1 starts N worker processes itself (launch())")
    ap.add_argument("--launch-grace", type=float, default=30.0,
                    help="self-launched N > 1: seconds the other workers get after one fails before they "
                         "are killed")
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default=None, choices=["c2", "c3", "c4", "c5"],
                    help="c2 at N = 1, c3 at N > 1 by default")
    ap.add_argument("--mib", type=int, default=0, help="vector MiB per rank (0 = the config's)")
    ap.add_argument("--no-cpu-baseline", action="store_true",
                    help="skip the CPU leg (and with it the parity check against it)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--prewarm-ms", type=float, default=0.0,
                    help="N = 1: untimed back-to-back steps for this long before the W warmup steps "
                         "(0 = none); reported in the line")
    ap.add_argument("--pmc", default=os.path.join(ROOT, "profiles", "r06", "pmc_c2.json"),
                    help="committed rocprofv3 PMC summary for the traffic field")
    ap.add_argument("--block-cap", type=int, default=0)
    ap.add_argument("--nt-min-log2", type=int, default=0, help="-1 disables non-temporal loads/stores")
    ap.add_argument("--sets", type=int, default=4,
                    help="input sets used round-robin (4 x 512 MiB keeps every step out of the 256 MiB "
                         "Infinity Cache: the number is HBM-bound, not cache-bound)")
    ap.add_argument("--exchange", default="auto",
                    help="auto: every eager variant of EXCH (and the graph ones with --graphs), the "
                         "fastest clean one makes the line; or a comma list of them")
    ap.add_argument("--graphs", action="store_true",
                    help="auto also tries the HIP-graph variants (the '+g' ones of EXCH)")
    ap.add_argument("--tune-steps", type=int, default=5)
    ap.add_argument("--extra-configs", default="auto",
                    help="N > 1: more BASELINE configs measured after the line, on the same communicator "
                         "(auto: c4 at N = 4, c5 at N = 8; none; or a comma list)")
    ap.add_argument("--gloo-timeout", type=float, default=600.0,
                    help="N > 1: seconds any gloo operation may wait for a peer")
    ap.add_argument("--variant-timeout", type=float, default=60.0,
                    help="N > 1: seconds one checked step of an exchange variant may take before the "
                         "variant counts as hung (its communicator is aborted and rebuilt)")
    ap.add_argument("--no-native", action="store_true",
                    help="N > 1: skip the RCCL-native reduction timed after the line (SURVEY.md 8(e) ablation)")
    ap.add_argument("--host-e2e", action="store_true",
                    help="N = 1: also time the op on host buffers (PCIe-inclusive) after the timed region; "
                         "off by default: it launches the measured kernel template on PCIe-bound operands, "
                         "which would skew a kernel-trace average of the same command")
    ap.add_argument("--no-kernels", action="store_true",
                    help="N = 1: skip the C3 / C4 / C5 combine-kernel rates after the timed region")
    ap.add_argument("--transport", default="rccl", choices=["rccl", "host", "rccl-net"],
                    help="host: ranks may share a GPU, bytes move through gloo; rccl-net: ranks may "
                         "share a GPU, bytes move through RCCL's own socket transport (each rank "
                         "names itself a separate host).  Both test the multi-GPU leg on a 1-GPU "
                         "box; neither is a performance configuration")
    args = ap.parse_args(argv)
    if args.exchange != "auto":
        bad = [x for x in args.exchange.split(",") if x not in EXCH]
        if bad:
            ap.error("--exchange: unknown variant(s) %s (known: %s)" % (",".join(bad), ",".join(EXCH)))
    return args


# ------------------------------------------------------------ wall clock --

class Stages:
    """Wall seconds per stage of this process, contiguous from the process's
    creation (psutil): the stages partition the wall clock up to the last
    mark, interpreter start-up and imports included, so a run that outlasts
    a timeout says where the time went.  Rank 0 also prints each mark to
    stderr (a long multi-GPU run keeps saying it is alive)."""

    def __init__(self, verbose=False):
        try:
            import psutil
            self.t0 = psutil.Process().create_time()
        except Exception:            # no psutil: from here on
            self.t0 = time.time()
        self.last = self.t0
        self.s = {}
        self.verbose = verbose

    def mark(self, name):
        now = time.time()
        self.s[name] = round(self.s.get(name, 0.0) + now - self.last, 3)
        self.last = now
        if self.verbose:
            sys.stderr.write("bench: %-28s %8.2f s (wall %.1f s)\n" % (name, self.s[name], now - self.t0))
            sys.stderr.flush()

    def report(self):
        now = time.time()
        return {"stage_s": dict(self.s), "wall_s": round(now - self.t0, 3),
                "unaccounted_s": round(now - self.last, 3)}


ENV_PREFIXES = ("NCCL_", "RCCL_", "MVX_", "HSA_", "HIP_VISIBLE", "ROCR_VISIBLE", "CUDA_VISIBLE",
                "GPU_MAX_HW_QUEUES", "TORCH_NCCL")


def env_echo(env=None):
    """The RCCL / HIP / MVX knobs this run saw (DESIGN.md section 6 names
    the ones a node run needs: none beyond the image's)."""
    env = os.environ if env is None else env
    return {k: env[k] for k in sorted(env) if k.startswith(ENV_PREFIXES)}


# --------------------------------------------------------------- launcher --

def decide_launch(gpus, env):
    """What main() does with --gpus under this environment:
    ("single", 1) -- N = 1 in this process; ("self", N) -- no launcher set
    WORLD_SIZE and N > 1: start N workers (launch()); ("worker", W) -- a
    launcher (torchrun, or launch() itself) set WORLD_SIZE = W and --gpus is
    absent or equal; ("mismatch", msg) -- --gpus names another world size."""
    ws = env.get("WORLD_SIZE")
    if ws is None:
        n = 1 if gpus is None else gpus
        if n < 1:
            return "mismatch", "--gpus %d: need at least 1" % n
        return ("self", n) if n > 1 else ("single", 1)
    w = int(ws)
    if gpus is not None and gpus != w:
        return "mismatch", "--gpus %d but the launcher started WORLD_SIZE=%d ranks" % (gpus, w)
    return ("worker", w) if w > 1 else ("single", 1)


def worker_env(base, rank, n, port):
    """The environment of self-launched worker `rank` of n (torchrun's names)."""
    env = dict(base)
    env.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
               GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), MVX_BENCH_LAUNCHER="self")
    return env


class _StdoutToStderr:
    """fd 1 points at stderr while native code that reports on stdout runs
    (gloo prints each rank's connection count when the process group
    forms): the driver reads rank 0's one JSON line from stdout, and under
    torchrun every rank's stdout is merged into it."""

    def __enter__(self):
        sys.stdout.flush()
        self.saved = os.dup(1)
        os.dup2(2, 1)
        return self

    def __exit__(self, *exc):
        import ctypes
        sys.stdout.flush()
        ctypes.CDLL(None).fflush(None)       # C stdio's buffer, before fd 1 goes back
        os.dup2(self.saved, 1)
        os.close(self.saved)
        return False


def _rc_of(rc):
    return 128 - rc if rc < 0 else rc      # a signal -> 128 + signo, as a shell reports it


KFD_NODES = "/sys/class/kfd/kfd/topology/nodes"


def visible_gpus(env=None, nodes=None):
    """GPUs this process may use, counted without HIP or torch: the KFD
    topology's nodes with SIMDs (a CPU node has simd_count 0), narrowed by
    ROCR_VISIBLE_DEVICES and then HIP_VISIBLE_DEVICES / CUDA_VISIBLE_DEVICES
    (indices, or ROCr's GPU-<unique_id> names).  None when the topology
    cannot be read (then nothing is checked before the workers start)."""
    env = os.environ if env is None else env
    nodes = nodes or env.get("MVX_KFD_NODES", KFD_NODES)
    try:
        names = sorted(os.listdir(nodes), key=lambda x: int(x) if x.isdigit() else 1 << 30)
    except OSError:
        return None
    gpus = []
    for name in names:
        try:
            with open(os.path.join(nodes, name, "properties")) as f:
                props = dict(line.split(None, 1) for line in f if len(line.split(None, 1)) == 2)
        except OSError:
            continue
        if int(props.get("simd_count", "0")) > 0:
            gpus.append("GPU-%016x" % int(props.get("unique_id", "0")))

    def narrow(ids, var):
        v = env.get(var)
        if v is None:
            return ids
        out = []
        for e in (x.strip() for x in v.split(",")):
            if e.isdigit() and int(e) < len(ids):
                out.append(ids[int(e)])
            elif e.upper().startswith("GPU-") and e.lower() in (i.lower() for i in ids):
                out.append(e)
            else:
                break                      # the runtimes stop at the first invalid entry
        return out

    gpus = narrow(gpus, "ROCR_VISIBLE_DEVICES")
    gpus = narrow(gpus, "HIP_VISIBLE_DEVICES" if "HIP_VISIBLE_DEVICES" in env else "CUDA_VISIBLE_DEVICES")
    return len(gpus)


def launch(args, n, argv):
    """--gpus N > 1 with no WORLD_SIZE: one worker process per GPU, started
    before this process touches the GPU (it never does), never by exec.
    Rank 0's stdout is read here; its JSON line gets a "launch" entry (this
    process's wall clock around the whole job, the workers' exit codes) and
    is printed.  If a worker fails the others get --launch-grace seconds,
    then are killed.  Exit code: the workers' worst."""
    import signal
    import socket
    import subprocess
    import threading
    if args.transport == "rccl":
        have = visible_gpus()     # no HIP call (and no torch) in this process
        if have is not None and have < n:
            sys.stderr.write("bench: --gpus %d over RCCL needs %d GPUs, this box has %d (RCCL refuses two "
                             "ranks on one GPU; --transport rccl-net or host shares one)\n" % (n, n, have))
            return 2
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    t0 = time.time()
    cmd = [sys.executable, os.path.abspath(__file__)] + list(argv)

    def die_with_parent():
        try:
            import ctypes
            ctypes.CDLL("libc.so.6").prctl(1, signal.SIGKILL)   # PR_SET_PDEATHSIG
        except Exception:
            pass

    procs = [subprocess.Popen(cmd, env=worker_env(os.environ, r, n, port),
                              stdout=subprocess.PIPE if r == 0 else None, preexec_fn=die_with_parent)
             for r in range(n)]
    out0 = []
    reader = threading.Thread(target=lambda: out0.extend(procs[0].stdout.read().decode().splitlines()),
                              daemon=True)
    reader.start()

    def stop(signum, frame):
        for p in procs:
            if p.poll() is None:
                p.kill()
        sys.exit(128 + signum)

    old = {s: signal.signal(s, stop) for s in (signal.SIGTERM, signal.SIGINT)}
    failed_at = None
    try:
        while any(p.poll() is None for p in procs):
            if failed_at is None and any(p.poll() not in (None, 0) for p in procs):
                failed_at = time.time()
            if failed_at is not None and time.time() - failed_at > args.launch_grace:
                for p in procs:
                    if p.poll() is None:
                        p.kill()
            time.sleep(0.1)
    finally:
        for s, h in old.items():
            signal.signal(s, h)
    reader.join(timeout=10)
    rcs = [p.returncode for p in procs]
    wall = time.time() - t0
    for line in out0:                  # stdout carries the JSON line only; the rest goes to stderr
        if line.startswith("{"):
            try:
                d = json.loads(line)
            except ValueError:
                print(line, file=sys.stderr, flush=True)
                continue
            d["launch"] = {"mode": "self (bench.py --gpus %d without a launcher: %d worker processes)" % (n, n),
                           "workers": n, "wall_s": round(wall, 3), "worker_rcs": rcs}
            print(json.dumps(d), flush=True)
        else:
            print(line, file=sys.stderr, flush=True)
    return max(_rc_of(rc) for rc in rcs)


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _digest(u8):
    try:
        import xxhash
        return xxhash.xxh3_128_hexdigest(memoryview(u8))
    except ImportError:
        return hashlib.blake2b(memoryview(u8), digest_size=16).hexdigest()


# ---------------------------------------------------------------- inputs ---

def synth_f32(n, seed, device):
    """Mixed-sign f32 with an exponent spread, made on the GPU."""
    import torch
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    m = torch.randint(-1000000, 1000001, (n,), generator=g, device=device, dtype=torch.int32)
    s = torch.randint(1, 1001, (n,), generator=g, device=device, dtype=torch.int32)
    return (m.to(torch.float32) * 1e-3 * s.to(torch.float32)).contiguous()


def synth(cfg, n, rank, device):
    """Rank `rank`'s send vector of config cfg as a uint8 device tensor: c3
    mixed-sign f32; c4 int64 words with P(bit = 1) = 15/16 (OR of four random
    words, so BAND over the ranks is not all zero); c5 {v = u % 1024 (many
    ties), loc = rank * n + i} FLOAT_INT pairs."""
    import torch
    seed = 0x9E3779B9 ^ (rank * 1000003 + 1)
    if cfg == "c3":
        return synth_f32(n, seed, device).view(torch.uint8)
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    if cfg == "c4":
        w = torch.zeros(n, dtype=torch.int64, device=device)
        for _ in range(4):
            w |= torch.randint(-(1 << 63), (1 << 63) - 1, (n,), generator=g, device=device, dtype=torch.int64)
        return w.view(torch.uint8)
    pair = torch.empty((n, 2), dtype=torch.int32, device=device)
    pair[:, 0] = torch.randint(0, 1024, (n,), generator=g, device=device, dtype=torch.int32).to(
        torch.float32).view(torch.int32)
    pair[:, 1] = torch.arange(n, dtype=torch.int32, device=device) + rank * n
    return pair.view(-1).view(torch.uint8)


# ------------------------------------------------------------------- N = 1 --

def cpu_baseline_op(n_bytes, seconds):
    """Oracle MPIR_SUM (oracle/cpu_ops.c, the reference's loop) on 1 host core."""
    import numpy as np
    from oracle import oracle as O
    n = n_bytes // 4
    a = np.empty(n, np.float32)
    b = np.empty(n, np.float32)
    O.fill(a, n, 0, 0)
    O.fill(b, n, 0, 1)
    O.op(MPI_SUM, MPI_FLOAT, a.view(np.uint8), b.view(np.uint8), n)  # warm pages
    reps, t0 = 0, time.perf_counter()
    while True:
        O.op(MPI_SUM, MPI_FLOAT, a.view(np.uint8), b.view(np.uint8), n)
        reps += 1
        dt = time.perf_counter() - t0
        if dt >= seconds:
            break
    return {"value": round(n_bytes * reps / dt / GIB, 3), "unit": "GiB/s", "cores": 1, "kind": "port",
            "sample": "oracle MPIR_SUM float32, %d MiB vectors x %d reps (%.1f s) on 1 host core"
                      % (n_bytes // MIB, reps, dt),
            "cpu": _cpu_model()}


def parity_op(mvx, x_in, x_io, n, stream):
    """One untimed MPI_SUM step on copies, against the oracle's MPIR_SUM of
    the same inputs (global_ops.c:364-369) on the host."""
    import numpy as np
    import torch
    from oracle import oracle as O
    a, b = x_in.clone(), x_io.clone()
    rc = mvx.op_apply(MPI_SUM, MPI_FLOAT, a, b, n, stream)
    torch.cuda.synchronize()
    ref = x_io.cpu().numpy().copy()
    O.op(MPI_SUM, MPI_FLOAT, x_in.cpu().numpy().view(np.uint8), ref.view(np.uint8), n)
    ok = rc == 0 and np.array_equal(b.cpu().numpy().view(np.uint32), ref.view(np.uint32))
    return "bit-exact vs oracle MPIR_SUM (1 step, %d elements)" % n if ok else "MISMATCH (rc=%d)" % rc


def load_traffic(path, kernel_tag, kernel_symbol, nbytes):
    """Per-launch HBM bytes from a committed rocprofv3 PMC summary -- only if
    it was collected for exactly the kernel template this run launched, at
    this size (FETCH_SIZE doubled on gfx950, tools/pmc_summary.py)."""
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None, "no PMC summary at %s" % os.path.relpath(path, ROOT)
    if d.get("kernel_tag") != kernel_tag or d.get("vector_bytes") != nbytes:
        return None, "PMC summary is for %s at %s bytes" % (d.get("kernel_tag"), d.get("vector_bytes"))
    if d.get("kernel_match") != kernel_symbol:
        return None, "PMC summary template %r != launched %r" % (d.get("kernel_match"), kernel_symbol)
    return d.get("hbm_bytes_per_launch"), os.path.relpath(path, ROOT)


def prewarm(args, step):
    """Untimed, before the W warmup steps: back-to-back steps for
    --prewarm-ms of wall time, so the timed steps do not start on a GPU
    still raising its clocks (a 5-step warmup is < 1 ms of work).  Reported
    in the line as "prewarm"."""
    import torch
    if args.prewarm_ms <= 0:
        return None
    n, t0 = 0, time.perf_counter()
    while True:
        for _ in range(8):
            step()
        n += 8
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        if dt * 1e3 >= args.prewarm_ms:
            break
    return {"steps": n, "ms": round(dt * 1e3, 1),
            "note": "untimed steps before the W warmup steps (clock ramp-up); not in value"}


def run_single(args, mvx, dev, clock):
    import torch
    nbytes = (args.mib or 256) * MIB
    n = nbytes // 4
    stream = torch.cuda.current_stream()
    x_in = [synth_f32(n, 0x9E3779B9 ^ (2 * s * 1000003 + 1), dev) for s in range(args.sets)]
    x_io = [synth_f32(n, 0x9E3779B9 ^ ((2 * s + 1) * 1000003 + 1), dev) for s in range(args.sets)]
    # the parity check reads set 0 before any step has touched it
    keep = None if args.no_cpu_baseline else (x_in[0].clone(), x_io[0].clone())
    it = [0]

    def step():
        s = it[0] % args.sets
        it[0] += 1
        rc = mvx.op_apply(MPI_SUM, MPI_FLOAT, x_in[s], x_io[s], n, stream)
        if rc:
            raise RuntimeError("mvx_op_apply rc=%d" % rc)

    # from input synthesis to the last timed step the GPU never idles: the
    # host-side parity check and the CPU leg run after the timed region
    torch.cuda.synchronize()
    clock.mark("inputs")
    warm = prewarm(args, step)
    times = timed(args, step, stream, 1)
    clock.mark("timed steps")
    # cpu_baseline leg, part 1: the reference op on the same inputs (checker)
    parity = None
    if keep is not None:
        parity = parity_op(mvx, keep[0], keep[1], n, stream)
        del keep
    kernel = mvx.last_kernel()
    symbol = mvx.last_kernel_symbol()
    kern_s = times["dev_ms"] / 1e3 / args.steps           # HIP events on the launch stream
    alg_bytes = 3 * nbytes                                  # read in, read inout, write inout
    achieved = alg_bytes / kern_s / 1e9
    traffic, tsrc = load_traffic(args.pmc, kernel, symbol, nbytes)
    roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_source": tsrc,
            "kernel": kernel, "kernel_symbol": symbol, "kernel_us": round(kern_s * 1e6, 2),
            # per-launch distribution from the event-per-step pass (timed())
            "kernel_us_evented_median": round(times["median_ms"] * 1e3, 2),
            "kernel_us_evented_min": round(times["min_ms"] * 1e3, 2),
            "alg_bytes_per_launch": alg_bytes}
    out = result(args, 1, nbytes, times, "f32",
                 {"workload": "config2: device-resident pairwise MPI_SUM float32 %d MiB (local MPI_Op kernel), "
                              "%d input sets round-robin" % (nbytes // MIB, args.sets),
                  "vector_bytes_per_rank": nbytes, "op": "MPI_SUM", "datatype": "MPI_FLOAT",
                  "parallelism": "single GPU"}, roof)
    out["parity"] = parity
    out["prewarm"] = warm
    if not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline_op(nbytes, args.cpu_seconds)
    if not args.no_kernels:
        out["combine_kernels"] = combine_kernels(mvx)
        roof["mix_ceiling"] = mix_ceiling(x_in, x_io, nbytes, achieved, stream)
    if args.host_e2e:
        out["host_end_to_end"] = host_end_to_end(mvx, nbytes)
    clock.mark("parity, cpu baseline, combine kernels, ceilings")
    out["env"] = env_echo()
    out["wall"] = clock.report()
    print(json.dumps(out), flush=True)


def combine_kernels(mvx):
    """After the timed region: the combine kernel each rank of the
    multi-GPU configs launches, at that config's shapes, alone on this GPU
    (tools/bench_kernels.py: rotating buffer sets, HIP events on the launch
    stream) -- C3 8-leaf SUM f32 tree over 32 MiB leaves, C4 4-leaf BAND int64
    chain over 256 MiB, C5 8-leaf MAXLOC FLOAT_INT tree over 64 MiB."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import bench_kernels as BK
    rows = [BK.run(mvx, "C3", MPI_SUM, MPI_FLOAT, 8, 0, 32 * MIB, 4, quiet=True),
            BK.run(mvx, "C4", MPI_BAND, MPI_LONG, 4, 1, 256 * MIB, 2, quiet=True),
            BK.run(mvx, "C5", MPI_MAXLOC, MPI_FLOAT_INT, 8, 0, 64 * MIB, 2, quiet=True)]
    return [{k: r[k] for k in ("config", "kernel", "k", "alg_bytes_per_launch", "kernel_us", "hbm_frac")}
            for r in rows]


def mix_ceiling(x_in, x_io, nbytes, achieved_gbs, stream, reps=20):
    """After the timed region: what this GPU's HBM reaches for the C2
    kernel's own traffic on the same rotating buffers -- both vectors read
    alone, one written alone, a copy (tools/ceiling.hip, the fastest form of
    each stream in tools/tune_sum3.hip).  Two ceilings for the 2-read /
    1-write kernel: `additive` -- the reads' time plus the write's, as if
    reads and writes never shared the bus (a bound no mixed stream was seen
    to reach: the copy kernel makes 0.91 of it); `mixed_line` -- the rate on
    the line from read-only (write share 0) to copy (1/2) at the kernel's
    write share 1/3.  8 TB/s stays the line's `peak`."""
    import ctypes
    path = os.path.join(ROOT, "tools", "libmvx_ceiling.so")
    try:
        lib = ctypes.CDLL(path)
    except OSError as e:
        return {"error": "%s: %s" % (os.path.relpath(path, ROOT), e)}
    fn = lib.mvx_ceiling_run
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_void_p), ctypes.c_int,
                   ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p, ctypes.POINTER(ctypes.c_float)]
    sets = len(x_in)
    a = (ctypes.c_void_p * sets)(*[t.data_ptr() for t in x_in])
    b = (ctypes.c_void_p * sets)(*[t.data_ptr() for t in x_io])
    us = {}
    for mode, name in ((0, "read2"), (1, "write1"), (2, "copy")):
        t = ctypes.c_float()
        if fn(mode, a, b, sets, nbytes, reps, ctypes.c_void_p(stream.cuda_stream), ctypes.byref(t)):
            return {"error": "mvx_ceiling_run(%d) failed" % mode}
        us[name] = float(t.value)
    return ceiling_summary(nbytes, us, achieved_gbs)


def ceiling_summary(nbytes, us, achieved_gbs):
    """The two ceilings of a 2-read / 1-write stream of `nbytes` vectors from
    the launch times (us) of reading both vectors ("read2"), writing one
    ("write1") and copying one ("copy"); see mix_ceiling."""
    read_gbs = 2 * nbytes / (us["read2"] * 1e-6) / 1e9
    copy_gbs = 2 * nbytes / (us["copy"] * 1e-6) / 1e9
    additive = 3 * nbytes / ((us["read2"] + us["write1"]) * 1e-6) / 1e9
    line = read_gbs + (copy_gbs - read_gbs) * (1 / 3) / (1 / 2)   # write share 1/3 on the 0 .. 1/2 line
    return {"read_GBs": round(read_gbs, 1), "write_GBs": round(nbytes / (us["write1"] * 1e-6) / 1e9, 1),
            "copy_GBs": round(copy_gbs, 1), "us": {k: round(v, 2) for k, v in us.items()},
            "additive_GBs": round(additive, 1), "frac_of_additive": round(achieved_gbs / additive, 4),
            "mixed_line_GBs": round(line, 1), "frac_of_mixed_line": round(achieved_gbs / line, 4),
            "note": "measured ceilings of the kernel's own 2-read/1-write mix (tools/ceiling.hip); not the peak"}


def host_end_to_end(mvx, nbytes, budget=0.25):
    """After the timed region, never `value`: the same op when the MPI user
    buffers live in host memory, as the reference's do (north_star: the
    PCIe-inclusive rate).  MPIR_SUM(invec, inoutvec) on the
    product's host path -- page-locked operands DMA'd directly, pageable ones
    through the bounce pipeline -- 2 vectors H2D and 1 D2H per call.  Median
    call time over `budget` seconds after one checked call (against numpy:
    float32 sums of small integers are exact)."""
    import numpy as np
    import torch
    n = nbytes // 4
    rng = np.random.default_rng(7)
    a = rng.integers(-8, 8, n).astype(np.float32)
    b = rng.integers(-8, 8, n).astype(np.float32)
    want = a + b
    rows = []
    for where in ("pinned", "pageable"):
        if where == "pinned":
            x, y = torch.from_numpy(a).pin_memory(), torch.from_numpy(b).pin_memory()
        else:
            x, y = a.copy(), b.copy()
        mvx.MPIR_call("MPIR_SUM", x, y, n, MPI_FLOAT)
        got = y.numpy() if torch.is_tensor(y) else y
        ok = mvx.op_errno() == 0 and bool(np.array_equal(got, want))
        ts, t_end = [], time.perf_counter() + budget
        while len(ts) < 3 or time.perf_counter() < t_end:
            t0 = time.perf_counter()
            mvx.MPIR_call("MPIR_SUM", x, y, n, MPI_FLOAT)
            ts.append(time.perf_counter() - t0)
        ts.sort()
        t = ts[len(ts) // 2]
        rows.append({"buffers": where, "ms": round(t * 1e3, 3), "calls": len(ts),
                     "GiB_per_s_per_vector": round(nbytes / t / GIB, 2),
                     "pcie_GBps": round(3 * nbytes / t / 1e9, 1), "checked": ok})
        del x, y
    return {"op": "MPIR_SUM float32 %d MiB, host operands (2 H2D + 1 D2H per call)" % (nbytes // MIB),
            "rows": rows}


# ------------------------------------------------------------------ common --

class StepFailure(Exception):
    """A block of steps returned an error (worst = 1) or did not complete in
    time (worst = 2) on some rank; every rank raises it alike."""

    def __init__(self, worst, limit):
        super().__init__(worst)
        self.worst, self.limit = worst, limit

    def text(self):
        return ("an error return on some rank" if self.worst == 1 else
                "a step did not complete within %.0f s" % self.limit)


def timed(args, step, stream, world, agree=None, limit=None):
    """W untimed steps, then K steps between barrier + synchronize, with one
    HIP event pair on the launch stream around them (the mean: nothing else
    is enqueued between the steps).  Then, untimed, K more steps with an
    event after each for the median / min (an event between two kernels adds
    a few microseconds of its own, so these are not used for the mean).

    N > 1 (agree given): every block of steps ends in a bounded wait for the
    launch stream (busy polling, `limit` seconds) and a status agreement over
    gloo -- the barrier -- so an error return or a step that never completes
    on any rank raises StepFailure on every rank instead of blocking them in
    torch.cuda.synchronize or killing one rank."""
    import torch
    import torch.distributed as dist

    def settle(block):
        if agree is None:
            block()
            torch.cuda.synchronize()
            if world > 1:
                dist.barrier()
            return
        st = 0
        try:
            block()
        except RuntimeError:
            st = 1
        if st == 0 and not _wait_stream(stream, limit, spin=True):
            st = 2
        worst = agree(st)
        if worst:
            raise StepFailure(worst, limit)
        torch.cuda.synchronize()

    def run(k, evs=None):
        def block():
            for i in range(k):
                step()
                if evs is not None:
                    evs[i + 1].record(stream)
        return block

    settle(run(args.warmup))
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    wall = [0.0]

    def timed_block():
        t0 = time.perf_counter()
        e0.record(stream)
        run(args.steps)()
        e1.record(stream)
        if agree is None:
            torch.cuda.synchronize()
        elif not _wait_stream(stream, limit, spin=True):
            raise _Hung()
        wall[0] = time.perf_counter() - t0      # this rank's K steps; MAX over ranks below

    if agree is None:
        timed_block()
        settle(lambda: None)
    else:
        st = 0
        try:
            timed_block()
        except RuntimeError:
            st = 1
        except _Hung:
            st = 2
        worst = agree(st)
        if worst:
            raise StepFailure(worst, limit)
    wall = wall[0]
    dev_ms = e0.elapsed_time(e1)
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
    evs[0].record(stream)
    settle(run(args.steps, evs))
    per = [evs[i].elapsed_time(evs[i + 1]) for i in range(args.steps)]
    t_local = max(wall, dev_ms / 1e3)
    if world > 1:
        t = torch.tensor([t_local], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        t_local = float(t.item())
    return {"t_job": t_local, "dev_ms": dev_ms, "mean_ms": dev_ms / args.steps,
            "median_ms": statistics.median(per), "min_ms": min(per)}


def result(args, world, nbytes, times, dtype, config, roof):
    ms_per_step = times["t_job"] * 1e3 / args.steps
    return {
        "metric": "GiB/s device-resident Allreduce(SUM,float32) at 1/2/4/8 GPUs; % HBM/xGMI peak",
        "value": round(world * nbytes * args.steps / times["t_job"] / GIB, 2), "unit": "GiB/s",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 5),
        "step_ms": {"mean": round(times["mean_ms"], 5),
                    # a second, untimed pass of K steps with an event after each
                    # (each event adds a few microseconds between steps)
                    "evented_median": round(times["median_ms"], 5), "evented_min": round(times["min_ms"], 5)},
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": dtype,
        "data": "synthetic (generated on device, SURVEY.md 8(d) distributions)",
        "config": config, "roofline": roof,
    }


# ------------------------------------------------------------------- N > 1 --

def reference_run(cfg, world, n, dev, want_time):
    """Rank 0: every rank's inputs (same generator), the reference schedule
    on `world` host threads (oracle/cpu_coll.c, one thread per rank, as the
    reference's p processes) -> per-rank result digests and seconds per
    collective."""
    import numpy as np
    import torch
    from oracle import oracle as O
    coll, dtype, op, E, _, _ = CONFIGS[cfg]
    sends = []
    for r in range(world):
        sends.append(synth(cfg, n, r, dev).cpu().numpy())
        torch.cuda.empty_cache()
    cnts = [n // world] * world if coll == "reduce_scatter" else None
    nrecv = (n // world) if cnts else n
    recvs = [np.zeros(nrecv * E, np.uint8) for _ in range(world)]
    ocoll = 3 if cnts else 1
    # scratch per rank thread: the whole vector (Allreduce), the rank's block
    # (pairwise Reduce_scatter), or 2 x the vector (recursive halving)
    tmp_elems = n if not cnts else (nrecv if O.algorithm(ocoll, world, n, dtype) == O.ALG_RS_PAIRWISE else 2 * n)
    tmps = [np.zeros(tmp_elems * E, np.uint8) for _ in range(world)]
    secs = O.threads_coll(ocoll, sends, recvs, tmps, n, dtype, op, 0, cnts, 1)
    digests = [_digest(r) for r in recvs]
    reps = 0
    if want_time:
        reps = max(1, min(20, int(10.0 / max(secs, 1e-3))))
        secs = O.threads_coll(ocoll, sends, recvs, tmps, n, dtype, op, 0, cnts, reps)
    del sends, tmps
    return digests, secs, reps


def plan_bytes(mvx, coll, world, rank, n, cnts, dtype, op):
    """Bytes this rank sends and receives in phase A (exchange) and phase C
    (distribution) of its plan (mvx_plan_build), for the per-link reading of
    the phase rates: over direct xGMI links each peer's share travels on its
    own link."""
    kind = mvx.COLL_ALLREDUCE if coll == "allreduce" else mvx.COLL_REDUCE_SCATTER
    P = mvx.plan(kind, world, rank, n, dtype, op, recvcnts=cnts if coll == "reduce_scatter" else None)
    E = P.esize
    out = {}
    for ph, snd, rcv in (("A", P.a_send, P.a_recv), ("C", P.b_send, P.b_recv)):
        s_peer = [snd[q].cnt * E for q in range(world) if q != rank]
        r_peer = [rcv[q].cnt * E for q in range(world) if q != rank]
        out[ph] = {"sent": sum(s_peer), "received": sum(r_peer),
                   "max_per_peer": max(s_peer + r_peer) if world > 1 else 0,
                   "peers": sum(1 for v in r_peer if v)}
    return out


def phase_breakdown(comm, step, coll, world, nbytes, pb, stream, agree, limit, reps=3):
    """Untimed, after the timed region: `reps` more steps with HIP events
    around phase A (exchange), B (combine) and C (distribution) on the launch
    stream (mvx_comm_set_phase_timing); the median of each, MAX over ranks,
    with the rate each phase reached: A / C as the bytes each rank sends and
    receives per ms (and per link: the largest single peer's share over the
    phase time, against XGMI_LINK_GBS), B as the combine's HBM bytes.  Each
    step is waited for with a bound (StepFailure, as in timed())."""
    import torch
    import torch.distributed as dist
    comm.set_phase_timing(True)
    got = []
    for _ in range(reps):
        st = 0
        try:
            step()
        except RuntimeError:
            st = 1
        if st == 0 and not _wait_stream(stream, limit):
            st = 2
        worst = agree(st)
        if worst:
            comm.set_phase_timing(False)
            raise StepFailure(worst, limit)
        got.append(comm.phase_times())
    comm.set_phase_timing(False)
    out = {}
    for key in ("A", "B", "C", "total"):
        vals = [g[key] for g in got if g[key] is not None]
        v = statistics.median(vals) if vals else -1.0
        t = torch.tensor([v], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        out[key + "_ms"] = None if t.item() < 0 else round(float(t.item()), 4)
    p = world
    for ph in ("A", "C"):
        b = pb[ph]
        out[ph + "_bytes"] = {"sent": b["sent"], "received": b["received"], "peers": b["peers"],
                              "max_per_peer": b["max_per_peer"]}
        ms = out[ph + "_ms"]
        if ms and (b["sent"] or b["received"]):
            sec = ms * 1e-3
            out[ph + "_GBs_per_rank"] = {"sent": round(b["sent"] / sec / 1e9, 1),
                                         "received": round(b["received"] / sec / 1e9, 1),
                                         "per_link": round(b["max_per_peer"] / sec / 1e9, 1),
                                         "link_frac": round(b["max_per_peer"] / sec / 1e9 / XGMI_LINK_GBS, 4)}
    if out["B_ms"]:
        out["B_hbm_GBs"] = round((p + 1) * nbytes / p / (out["B_ms"] * 1e-3) / 1e9, 1)
    out["note"] = ("one untimed step per sample with events between the phases; "
                   "the pipelined variant overlaps them (total only)")
    return out


def _fail_injected(name, rank):
    """MVX_BENCH_FAIL=variant@rank: that rank's steps under that exchange
    variant report an error after running (a test of the variant choice)"""
    spec = os.environ.get("MVX_BENCH_FAIL", "")
    return any(x == "%s@%d" % (name, rank) for x in spec.split(",") if x)


def _hang_injected(name, rank):
    """MVX_BENCH_HANG=variant@rank: that rank never issues the checked step
    of that exchange variant, so its peers' transfers wait forever (a test
    of the hang path: variant timeout, communicator abort, a fresh one)"""
    spec = os.environ.get("MVX_BENCH_HANG", "")
    return any(x == "%s@%d" % (name, rank) for x in spec.split(",") if x)


class _Hung(Exception):
    pass


def _wait_stream(stream, seconds, spin=False):
    """True once the stream drained, False after `seconds` (a hung transfer).
    spin: poll without sleeping (inside a timed region, where a 0.5 ms nap
    would be read as step time)."""
    t0 = time.perf_counter()
    nap = 0.0 if spin else 0.0005
    while not stream.query():
        if time.perf_counter() - t0 > seconds:
            return False
        time.sleep(nap)
    return True


EXCH_NAMES = {-1: "none", 0: "p2p", 1: "pipe", 2: "coll"}
GRAPH_STATES = {0: "eager", 1: "replayed", 2: "captured"}


def choose_variant(names, tried):
    """The fastest variant that ran clean (timed) and whose parity did not
    fail, in `names` order on ties; None when there is none.  A MISMATCH
    stays on record in exchange_tuning but is never the one timed."""
    ok = [k for k in names if tried.get(k, {}).get("ms_per_step") is not None
          and tried[k].get("parity") is not False]
    return min(ok, key=lambda k: tried[k]["ms_per_step"]) if ok else None


# BASELINE's multi-GPU configs by GPU count: at N = 4 and N = 8 the line
# also carries the config quoted at that count (after the timed region)
EXTRA_AT = {4: ["c4"], 8: ["c5"]}


def step_limit(args, est_s):
    """Seconds a block of steps may take before it counts as hung: the
    variant timeout, or 10 x the block at the checked step's pace."""
    return max(args.variant_timeout, 10.0 * max(args.steps, args.warmup, 1) * est_s)


def checked_step(step, stream, limit):
    """One step and a bounded wait: (status 0 ok / 1 error / 2 hung, seconds)"""
    t0 = time.perf_counter()
    try:
        step()
    except RuntimeError:
        return 1, time.perf_counter() - t0
    ok = _wait_stream(stream, limit)
    return (0 if ok else 2), time.perf_counter() - t0


def run_extra(args, mvx, dev, world, rank, comm, exch_name, cfg, agree, stream):
    """After the line is measured: one more BASELINE config on the same
    communicator -- its reference digests (rank 0, the reference schedule on
    p host threads, untimed), one checked step (a hang or an error is
    recorded, not fatal), then W + K timed steps.  Returns (summary, worst
    status: 0 ok, 1 error, 2 hung)."""
    import torch
    import torch.distributed as dist
    coll, dtype, op, E, mib, desc = CONFIGS[cfg]
    nbytes = (args.mib or mib) * MIB
    n = nbytes // E
    n -= n % world
    nbytes = n * E
    ref = None
    if not args.no_cpu_baseline:
        box = [reference_run(cfg, world, n, dev, False)[0] if rank == 0 else None]
        dist.broadcast_object_list(box, src=0)
        ref = box[0]
    sendbuf = synth(cfg, n, rank, dev)
    nrecv = n // world if coll == "reduce_scatter" else n
    recvbuf = torch.empty(nrecv * E, dtype=torch.uint8, device=dev)
    cnts = [n // world] * world
    comm.reserve(2 * nbytes)
    apply_variant(comm, exch_name)
    out = {"config": cfg, "workload": "%s %d MiB per rank" % (desc, nbytes // MIB),
           "vector_bytes_per_rank": nbytes, "exchange": exch_name}

    def step():
        if coll == "allreduce":
            rc = comm.allreduce_async(sendbuf, recvbuf, n, dtype, op, stream)
        else:
            rc = comm.reduce_scatter_async(sendbuf, recvbuf, cnts, dtype, op, stream)
        if rc:
            raise RuntimeError("%s rc=%d" % (coll, rc))

    status, est = checked_step(step, stream, args.variant_timeout)
    worst = agree(status)
    if worst:
        out["error"] = "an error return on some rank" if worst == 1 else "the checked step did not complete"
        return out, worst
    parity = None
    if ref is not None:
        allg = [None] * world
        dist.all_gather_object(allg, _digest(recvbuf.cpu().numpy()))
        parity = allg == ref
    out["exchange_ran"] = EXCH_NAMES.get(comm.last_exchange(), "?")
    try:
        times = timed(args, step, stream, world, agree, step_limit(args, est))
    except StepFailure as e:
        out["error"] = "timed steps: " + e.text()
        return out, e.worst
    p = world
    sec = times["t_job"] / args.steps
    busbw = (2 if coll == "allreduce" else 1) * (p - 1) / p * nbytes / sec / 1e9
    peak = min(p - 1, 7) * XGMI_LINK_GBS
    out.update(value=round(world * nbytes * args.steps / times["t_job"] / GIB, 2), unit="GiB/s",
               ms_per_step=round(sec * 1e3, 5), busbw_GBs=round(busbw, 1), frac=round(busbw / peak, 4),
               xgmi_peak_GBs=peak,
               parity=("bit-exact vs the reference schedule, all %d ranks" % p) if parity
               else ("MISMATCH" if parity is False else None))
    del sendbuf, recvbuf
    torch.cuda.empty_cache()
    return out, 0


def rccl_native(args, mvx, comm, cfg, n, sendbuf, world, dev, stream, agree, line_ms):
    """After the line: RCCL's own reduction on the same communicator and the
    same vectors -- ncclAllReduce (C3) or ncclReduceScatter (C4: over the
    same int64 bytes as a SUM, RCCL has no BAND) -- the ablation SURVEY.md
    8(e) keeps beside the path: RCCL's ring / tree order, not the
    reference's, so it is a speed reference, never the line.  C5's pairs
    have no RCCL reduction: None.  Returns (summary, worst status)."""
    import torch
    coll, dtype, _, E, _, _ = CONFIGS[cfg]
    if dtype not in (MPI_FLOAT, MPI_LONG):
        return None, 0
    kind = mvx.COLL_ALLREDUCE if coll == "allreduce" else mvx.COLL_REDUCE_SCATTER
    cnt = n if coll == "allreduce" else n // world
    out = torch.empty(cnt * E, dtype=torch.uint8, device=dev)

    def step():
        rc = comm.rccl_native(kind, sendbuf, out, cnt, dtype, stream)
        if rc:
            raise RuntimeError("mvx_comm_rccl_native rc=%d" % rc)

    status, est = checked_step(step, stream, args.variant_timeout)
    worst = agree(status)
    res = {"op": "ncclAllReduce(ncclSum)" if coll == "allreduce" else "ncclReduceScatter(ncclSum)",
           "note": "RCCL's own reduction on the same communicator and vectors (SURVEY.md 8(e) ablation): "
                   "its ring / tree order is not the reference's and it has no BAND, so this is a speed "
                   "reference for the exchange, never the line"}
    if worst:
        res["error"] = "an error return on some rank" if worst == 1 else "the checked step did not complete"
        return res, worst
    try:
        times = timed(args, step, stream, world, agree, step_limit(args, est))
    except StepFailure as e:
        res["error"] = "timed steps: " + e.text()
        return res, e.worst
    sec = times["t_job"] / args.steps
    p = world
    nbytes = n * E
    busbw = (2 if coll == "allreduce" else 1) * (p - 1) / p * nbytes / sec / 1e9
    peak = min(p - 1, 7) * XGMI_LINK_GBS
    res.update(ms_per_step=round(sec * 1e3, 5), busbw_GBs=round(busbw, 1), frac=round(busbw / peak, 4),
               line_over_native=round(line_ms / (sec * 1e3), 3))
    del out
    return res, 0


def rccl_view(comm, world, dev, transport):
    """RCCL's own account of the communicator, every rank's answer
    all-gathered (mvx_comm_rccl_info: ncclCommCount, ncclCommCuDevice,
    ncclGetVersion) next to the HIP device each rank drives (PCI location,
    UUID): what says the N ranks of the line sat on N distinct GPUs."""
    import torch
    import torch.distributed as dist
    info = comm.rccl_info()
    pr = torch.cuda.get_device_properties(dev)
    me = {"rccl": info, "hip_device": dev.index,
          "pci": "%04x:%02x:%02x" % (pr.pci_domain_id, pr.pci_bus_id, pr.pci_device_id),
          "uuid": str(getattr(pr, "uuid", ""))}
    allg = [None] * world
    dist.all_gather_object(allg, me)
    out = {"transport": transport,
           "hip_devices": [a["hip_device"] for a in allg],
           "pci": [a["pci"] for a in allg],
           "distinct_gpus": len({a["uuid"] or a["pci"] for a in allg})}
    if any(a["rccl"] is None for a in allg):
        out.update(nranks=None, devices=None, version=None,
                   note="no RCCL communicator (caller-supplied transport)")
        return out
    nr = [a["rccl"]["nranks"] for a in allg]
    out.update(nranks=nr[0] if len(set(nr)) == 1 else nr,
               devices=[a["rccl"]["device"] for a in allg],
               version=allg[0]["rccl"]["version"])
    return out


def run_multi(args, mvx, dev, world, rank, local, clock):
    import torch
    import torch.distributed as dist
    cfg = args.config or "c3"
    coll, dtype, op, E, mib, desc = CONFIGS[cfg]
    nbytes = (args.mib or mib) * MIB
    n = nbytes // E
    n -= n % world
    nbytes = n * E
    # a stream of its own (not the null stream): graph variants launch on it
    # directly instead of forking from and joining back to the null stream
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    tp = importlib.import_module("mvapich-cce_amd.transport") if args.transport == "host" else None

    def new_comm():
        if tp is not None:
            return mvx.Comm.from_transport(tp.TorchP2PTransport(), dev.index)
        return mvx.Comm.from_torch_distributed(dev.index)

    comm = new_comm()
    rccl = rccl_view(comm, world, dev, args.transport)
    clock.mark("communicator")
    sets = max(1, min(args.sets, 2))
    sendbuf = [synth(cfg, n, rank, dev) for _ in range(sets)]
    nrecv = n // world if coll == "reduce_scatter" else n
    recvbuf = [torch.empty(nrecv * E, dtype=torch.uint8, device=dev) for _ in range(sets)]
    cnts = [n // world] * world
    comm.reserve(2 * nbytes)
    torch.cuda.synchronize()
    clock.mark("inputs")
    it = [0]
    cur = {"name": None, "comm": comm, "best": None}

    def step():
        s = it[0] % sets
        it[0] += 1
        c = cur["comm"]
        if it[0] == 1 and _hang_injected(cur["name"], rank):
            return
        if coll == "allreduce":
            rc = c.allreduce_async(sendbuf[s], recvbuf[s], n, dtype, op, stream)
        else:
            rc = c.reduce_scatter_async(sendbuf[s], recvbuf[s], cnts, dtype, op, stream)
        if rc == 0 and _fail_injected(cur["name"], rank):
            rc = 15          # MPI_ERR_OTHER, after a complete step
        if rc:
            raise RuntimeError("%s rc=%d" % (coll, rc))

    # the reference's result (and the CPU baseline) on rank 0's host
    # cpu_baseline leg: the reference schedule on p host threads -- timed, and
    # its per-rank results are the parity reference
    ref, cpu = None, None
    if not args.no_cpu_baseline:
        if rank == 0:
            ref, secs, reps = reference_run(cfg, world, n, dev, True)
            cpu = {"value": round(world * nbytes / secs / GIB, 3), "unit": "GiB/s", "cores": world,
                   "kind": "port",
                   "sample": "reference schedule (oracle/cpu_coll.c) of the same %s on %d host threads, "
                             "one per rank, %d reps" % (cfg, world, reps),
                   "cpu": _cpu_model(), "ms_per_collective": round(secs * 1e3, 3)}
        box = [ref]
        dist.broadcast_object_list(box, src=0)
        ref = box[0]
    clock.mark("reference run (rank 0)")

    def agree(flag):
        """every rank's status, MAX over ranks (gloo: the host side, which a
        stuck GPU stream cannot block)"""
        t = torch.tensor([flag], dtype=torch.int64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return int(t.item())

    def parity_check():
        """set 0's result on every rank against the reference's digests"""
        if ref is None:
            return None
        mine = _digest(recvbuf[0].cpu().numpy())
        allg = [None] * world
        dist.all_gather_object(allg, mine)
        return allg == ref

    def emit(out):
        """rank 0 prints the line, with where the wall clock went"""
        if rank == 0 and out is not None:
            out["config"]["exchange_tuning"] = tried
            out["rccl"] = rccl
            out["env"] = env_echo()
            clock.mark("finish")
            out["wall"] = clock.report()
            print(json.dumps(out), flush=True)

    def recover(worst, entry):
        """after a failed block on every rank: a hang tears the communicator
        down (ncclCommAbort) and builds a fresh one.  If the stream stays
        blocked even then, rank 0 prints the line already measured and the
        run ends (exit 0 with a line, 1 without)."""
        if worst != 2:
            return
        cur["comm"].abort()
        if agree(0 if _wait_stream(stream, args.variant_timeout) else 1):
            entry["error"] += "; the stream stayed blocked after ncclCommAbort"
            emit(cur["best"])
            sys.stdout.flush()
            sys.stderr.flush()
            os._exit(0 if cur["best"] is not None else 1)
        cur["comm"] = new_comm()
        cur["comm"].reserve(2 * nbytes)

    def measure(name, est_s):
        """the K timed steps (and the per-phase breakdown) of variant `name`:
        one candidate line.  StepFailure propagates from the timed steps; a
        failure in the untimed phase steps is recorded in the line's phases
        and returned as its status."""
        cur["name"] = name
        apply_variant(cur["comm"], name)
        limit = step_limit(args, est_s)
        times = timed(args, step, stream, world, agree, limit)
        ran = EXCH_NAMES.get(cur["comm"].last_exchange(), "?")
        graph = GRAPH_STATES.get(cur["comm"].last_graph()[0]) if EXCH[name][2] else None
        # set 0's result as the timed steps left it (graph replays included)
        # against the reference again
        post = parity_check()
        pb = plan_bytes(mvx, coll, world, rank, n, cnts, dtype, op)
        status = 0
        try:
            phases = phase_breakdown(cur["comm"], step, coll, world, nbytes, pb, stream, agree, limit)
        except StepFailure as e:
            phases, status = {"error": "phase-timing steps: " + e.text()}, e.worst
        p = world
        sec = times["t_job"] / args.steps
        if coll == "allreduce":
            busbw = 2 * (p - 1) / p * nbytes / sec / 1e9
            note = "busbw = 2(p-1)/p*S/t"
        else:
            busbw = (p - 1) / p * nbytes / sec / 1e9
            note = "busbw = (p-1)/p*S/t"
        links = min(p - 1, 7)
        peak = links * XGMI_LINK_GBS
        roof = {"bound": "xgmi", "achieved": round(busbw, 1), "peak": peak, "unit": "GB/s",
                "frac": round(busbw / peak, 4), "traffic": None, "kernel": mvx.last_kernel(),
                "note": "%s against %d direct xGMI links x %.0f GB/s" % (note, links, XGMI_LINK_GBS),
                "combine_hbm_bytes_per_step": (p + 1) * nbytes // p, "phases": phases}
        out = result(args, world, nbytes, times, {"c3": "f32", "c4": "int64", "c5": "f32+int32"}[cfg],
                     {"workload": "%s: %s %d MiB per rank, RCCL xGMI exchange + reference-order combine"
                                  % (cfg, desc, nbytes // MIB),
                      "vector_bytes_per_rank": nbytes, "parallelism": "dp%d (blocks sharded over ranks)" % p,
                      "exchange": name, "exchange_ran": ran, "graph": graph, "exchange_tuning": None,
                      "transport": args.transport}, roof)
        parity = tried[name]["parity"]
        if post is False:
            parity = False
        out["parity"] = (("bit-exact vs the reference schedule, all %d ranks" % p) if parity
                         else ("MISMATCH" if parity is False else None))
        out["parity_after_timed"] = post
        out["cpu_baseline"] = cpu
        return out, status

    # Exchange variants in EXCH order (p2p first, coll last).  Each gets one
    # checked step, then --tune-steps timed steps if every rank completed it
    # without an error; a variant that errs or never completes on any rank --
    # in its checked step, its tuning steps, its timed steps or its phase
    # steps -- is recorded and left out (a hung one first tears the
    # communicator down and builds a fresh one).  The first clean variant is
    # measured for the line at once (K timed steps), and a later one is
    # measured again only if its tuning steps ran faster -- so a line exists
    # before any riskier variant runs, and a variant that wedges the GPU for
    # good ends the run with the line already measured rather than with none.
    names = auto_variants(args) if args.exchange == "auto" else args.exchange.split(",")
    tried = {}

    for name in names:
        mode = EXCH[name][0]
        cur["name"] = name
        status = 1 if apply_variant(cur["comm"], name) else 0
        est = 0.0
        if agree(status) == 0:
            it[0] = 0
            status, est = checked_step(step, stream, args.variant_timeout)
        worst = agree(status)
        ok, ran = None, None
        if worst == 0:
            ok = parity_check()
            ran = EXCH_NAMES.get(cur["comm"].last_exchange(), "?")
            if ran != EXCH_NAMES[mode]:
                ran += " (fallback)"
        entry = {"ran": ran}
        tried[name] = entry
        if worst:
            entry.update(ms_per_step=None, parity=None,
                         error="an error return on some rank" if worst == 1 else
                               "a step did not complete within %.0f s" % args.variant_timeout)
            recover(worst, entry)
            clock.mark("variant %s" % name)
            continue
        t = torch.zeros(1, dtype=torch.float64)
        terr = 0
        if EXCH[name][2]:
            # graphs: each input set's first call ran eagerly, its second is
            # captured -- untimed here, so the tuning steps are replays.  A
            # first launch that never completes is a hung variant like any
            # other: a bounded wait, then agree / recover.
            try:
                for _ in range(2 * sets):
                    step()
            except RuntimeError:
                terr = 1
            if terr == 0 and not _wait_stream(stream, step_limit(args, est)):
                terr = 2
            worst = agree(terr)
            if worst:
                entry.update(ms_per_step=None, parity=ok,
                             error=("an error return on some rank while capturing" if worst == 1 else
                                    "a captured step did not complete within %.0f s" % step_limit(args, est)))
                recover(worst, entry)
                clock.mark("variant %s" % name)
                continue
        torch.cuda.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        issue = []
        for _ in range(args.tune_steps):      # every rank issues every step
            t1 = time.perf_counter()
            try:
                step()
            except RuntimeError:
                terr = 1
            issue.append(time.perf_counter() - t1)
        tlim = step_limit(args, est)
        if terr == 0 and not _wait_stream(stream, tlim, spin=True):
            terr = 2
        t[0] = time.perf_counter() - t0
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        # host time inside one collective call (plan, staging, RCCL enqueue
        # and kernel launches; RCCL returns before the transfers end), the
        # median over the tuning steps, MAX over ranks
        hi = torch.tensor([statistics.median(issue)], dtype=torch.float64)
        dist.all_reduce(hi, op=dist.ReduceOp.MAX)
        worst = agree(terr)
        if worst:
            entry.update(ms_per_step=None, parity=ok,
                         error=("an error return on some rank while tuning" if worst == 1 else
                                "a tuning step did not complete within %.0f s" % tlim))
            recover(worst, entry)
            clock.mark("variant %s" % name)
            continue
        torch.cuda.synchronize()
        entry.update(ms_per_step=round(float(t.item()) * 1e3 / args.tune_steps, 4), parity=ok,
                     host_issue_us=round(float(hi.item()) * 1e6, 1))
        if EXCH[name][2]:
            # what the last tuning step was: a replayed graph (1), a capture (2)
            # or an eager call (0: graphs off on this communicator, see error)
            gs, ge = cur["comm"].last_graph()
            entry["graph"] = {"state": GRAPH_STATES.get(gs, gs), "capture_error": ge}
        # measure for the line: the first clean variant, then any that tuned
        # faster than the one measured (every rank decides alike: the tuning
        # time is the MAX over ranks and parity is compared on every rank)
        best = cur["best"]
        if choose_variant([name], tried) == name and (
                best is None or entry["ms_per_step"] < tried[best["config"]["exchange"]]["ms_per_step"]):
            box = [name]
            dist.broadcast_object_list(box, src=0)
            try:
                cand, pstat = measure(box[0], max(est, entry["ms_per_step"] * 1e-3))
            except StepFailure as e:
                entry.update(ms_per_step=None, error="timed steps: " + e.text())
                recover(e.worst, entry)
                clock.mark("variant %s" % name)
                continue
            if cand.get("parity_after_timed") is False:
                entry.update(parity=False, error="MISMATCH in the result the timed steps left")
            elif best is None or cand["ms_per_step"] < best["ms_per_step"]:
                cur["best"] = cand
            if pstat:
                entry["error"] = cand["roofline"]["phases"]["error"]
                recover(pstat, entry)
        clock.mark("variant %s" % name)
    out = cur["best"]
    if out is None:
        if rank == 0:
            sys.stderr.write("bench: no exchange variant ran clean with parity: %s\n" % json.dumps(tried))
        return None, emit
    # the other BASELINE configs quoted at this GPU count, on the same
    # communicator and exchange variant, after the line's timed region
    extras = EXTRA_AT.get(world, []) if args.extra_configs == "auto" else \
        [c for c in args.extra_configs.split(",") if c and c != "none"]
    others, aborted = [], False
    for cfg2 in extras:
        if cfg2 == cfg:
            continue
        res, worst = run_extra(args, mvx, dev, world, rank, cur["comm"], out["config"]["exchange"], cfg2,
                               agree, stream)
        others.append(res)
        clock.mark("other config %s" % cfg2)
        if worst == 2:           # a hang: leave the communicator, keep the line
            cur["comm"].abort()
            aborted = True
            break
    if others:
        out["other_configs"] = others
    if not aborted and not args.no_native and args.transport != "host":
        nat, worst = rccl_native(args, mvx, cur["comm"], cfg, n, sendbuf[0], world, dev, stream, agree,
                                 out["ms_per_step"])
        if nat is not None:
            out["rccl_native"] = nat
            clock.mark("rccl native")
        if worst == 2:
            cur["comm"].abort()
            aborted = True
    if not aborted:
        cur["comm"].free()
    return out, emit


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    how, val = decide_launch(args.gpus, os.environ)
    if how == "mismatch":
        sys.stderr.write("bench: %s\n" % val)
        sys.exit(2)
    if how == "self":
        sys.exit(launch(args, val, argv))
    world = val
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    clock = Stages(verbose=rank == 0 and world > 1)
    import torch
    import torch.distributed as dist

    if args.transport == "rccl-net":
        importlib.import_module("mvapich-cce_amd.transport").rccl_net_env(rank)
    dev_index = local % torch.cuda.device_count() if args.transport != "rccl" else local
    torch.cuda.set_device(dev_index)
    dev = torch.device("cuda", dev_index)
    mvx = importlib.import_module("mvapich-cce_amd")
    if args.block_cap or args.nt_min_log2:
        mvx.set_launch(args.block_cap, args.nt_min_log2)
    if world == 1:
        if args.config not in (None, "c2"):
            sys.exit("configs c3-c5 are multi-GPU: run with --gpus N (N > 1)")
        clock.mark("start-up (imports)")
        run_single(args, mvx, dev, clock)
        return
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    # gloo bootstraps, agrees and checks (and is the host transport's byte
    # mover): a peer that never arrives fails the call after this long
    # instead of gloo's 30 minutes; rank 0's reference run (tens of seconds
    # at C5 x 8) stays well inside it
    import datetime
    with _StdoutToStderr():
        dist.init_process_group("gloo", rank=rank, world_size=world,
                                timeout=datetime.timedelta(seconds=args.gloo_timeout))
        dist.barrier()                       # (the connections form here or above)
    clock.mark("start-up (imports, process group)")
    out, emit = run_multi(args, mvx, dev, world, rank, local, clock)
    emit(out)
    dist.barrier()
    dist.destroy_process_group()
    if out is None:
        sys.exit(1)


if __name__ == "__main__":
    main()
