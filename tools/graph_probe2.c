/*
 * graph_probe2.c -- the round-4 hipGraphLaunch SIGSEGV, without libmvx.
 *
 * Round 4 saw RCCL communicators of 2 and 4 ranks (sharing one GPU over
 * RCCL's socket transport) die with SIGSEGV in the launch of a freshly
 * captured graph, after graph execs of earlier jobs had been destroyed
 * (profiles/r04/graph_crash_after_destroy_p2.log:1001-1011): P2P graphs
 * captured after the destroys launched, a COLL graph (ncclAllToAll +
 * in-place ncclAllGather) did not; at p = 4 a PIPE graph (fork / join to a
 * second stream) did not.  libmvx destroys each hipGraph_t right after
 * instantiating it and keeps only the exec.
 *
 * Each scenario below runs in a fresh pair of processes (forked before any
 * HIP call, NCCL_HOSTID per rank as transport.rccl_net_env), so one that
 * crashes does not stop the others; the parent prints one verdict line per
 * scenario (ok / exit code / signal).  Scenarios differ in one thing each:
 *
 *   coll_after_destroy      capture P2P graphs G1 G2 (graphs destroyed at
 *                           instantiation, as libmvx), launch, destroy G1's
 *                           exec, eager COLL, capture COLL, launch x3
 *   coll_no_destroy         the same, G1's exec kept
 *   coll_after_destroy_keep the same as the first, every hipGraph_t kept
 *                           alive until the end (only execs destroyed)
 *   p2p_after_destroy       the first, with a P2P job captured last
 *   coll_then_coll          capture COLL, launch, destroy its exec, capture
 *                           COLL again, launch x3
 *   fork_after_destroy      the first, with a fork / join capture (PIPE's
 *                           shape: P2P groups, a memset forked to stream 2)
 *   coll_destroy_sync       the first, with hipDeviceSynchronize and an
 *                           eager RCCL call between the destroy and the
 *                           capture (RCCL reclaims a destroyed graph's plan
 *                           on its next call)
 *   coll_free_then_destroy  libmvx's round-4 order when its staging pool
 *                           grew: COLL captured on buffer A, launched; A
 *                           freed (hipFree) while the exec lives; the exec
 *                           destroyed; buffer B allocated; COLL eager, then
 *                           captured on B and launched x3
 *   coll_destroy_then_free  the same with the exec destroyed before A is
 *                           freed
 *   p2p_free_then_destroy   the first order with P2P groups instead of COLL
 *   null_fork_pipe_cumask   null_fork_pipe with stream 2 made as libmvx
 *                           makes PIPE's combine stream
 *                           (hipExtStreamCreateWithCUMask: a blocking
 *                           stream with a full CU mask) and three forks to
 *                           it per job, one join (PIPE's shape)
 *   fork_cumask_stream      the same on a plain capturing stream (no null
 *                           stream)
 *   copy_then_pipe          G1, G2 = a group plus a device-to-device
 *                           hipMemcpyAsync (libmvx's one-leaf combines and
 *                           own-block copies), G1 destroyed, then PIPE's
 *                           shape captured and launched
 *   null_copy_then_pipe     the same on the null-stream path
 *   churn_pipe              200 rounds of: capture PIPE's shape, instantiate,
 *                           launch, destroy the exec (libmvx with eviction
 *                           crashed after 40-70 graphs per process)
 *   churn_fork_norccl       the same with no RCCL call in the graph (a
 *                           memset on each branch)
 *   churn_p2p               the same with one group per graph
 *   churn_fork_keep         churn_fork_norccl without destroying: every
 *                           exec kept until the end
 *   churn_single            churn_fork_norccl with no fork (one stream)
 *   null_fork_{p2p,coll,pipe}  libmvx's blocking (null-stream) path: the
 *                           job's eager runs on the null stream; its graphs
 *                           are captured on a second stream (gs) and
 *                           launched forked from / joined back to the null
 *                           stream with events; G1 G2 captured and
 *                           launched, G1's exec destroyed, an eager job on
 *                           the null stream, then G3 captured and launched
 *
 *   gcc -O2 -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include tools/graph_probe2.c \
 *       -o tools/graph_probe2 -L/opt/rocm/lib -lrccl -lamdhip64
 *   tools/graph_probe2 [scenario ...]      (default: all)
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/wait.h>
#include <unistd.h>

#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#define N (1 << 20)
#define P 2
#define CHK(x, what)                                                     \
    do {                                                                 \
        if (!(x)) {                                                      \
            fprintf(stderr, "rank %d: %s failed\n", rank, what);         \
            return 1;                                                    \
        }                                                                \
    } while (0)

static const char *g_names[] = {"coll_after_destroy", "coll_no_destroy", "coll_after_destroy_keep",
                                "p2p_after_destroy", "coll_then_coll", "fork_after_destroy",
                                "coll_destroy_sync", "coll_free_then_destroy", "coll_destroy_then_free",
                                "p2p_free_then_destroy", "null_fork_p2p", "null_fork_coll", "null_fork_pipe",
                                "null_fork_pipe_cumask", "fork_cumask_stream", "copy_then_pipe",
                                "null_copy_then_pipe", "churn_pipe", "churn_fork_norccl", "churn_p2p",
                                "churn_fork_keep", "churn_single"};
#define NSCEN ((int)(sizeof g_names / sizeof g_names[0]))

typedef struct {
    ncclComm_t comm;
    int rank;
    int *send, *recv, *host;
    hipStream_t st, s2, gs;
    hipEvent_t ev[2], gev[2];
} ctx_t;

static void say(int rank, const char *s) { fprintf(stderr, "rank %d: %s\n", rank, s); }

static int p2p(ctx_t *c)
{
    if (ncclGroupStart() != ncclSuccess) return 1;
    if (ncclSend(c->send, N, ncclInt32, 1 - c->rank, c->comm, c->st) != ncclSuccess) return 1;
    if (ncclRecv(c->recv, N, ncclInt32, 1 - c->rank, c->comm, c->st) != ncclSuccess) return 1;
    return ncclGroupEnd() != ncclSuccess;
}

/* libmvx's COLL: all-to-all of p blocks, then an in-place all-gather */
static int coll(ctx_t *c)
{
    const size_t b = N / P;
    if (ncclAllToAll(c->send, c->recv, b, ncclInt32, c->comm, c->st) != ncclSuccess) return 1;
    return ncclAllGather(c->recv + c->rank * b, c->recv, b, ncclInt32, c->comm, c->st) != ncclSuccess;
}

/* PIPE's shape: a group, a fork to stream 2, a group, the join */
static int fork_join(ctx_t *c)
{
    if (p2p(c)) return 1;
    if (hipEventRecord(c->ev[0], c->st) != hipSuccess || hipStreamWaitEvent(c->s2, c->ev[0], 0) != hipSuccess)
        return 1;
    if (hipMemsetAsync(c->send + N / 2, 0, 4, c->s2) != hipSuccess) return 1;
    if (hipEventRecord(c->ev[1], c->s2) != hipSuccess) return 1;
    if (p2p(c)) return 1;
    return hipStreamWaitEvent(c->st, c->ev[1], 0) != hipSuccess;
}

/* PIPE's shape proper: per slice a group on st, a fork to s2 (events
 * reused by slice parity) and work there; one join at the end */
static int pipe3(ctx_t *c)
{
    int t;
    for (t = 0; t < 3; t++) {
        if (p2p(c)) return 1;
        if (hipEventRecord(c->ev[t & 1], c->st) != hipSuccess || hipStreamWaitEvent(c->s2, c->ev[t & 1], 0) != hipSuccess)
            return 1;
        if (hipMemsetAsync(c->send + N / 2 + t, 0, 4, c->s2) != hipSuccess) return 1;
    }
    if (hipEventRecord(c->ev[0], c->s2) != hipSuccess || hipStreamWaitEvent(c->st, c->ev[0], 0) != hipSuccess) return 1;
    return p2p(c);
}

/* a group, then a device-to-device copy on the same stream */
static int p2p_copy(ctx_t *c)
{
    if (p2p(c)) return 1;
    return hipMemcpyAsync(c->send + N / 2, c->recv, 4096, hipMemcpyDeviceToDevice, c->st) != hipSuccess;
}

typedef int (*job_fn)(ctx_t *);

/* capture `job` on st; the graph is destroyed at once unless keep != NULL */
static int capture(ctx_t *c, job_fn job, hipGraphExec_t *x, hipGraph_t *keep)
{
    hipGraph_t g = NULL;
    int rank = c->rank;
    CHK(hipStreamBeginCapture(c->st, hipStreamCaptureModeThreadLocal) == hipSuccess, "begin capture");
    CHK(job(c) == 0, "captured job");
    CHK(hipStreamEndCapture(c->st, &g) == hipSuccess && g, "end capture");
    say(rank, "instantiate");
    CHK(hipGraphInstantiate(x, g, NULL, NULL, 0) == hipSuccess, "instantiate");
    if (keep) *keep = g;
    else hipGraphDestroy(g);
    return 0;
}

static int launch(ctx_t *c, hipGraphExec_t x, int times)
{
    int i, rank = c->rank;
    for (i = 0; i < times; i++) {
        say(rank, "launch");
        CHK(hipGraphLaunch(x, c->st) == hipSuccess, "launch");
        CHK(hipStreamSynchronize(c->st) == hipSuccess, "launch sync");
    }
    return 0;
}

/* the job on a fresh pair of buffers of `bytes` each (c->send / c->recv
 * pointed at them); the old pair is freed before (free_first) or after the
 * exec that captured it is destroyed */
static int realloc_case(ctx_t *c, job_fn job, int free_first)
{
    int *a_send, *a_recv, *b_send, *b_recv;
    hipGraphExec_t g1, g2;
    int rank = c->rank;
    CHK(hipMalloc((void **)&a_send, N * sizeof(int)) == hipSuccess && hipMalloc((void **)&a_recv, N * sizeof(int)) == hipSuccess, "malloc a");
    CHK(hipMemcpy(a_send, c->host, N * sizeof(int), hipMemcpyHostToDevice) == hipSuccess, "h2d a");
    c->send = a_send; c->recv = a_recv;
    CHK(job(c) == 0 && hipStreamSynchronize(c->st) == hipSuccess, "eager on a");
    CHK(capture(c, job, &g1, NULL) == 0, "capture on a");
    CHK(launch(c, g1, 2) == 0, "launch on a");
    CHK(hipDeviceSynchronize() == hipSuccess, "sync");
    if (free_first) {
        say(rank, "free a, exec alive");
        hipFree(a_send); hipFree(a_recv);
        say(rank, "destroy exec of a");
        hipGraphExecDestroy(g1);
    } else {
        say(rank, "destroy exec of a");
        hipGraphExecDestroy(g1);
        say(rank, "free a");
        hipFree(a_send); hipFree(a_recv);
    }
    CHK(hipMalloc((void **)&b_send, 2 * N * sizeof(int)) == hipSuccess && hipMalloc((void **)&b_recv, 2 * N * sizeof(int)) == hipSuccess, "malloc b");
    CHK(hipMemcpy(b_send, c->host, N * sizeof(int), hipMemcpyHostToDevice) == hipSuccess, "h2d b");
    c->send = b_send; c->recv = b_recv;
    CHK(job(c) == 0 && hipStreamSynchronize(c->st) == hipSuccess, "eager on b");
    CHK(capture(c, job, &g2, NULL) == 0, "capture on b");
    CHK(launch(c, g2, 3) == 0, "launch on b");
    hipGraphExecDestroy(g2);
    return 0;
}

static int scenario_graphs(ctx_t *c, int s)
{
    hipGraphExec_t g1, g2, g3;
    hipGraph_t k1 = NULL, k2 = NULL, k3 = NULL;
    const int keep = s == 2;
    int rank = c->rank;
    job_fn last = s == 3 ? p2p : s == 5 ? fork_join : (s == 16 || s == 17) ? pipe3 : coll;
    job_fn first = s == 16 ? p2p_copy : p2p;

    if (s == 4) {                                   /* coll_then_coll */
        CHK(coll(c) == 0 && hipStreamSynchronize(c->st) == hipSuccess, "eager coll");
        CHK(capture(c, coll, &g1, NULL) == 0, "capture coll 1");
        CHK(launch(c, g1, 2) == 0, "launch coll 1");
        say(rank, "destroy exec");
        hipGraphExecDestroy(g1);
        CHK(capture(c, coll, &g2, NULL) == 0, "capture coll 2");
        CHK(launch(c, g2, 3) == 0, "launch coll 2");
        hipGraphExecDestroy(g2);
        return 0;
    }
    CHK(first(c) == 0 && hipStreamSynchronize(c->st) == hipSuccess, "eager p2p");
    CHK(capture(c, first, &g1, keep ? &k1 : NULL) == 0, "capture p2p 1");
    CHK(launch(c, g1, 2) == 0, "launch p2p 1");
    CHK(capture(c, first, &g2, keep ? &k2 : NULL) == 0, "capture p2p 2");
    CHK(launch(c, g2, 2) == 0, "launch p2p 2");
    if (s != 1) {
        say(rank, "destroy exec 1");
        hipGraphExecDestroy(g1);
    }
    if (s == 6) {
        CHK(hipDeviceSynchronize() == hipSuccess, "device sync");
        CHK(p2p(c) == 0 && hipStreamSynchronize(c->st) == hipSuccess, "eager p2p after destroy");
    }
    CHK(last(c) == 0 && hipStreamSynchronize(c->st) == hipSuccess, "eager last job");
    CHK(capture(c, last, &g3, keep ? &k3 : NULL) == 0, "capture last job");
    CHK(launch(c, g3, 3) == 0, "launch last job");
    say(rank, "teardown");
    hipGraphExecDestroy(g3);
    hipGraphExecDestroy(g2);
    if (s == 1) hipGraphExecDestroy(g1);
    if (k1) hipGraphDestroy(k1);
    if (k2) hipGraphDestroy(k2);
    if (k3) hipGraphDestroy(k3);
    return 0;
}

/* a graph launched as libmvx launches one for a null-stream call */
static int launch_null(ctx_t *c, hipGraphExec_t x, int times)
{
    int i, rank = c->rank;
    for (i = 0; i < times; i++) {
        say(rank, "launch forked from the null stream");
        CHK(hipEventRecord(c->gev[0], NULL) == hipSuccess && hipStreamWaitEvent(c->gs, c->gev[0], 0) == hipSuccess,
            "fork");
        CHK(hipGraphLaunch(x, c->gs) == hipSuccess, "launch");
        CHK(hipEventRecord(c->gev[1], c->gs) == hipSuccess && hipStreamWaitEvent(NULL, c->gev[1], 0) == hipSuccess,
            "join");
        CHK(hipStreamSynchronize(NULL) == hipSuccess, "null sync");
    }
    return 0;
}

static int null_fork2(ctx_t *c, job_fn job, job_fn last);

static int null_fork(ctx_t *c, job_fn job) { return null_fork2(c, job, job); }

static int null_fork2(ctx_t *c, job_fn job, job_fn last)
{
    hipGraphExec_t g1, g2, g3;
    hipStream_t st = c->st;
    int rank = c->rank;
    /* eager on the null stream */
    c->st = NULL;
    CHK(job(c) == 0 && hipStreamSynchronize(NULL) == hipSuccess, "eager on the null stream");
    /* captures on gs */
    c->st = c->gs;
    CHK(capture(c, job, &g1, NULL) == 0, "capture 1 on gs");
    CHK(launch_null(c, g1, 2) == 0, "launch 1");
    CHK(capture(c, job, &g2, NULL) == 0, "capture 2 on gs");
    CHK(launch_null(c, g2, 2) == 0, "launch 2");
    say(rank, "destroy exec 1");
    hipGraphExecDestroy(g1);
    c->st = NULL;
    CHK(last(c) == 0 && hipStreamSynchronize(NULL) == hipSuccess, "eager on the null stream after destroy");
    c->st = c->gs;
    CHK(capture(c, last, &g3, NULL) == 0, "capture 3 on gs");
    CHK(launch_null(c, g3, 3) == 0, "launch 3");
    hipGraphExecDestroy(g3);
    hipGraphExecDestroy(g2);
    c->st = st;
    return 0;
}

/* fork / join with memsets only: no RCCL in the graph */
static int fork_norccl(ctx_t *c)
{
    int t;
    for (t = 0; t < 3; t++) {
        if (hipMemsetAsync(c->recv + t, 0, 4, c->st) != hipSuccess) return 1;
        if (hipEventRecord(c->ev[t & 1], c->st) != hipSuccess || hipStreamWaitEvent(c->s2, c->ev[t & 1], 0) != hipSuccess)
            return 1;
        if (hipMemsetAsync(c->send + N / 2 + t, 0, 4, c->s2) != hipSuccess) return 1;
    }
    if (hipEventRecord(c->ev[0], c->s2) != hipSuccess || hipStreamWaitEvent(c->st, c->ev[0], 0) != hipSuccess) return 1;
    return hipMemsetAsync(c->recv + 8, 0, 4, c->st) != hipSuccess;
}

/* memsets on one stream: a graph with a single branch */
static int single_norccl(ctx_t *c)
{
    int t;
    for (t = 0; t < 4; t++)
        if (hipMemsetAsync(c->recv + t, 0, 4, c->st) != hipSuccess) return 1;
    return 0;
}

static int churn(ctx_t *c, job_fn job, int rounds, int keep)
{
    static hipGraphExec_t kept[256];
    hipGraphExec_t x;
    int i, rank = c->rank;
    char msg[64];
    CHK(job(c) == 0 && hipStreamSynchronize(c->st) == hipSuccess, "eager");
    for (i = 0; i < rounds; i++) {
        if (i % 10 == 0) {
            snprintf(msg, sizeof msg, "churn round %d", i);
            say(rank, msg);
        }
        CHK(capture(c, job, &x, NULL) == 0, "capture");
        CHK(hipGraphLaunch(x, c->st) == hipSuccess && hipStreamSynchronize(c->st) == hipSuccess, "launch");
        if (keep && i < 256) kept[i] = x;
        else CHK(hipGraphExecDestroy(x) == hipSuccess, "destroy");
    }
    for (i = 0; keep && i < rounds && i < 256; i++) hipGraphExecDestroy(kept[i]);
    return 0;
}

static int scenario(ctx_t *c, int s)
{
    if (s == 17) return churn(c, pipe3, 200, 0);
    if (s == 18) return churn(c, fork_norccl, 200, 0);
    if (s == 19) return churn(c, p2p, 200, 0);
    if (s == 20) return churn(c, fork_norccl, 200, 1);
    if (s == 21) return churn(c, single_norccl, 200, 0);
    if (s == 7 || s == 8) return realloc_case(c, coll, s == 7);
    if (s == 9) return realloc_case(c, p2p, 1);
    if (s == 15) return scenario_graphs(c, 16);
    if (s == 16) return null_fork2(c, p2p_copy, pipe3);
    if (s == 13 || s == 14) {                      /* s2 as PIPE's combine stream */
        uint32_t mask[16];
        int rank = c->rank;
        memset(mask, 0xff, sizeof mask);
        CHK(hipStreamDestroy(c->s2) == hipSuccess, "destroy s2");
        CHK(hipExtStreamCreateWithCUMask(&c->s2, 16, mask) == hipSuccess, "cu-mask stream");
        if (s == 13) return null_fork(c, pipe3);
        return scenario_graphs(c, 17);
    }
    if (s >= 10) return null_fork(c, s == 10 ? p2p : s == 11 ? coll : fork_join);
    return scenario_graphs(c, s);
}

static int run(int rank, ncclUniqueId id, int s)
{
    ctx_t c;
    int i;
    memset(&c, 0, sizeof c);
    c.rank = rank;
    CHK(hipSetDevice(0) == hipSuccess, "hipSetDevice");
    CHK(hipStreamCreateWithFlags(&c.st, hipStreamNonBlocking) == hipSuccess, "stream");
    CHK(hipStreamCreateWithFlags(&c.s2, hipStreamNonBlocking) == hipSuccess, "stream 2");
    CHK(hipStreamCreateWithFlags(&c.gs, hipStreamNonBlocking) == hipSuccess, "graph stream");
    for (i = 0; i < 2; i++) CHK(hipEventCreateWithFlags(&c.ev[i], hipEventDisableTiming) == hipSuccess, "event");
    for (i = 0; i < 2; i++) CHK(hipEventCreateWithFlags(&c.gev[i], hipEventDisableTiming) == hipSuccess, "event");
    CHK(hipMalloc((void **)&c.send, N * sizeof(int)) == hipSuccess, "malloc");
    CHK(hipMalloc((void **)&c.recv, N * sizeof(int)) == hipSuccess, "malloc");
    c.host = (int *)malloc(N * sizeof(int));
    for (i = 0; i < N; i++) c.host[i] = rank * 1000003 + i;
    CHK(hipMemcpy(c.send, c.host, N * sizeof(int), hipMemcpyHostToDevice) == hipSuccess, "h2d");
    CHK(ncclCommInitRank(&c.comm, P, id, rank) == ncclSuccess, "ncclCommInitRank");
    if (scenario(&c, s)) return 1;
    say(rank, "ok");
    ncclCommDestroy(c.comm);
    return 0;
}

static int one(int s)
{
    ncclUniqueId id;
    int fd[2], r, rc = 0, status;
    pid_t kid[P];
    char verdict[128] = "ok";
    if (pipe(fd)) return 1;
    for (r = 0; r < P; r++) {
        kid[r] = fork();
        if (kid[r] == 0) {
            char hid[48];
            snprintf(hid, sizeof hid, "probe2-%d-rank-%d", s, r);
            setenv("NCCL_HOSTID", hid, 1);
            if (r == 0) {
                close(fd[0]);
                if (ncclGetUniqueId(&id) != ncclSuccess) _exit(1);
                if (write(fd[1], &id, sizeof id) != sizeof id) _exit(1);
            } else {
                close(fd[1]);
                if (read(fd[0], &id, sizeof id) != sizeof id) _exit(1);
            }
            alarm(60);                       /* a hung scenario ends as SIGALRM */
            _exit(run(r, id, s));
        }
    }
    close(fd[0]);
    close(fd[1]);
    for (r = 0; r < P; r++) {
        waitpid(kid[r], &status, 0);
        if (!WIFEXITED(status) || WEXITSTATUS(status)) {
            snprintf(verdict, sizeof verdict, "rank %d %s %d", r, WIFSIGNALED(status) ? "signal" : "exit",
                     WIFSIGNALED(status) ? WTERMSIG(status) : WEXITSTATUS(status));
            rc = 1;
        }
    }
    printf("graph_probe2 %-24s %s\n", g_names[s], verdict);
    fflush(stdout);
    return rc;
}

int main(int argc, char **argv)
{
    int s, i, bad = 0;
    setenv("NCCL_SOCKET_IFNAME", "lo", 0);
    setenv("NCCL_IB_DISABLE", "1", 0);
    for (s = 0; s < NSCEN; s++) {
        int want = argc < 2;
        for (i = 1; i < argc; i++) want |= !strcmp(argv[i], g_names[s]);
        if (want) bad += one(s);
    }
    return bad ? 1 : 0;
}
