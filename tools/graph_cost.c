/*
 * graph_cost.c -- where does the host time of a PIPE-shaped call go, eager
 * and as a replayed HIP graph?  p processes (forked before any HIP call)
 * share the box's one GPU as p "hosts" (NCCL_HOSTID, RCCL's socket
 * transport, as transport.rccl_net_env) and issue round 3's PIPE shape for S
 * slices: step t groups slice t's exchange and slice t - 2's distribution (one
 * send / receive per peer and phase), slice t's combine runs on a second
 * stream forked and joined through events (a memset stands in for it).
 * The second shape is round 4's PIPE: a fork to the combine stream per
 * slice, one join, one distribution group.  (A third shape, the slices
 * alternating between two streams with each slice's exchange and combine in
 * stream order, did not finish at p = 8 within 200 s (round 4): RCCL groups
 * of one communicator on two streams are not ordered against each other,
 * so it is not a schedule to use.)
 * Measured per (shape, S, with or without RCCL): host time to issue the sequence
 * eagerly on an idle GPU, host time of one hipGraphLaunch of its capture on
 * an idle GPU, the mean over 10 launches issued back to back, and the
 * captured graph's nodes by type.  Without RCCL each transfer group is
 * replaced by one memset, so the two rows separate RCCL's share (its
 * kernels, and the host nodes its proxy needs per replay) from the
 * graph's own launch cost.  Rank 0 prints one JSON line per row.
 *
 *   gcc -O2 -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include tools/graph_cost.c \
 *       -o tools/graph_cost -L/opt/rocm/lib -lrccl -lamdhip64
 *   tools/graph_cost [p]
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/wait.h>
#include <time.h>
#include <unistd.h>

#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#define SLICE_BYTES (256 << 10)     /* per peer, per slice, per phase */
#define MAXS 8
#define REPS 10

static double now_us(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec * 1e6 + ts.tv_nsec * 1e-3;
}

static int cmp_d(const void *a, const void *b)
{
    double x = *(const double *)a, y = *(const double *)b;
    return x < y ? -1 : x > y;
}

static double median(double *v, int n)
{
    qsort(v, n, sizeof *v, cmp_d);
    return v[n / 2];
}

typedef struct {
    int rank, p;
    ncclComm_t comm;
    hipStream_t st, s2;
    hipEvent_t fe[2], je[2];
    char *send, *recv, *scratch;
} ctx_t;

#define OK(x) do { if ((x) != hipSuccess) return 1; } while (0)
#define NOK(x) do { if ((x) != ncclSuccess) return 1; } while (0)

/* one transfer group: slice a's exchange (a >= 0) and slice d's
 * distribution (d >= 0) with every peer */
static int group(ctx_t *c, int a, int d, int rccl)
{
    int s;
    if (!rccl) return hipMemsetAsync(c->scratch, a + d, 64, c->st) != hipSuccess;
    NOK(ncclGroupStart());
    for (s = 0; s < c->p; s++) {
        if (s == c->rank) continue;
        if (a >= 0) {
            NOK(ncclSend(c->send + ((size_t)a * c->p + s) * SLICE_BYTES, SLICE_BYTES, ncclChar, s, c->comm, c->st));
            NOK(ncclRecv(c->recv + ((size_t)a * c->p + s) * SLICE_BYTES, SLICE_BYTES, ncclChar, s, c->comm, c->st));
        }
        if (d >= 0) {
            NOK(ncclSend(c->send + ((size_t)(MAXS + d) * c->p + s) * SLICE_BYTES, SLICE_BYTES, ncclChar, s, c->comm, c->st));
            NOK(ncclRecv(c->recv + ((size_t)(MAXS + d) * c->p + s) * SLICE_BYTES, SLICE_BYTES, ncclChar, s, c->comm, c->st));
        }
    }
    NOK(ncclGroupEnd());
    return 0;
}

/* round 4's PIPE for S slices: slice t's exchange, a fork per slice to the
 * combine stream, one join and one distribution group */
static int issue_fork(ctx_t *c, int S, int rccl)
{
    int t, s;
    for (t = 0; t < S; t++) {
        if (group(c, t, -1, rccl)) return 1;
        OK(hipEventRecord(c->fe[t & 1], c->st));
        OK(hipStreamWaitEvent(c->s2, c->fe[t & 1], 0));
        OK(hipMemsetAsync(c->scratch + 4096 * (1 + (t & 1)), t, 4096, c->s2));
    }
    OK(hipEventRecord(c->je[0], c->s2));
    OK(hipStreamWaitEvent(c->st, c->je[0], 0));
    if (!rccl) return group(c, -1, 0, 0);
    NOK(ncclGroupStart());
    for (s = 0; s < c->p; s++) {
        if (s == c->rank) continue;
        NOK(ncclSend(c->send + ((size_t)MAXS * c->p + s) * SLICE_BYTES, (size_t)S * SLICE_BYTES, ncclChar, s, c->comm, c->st));
        NOK(ncclRecv(c->recv + ((size_t)MAXS * c->p + s) * SLICE_BYTES, (size_t)S * SLICE_BYTES, ncclChar, s, c->comm, c->st));
    }
    NOK(ncclGroupEnd());
    return 0;
}

/* PIPE's shape for S slices (S == 1: P2P's exchange, combine, distribution
 * on one stream); shape 1: issue_fork */
static int issue(ctx_t *c, int S, int rccl, int shape)
{
    int t;
    if (shape && S > 1) return issue_fork(c, S, rccl);
    if (S == 1) {
        if (group(c, 0, -1, rccl)) return 1;
        OK(hipMemsetAsync(c->scratch + 4096, 0, 4096, c->st));
        return group(c, -1, 0, rccl);
    }
    for (t = 0; t < S + 2; t++) {
        if (t >= 2) OK(hipStreamWaitEvent(c->st, c->je[t & 1], 0));
        if (group(c, t < S ? t : -1, t >= 2 ? t - 2 : -1, rccl)) return 1;
        if (t >= S) continue;
        OK(hipEventRecord(c->fe[t & 1], c->st));
        OK(hipStreamWaitEvent(c->s2, c->fe[t & 1], 0));
        OK(hipMemsetAsync(c->scratch + 4096 * (1 + (t & 1)), t, 4096, c->s2));
        OK(hipEventRecord(c->je[t & 1], c->s2));
    }
    return 0;
}

static int row(ctx_t *c, int S, int rccl, int shape)
{
    double e[REPS], g[REPS], t0, b2b;
    int i, k, nk[hipGraphNodeTypeCount];
    size_t nn = 0;
    hipGraph_t gr;
    hipGraphExec_t x;
    hipGraphNode_t *nodes;
    for (i = 0; i < REPS + 2; i++) {            /* the first two open connections */
        OK(hipDeviceSynchronize());
        t0 = now_us();
        if (issue(c, S, rccl, shape)) return 1;
        if (i >= 2) e[i - 2] = now_us() - t0;
    }
    OK(hipDeviceSynchronize());
    OK(hipStreamBeginCapture(c->st, hipStreamCaptureModeThreadLocal));
    if (issue(c, S, rccl, shape)) return 1;
    OK(hipStreamEndCapture(c->st, &gr));
    OK(hipGraphInstantiate(&x, gr, NULL, NULL, 0));
    OK(hipGraphGetNodes(gr, NULL, &nn));
    nodes = (hipGraphNode_t *)calloc(nn ? nn : 1, sizeof *nodes);
    OK(hipGraphGetNodes(gr, nodes, &nn));
    memset(nk, 0, sizeof nk);
    for (i = 0; i < (int)nn; i++) {
        hipGraphNodeType ty;
        OK(hipGraphNodeGetType(nodes[i], &ty));
        if ((int)ty >= 0 && ty < hipGraphNodeTypeCount) nk[ty]++;
    }
    free(nodes);
    for (i = 0; i < REPS + 1; i++) {
        OK(hipDeviceSynchronize());
        t0 = now_us();
        OK(hipGraphLaunch(x, c->st));
        if (i >= 1) g[i - 1] = now_us() - t0;
    }
    OK(hipDeviceSynchronize());
    t0 = now_us();
    for (i = 0; i < REPS; i++) OK(hipGraphLaunch(x, c->st));
    b2b = (now_us() - t0) / REPS;
    OK(hipDeviceSynchronize());
    hipGraphExecDestroy(x);
    hipGraphDestroy(gr);
    if (c->rank == 0) {
        printf("{\"p\": %d, \"shape\": \"%s\", \"slices\": %d, \"rccl\": %s, \"eager_issue_us\": %.1f, "
               "\"graph_launch_us\": %.1f, \"graph_launch_back_to_back_us\": %.1f, \"nodes\": {",
               c->p, shape ? "fork per slice, one join" : "join per slice", S, rccl ? "true" : "false", median(e, REPS), median(g, REPS), b2b);
        static const char *nm[] = {"kernel", "memcpy", "memset", "host", "graph", "empty", "wait_event",
                                   "event_record", "sem_signal", "sem_wait", "mem_alloc", "mem_free",
                                   "memcpy_from_symbol", "memcpy_to_symbol", "batch_mem_op"};
        for (i = 0, k = 0; i < hipGraphNodeTypeCount && i < 15; i++)
            if (nk[i]) printf("%s\"%s\": %d", k++ ? ", " : "", nm[i], nk[i]);
        printf("}}\n");
        fflush(stdout);
    }
    return 0;
}

static int run(int rank, int p, ncclUniqueId id)
{
    static const int SL[] = {1, 2, 4, 8};
    ctx_t c;
    int i, rccl, shape;
    const size_t bytes = (size_t)2 * MAXS * p * SLICE_BYTES;
    memset(&c, 0, sizeof c);
    c.rank = rank;
    c.p = p;
    OK(hipSetDevice(0));
    OK(hipStreamCreateWithFlags(&c.st, hipStreamNonBlocking));
    OK(hipStreamCreateWithFlags(&c.s2, hipStreamNonBlocking));
    for (i = 0; i < 2; i++) {
        OK(hipEventCreateWithFlags(&c.fe[i], hipEventDisableTiming));
        OK(hipEventCreateWithFlags(&c.je[i], hipEventDisableTiming));
    }
    OK(hipMalloc((void **)&c.send, bytes));
    OK(hipMalloc((void **)&c.recv, bytes));
    OK(hipMalloc((void **)&c.scratch, 4 << 20));
    OK(hipMemset(c.send, rank, bytes));
    NOK(ncclCommInitRank(&c.comm, p, id, rank));
    for (shape = 0; shape < 2; shape++)
        for (rccl = 1; rccl >= 0; rccl--)
            for (i = shape ? 1 : 0; i < 4; i++)
                if (row(&c, SL[i], rccl, shape)) {
                fprintf(stderr, "rank %d: row slices %d rccl %d failed\n", rank, SL[i], rccl);
                return 1;
            }
    OK(hipDeviceSynchronize());
    ncclCommDestroy(c.comm);
    return 0;
}

int main(int argc, char **argv)
{
    ncclUniqueId id;
    int p = argc > 1 ? atoi(argv[1]) : 8, fd[2], r, rc = 0, status;
    pid_t kid[64];
    if (p < 2 || p > 16) return 2;
    setenv("NCCL_SOCKET_IFNAME", "lo", 0);
    setenv("NCCL_IB_DISABLE", "1", 0);
    if (pipe(fd)) return 1;
    for (r = 0; r < p; r++) {
        kid[r] = fork();
        if (kid[r] == 0) {
            char hid[32];
            int k;
            snprintf(hid, sizeof hid, "cost-rank-%d", r);
            setenv("NCCL_HOSTID", hid, 1);
            if (r == 0) {
                close(fd[0]);
                if (ncclGetUniqueId(&id) != ncclSuccess) _exit(1);
                for (k = 1; k < p; k++)
                    if (write(fd[1], &id, sizeof id) != sizeof id) _exit(1);
            } else {
                close(fd[1]);
                if (read(fd[0], &id, sizeof id) != sizeof id) _exit(1);
            }
            _exit(run(r, p, id));
        }
    }
    close(fd[0]);
    close(fd[1]);
    for (r = 0; r < p; r++) {
        waitpid(kid[r], &status, 0);
        if (!WIFEXITED(status) || WEXITSTATUS(status)) {
            fprintf(stderr, "rank %d: %s %d\n", r, WIFSIGNALED(status) ? "signal" : "exit",
                    WIFSIGNALED(status) ? WTERMSIG(status) : WEXITSTATUS(status));
            rc = 1;
        }
    }
    return rc;
}
