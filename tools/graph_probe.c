/*
 * graph_probe.c -- does RCCL's grouped send / receive survive HIP stream
 * capture, instantiation and replay here?  Two processes (forked before any
 * HIP call) share the box's one GPU as two "hosts" (NCCL_HOSTID, RCCL's
 * socket transport, as transport.rccl_net_env), exchange a buffer eagerly,
 * then capture the same exchange into a graph, launch it three times and
 * check the bytes after each launch.  Prints one line per step, so a crash
 * names the step it happened in.
 *
 *   gcc -O2 -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include tools/graph_probe.c \
 *       -o tools/graph_probe -L/opt/rocm/lib -lrccl -lamdhip64
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/wait.h>
#include <unistd.h>

#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#define N (1 << 20)
#define CHK(x, what)                                                               \
    do {                                                                           \
        if (!(x)) {                                                                \
            fprintf(stderr, "rank %d: %s failed\n", rank, what);                   \
            return 1;                                                              \
        }                                                                          \
    } while (0)

static int step(int rank, const char *s)
{
    fprintf(stderr, "rank %d: %s\n", rank, s);
    return 0;
}

static int exchange(ncclComm_t comm, int rank, const int *send, int *recv, hipStream_t st)
{
    if (ncclGroupStart() != ncclSuccess) return 1;
    if (ncclSend(send, N, ncclInt32, 1 - rank, comm, st) != ncclSuccess) return 1;
    if (ncclRecv(recv, N, ncclInt32, 1 - rank, comm, st) != ncclSuccess) return 1;
    return ncclGroupEnd() != ncclSuccess;
}

/* two sends and two receives with the same peer in one group, as PIPE's
 * step t carries slice t's exchange and slice t - 2's distribution */
static int exchange2(ncclComm_t comm, int rank, const int *send, int *recv, hipStream_t st)
{
    if (ncclGroupStart() != ncclSuccess) return 1;
    if (ncclSend(send, N / 2, ncclInt32, 1 - rank, comm, st) != ncclSuccess) return 1;
    if (ncclRecv(recv, N / 2, ncclInt32, 1 - rank, comm, st) != ncclSuccess) return 1;
    if (ncclSend(send + N / 2, N / 2, ncclInt32, 1 - rank, comm, st) != ncclSuccess) return 1;
    if (ncclRecv(recv + N / 2, N / 2, ncclInt32, 1 - rank, comm, st) != ncclSuccess) return 1;
    return ncclGroupEnd() != ncclSuccess;
}

static int check(int rank, int *recv, int *host, int tag)
{
    int i;
    if (hipMemcpy(host, recv, N * sizeof(int), hipMemcpyDeviceToHost) != hipSuccess) return 1;
    for (i = 0; i < N; i++)
        if (host[i] != (1 - rank) * 1000003 + i) {
            fprintf(stderr, "rank %d: %d: recv[%d] = %d\n", rank, tag, i, host[i]);
            return 1;
        }
    return 0;
}

static int run(int rank, ncclUniqueId id)
{
    ncclComm_t comm;
    hipStream_t st;
    hipGraph_t g;
    hipGraphExec_t x;
    int *send, *recv, *host, i;
    CHK(hipSetDevice(0) == hipSuccess, "hipSetDevice");
    CHK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking) == hipSuccess, "stream");
    CHK(hipMalloc((void **)&send, N * sizeof(int)) == hipSuccess, "malloc");
    CHK(hipMalloc((void **)&recv, N * sizeof(int)) == hipSuccess, "malloc");
    host = (int *)malloc(N * sizeof(int));
    for (i = 0; i < N; i++) host[i] = rank * 1000003 + i;
    CHK(hipMemcpy(send, host, N * sizeof(int), hipMemcpyHostToDevice) == hipSuccess, "h2d");
    step(rank, "init");
    CHK(ncclCommInitRank(&comm, 2, id, rank) == ncclSuccess, "ncclCommInitRank");
    step(rank, "eager exchange");
    CHK(exchange(comm, rank, send, recv, st) == 0, "eager exchange");
    CHK(hipStreamSynchronize(st) == hipSuccess, "eager sync");
    CHK(check(rank, recv, host, -1) == 0, "eager result");
    step(rank, "capture");
    CHK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal) == hipSuccess, "begin capture");
    CHK(hipMemsetAsync(recv, 0, N * sizeof(int), st) == hipSuccess, "memset in capture");
    CHK(exchange(comm, rank, send, recv, st) == 0, "captured exchange");
    CHK(hipStreamEndCapture(st, &g) == hipSuccess, "end capture");
    step(rank, "instantiate");
    CHK(hipGraphInstantiate(&x, g, NULL, NULL, 0) == hipSuccess, "instantiate");
    for (i = 0; i < 3; i++) {
        step(rank, "launch");
        CHK(hipGraphLaunch(x, st) == hipSuccess, "launch");
        CHK(hipStreamSynchronize(st) == hipSuccess, "launch sync");
        CHK(check(rank, recv, host, i) == 0, "replayed result");
    }
    hipGraphExecDestroy(x);
    hipGraphDestroy(g);
    /* fork / join across two streams inside the capture, as the PIPE
     * variant does: (a) without RCCL, (b) with RCCL groups on the capturing
     * stream and work on the joined stream between them */
    {
        hipStream_t s2;
        hipEvent_t ev[4];
        int mode;
        CHK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking) == hipSuccess, "stream 2");
        for (i = 0; i < 4; i++) CHK(hipEventCreateWithFlags(&ev[i], hipEventDisableTiming) == hipSuccess, "event");
        for (mode = 0; mode < 6; mode++) {
            int t;
            static const char *name[] = {"fork-join capture, no RCCL", "fork-join capture with RCCL",
                                         "pipe-shaped capture, events reused", "pipe-shaped capture, fresh events",
                                         "two transfers per peer per group, one stream",
                                         "pipe-shaped, two transfers per peer per group"};
            step(rank, name[mode]);
            CHK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal) == hipSuccess, "begin capture 2");
            if (mode < 2) {
                if (mode) CHK(exchange(comm, rank, send, recv, st) == 0, "captured exchange 2a");
                else CHK(hipMemsetAsync(recv, 1, N * sizeof(int), st) == hipSuccess, "memset a");
                CHK(hipEventRecord(ev[0], st) == hipSuccess, "record fork");
                CHK(hipStreamWaitEvent(s2, ev[0], 0) == hipSuccess, "wait fork");
                CHK(hipMemsetAsync(send + N / 2, 0, 4, s2) == hipSuccess, "memset on joined stream");
                CHK(hipEventRecord(ev[1], s2) == hipSuccess, "record join");
                if (mode) CHK(exchange(comm, rank, send, recv, st) == 0, "captured exchange 2b");
                CHK(hipStreamWaitEvent(st, ev[1], 0) == hipSuccess, "wait join");
            } else if (mode == 4) {
                CHK(exchange2(comm, rank, send, recv, st) == 0, "captured double exchange");
                CHK(exchange2(comm, rank, send, recv, st) == 0, "captured double exchange");
            } else {
                /* PIPE's shape: step t exchanges, waits for the work of step
                 * t - 2 on s2, forks step t's work to s2; events of steps t
                 * and t - 2 share a slot (mode 2) or not (mode 3) */
                hipEvent_t fe[8], je[8];
                for (t = 0; t < 8; t++) {
                    if (mode != 3) { fe[t] = ev[t & 1]; je[t] = ev[2 + (t & 1)]; }
                    else {
                        CHK(hipEventCreateWithFlags(&fe[t], hipEventDisableTiming) == hipSuccess, "event");
                        CHK(hipEventCreateWithFlags(&je[t], hipEventDisableTiming) == hipSuccess, "event");
                    }
                }
                for (t = 0; t < 6; t++) {
                    if (t >= 2) CHK(hipStreamWaitEvent(st, je[t - 2], 0) == hipSuccess, "wait join");
                    if (mode == 5 && t >= 2 && t < 4)
                        CHK(exchange2(comm, rank, send, recv, st) == 0, "captured double exchange");
                    else
                        CHK(exchange(comm, rank, send, recv, st) == 0, "captured exchange");
                    if (t < 4) {
                        CHK(hipEventRecord(fe[t], st) == hipSuccess, "record fork");
                        CHK(hipStreamWaitEvent(s2, fe[t], 0) == hipSuccess, "wait fork");
                        CHK(hipMemsetAsync(send + N / 2, 0, 4, s2) == hipSuccess, "memset on joined stream");
                        CHK(hipEventRecord(je[t], s2) == hipSuccess, "record join");
                    }
                }
            }
            CHK(hipStreamEndCapture(st, &g) == hipSuccess, "end capture 2");
            step(rank, "instantiate 2");
            CHK(hipGraphInstantiate(&x, g, NULL, NULL, 0) == hipSuccess, "instantiate 2");
            for (i = 0; i < 3; i++) {
                step(rank, "launch 2");
                CHK(hipGraphLaunch(x, st) == hipSuccess, "launch 2");
                CHK(hipStreamSynchronize(st) == hipSuccess, "launch 2 sync");
            }
            hipGraphExecDestroy(x);
            hipGraphDestroy(g);
        }
    }
    step(rank, "ok");
    ncclCommDestroy(comm);
    return 0;
}

int main(void)
{
    ncclUniqueId id;
    int fd[2], r, rc = 0, status;
    pid_t kid[2];
    setenv("NCCL_SOCKET_IFNAME", "lo", 0);
    setenv("NCCL_IB_DISABLE", "1", 0);
    /* rank 0 makes the id (its process hosts RCCL's bootstrap root) and
     * passes it to rank 1; nothing in this parent touches HIP */
    if (pipe(fd)) return 1;
    for (r = 0; r < 2; r++) {
        kid[r] = fork();
        if (kid[r] == 0) {
            char hid[32];
            snprintf(hid, sizeof hid, "probe-rank-%d", r);
            setenv("NCCL_HOSTID", hid, 1);       /* before this process's first RCCL call */
            if (r == 0) {
                close(fd[0]);
                if (ncclGetUniqueId(&id) != ncclSuccess) _exit(1);
                if (write(fd[1], &id, sizeof id) != sizeof id) _exit(1);
            } else {
                close(fd[1]);
                if (read(fd[0], &id, sizeof id) != sizeof id) _exit(1);
            }
            _exit(run(r, id));
        }
    }
    close(fd[0]);
    close(fd[1]);
    for (r = 0; r < 2; r++) {
        waitpid(kid[r], &status, 0);
        if (!WIFEXITED(status) || WEXITSTATUS(status)) {
            fprintf(stderr, "rank %d: %s %d\n", r, WIFSIGNALED(status) ? "signal" : "exit",
                    WIFSIGNALED(status) ? WTERMSIG(status) : WEXITSTATUS(status));
            rc = 1;
        }
    }
    printf("graph_probe: %s\n", rc ? "FAILED" : "ok");
    return rc;
}
