/*
 * graph_app.c -- the PIPE variant's HIP-graph capture through libmvx.so from
 * C, outside Python: two processes (forked before any HIP call) on the box's
 * one GPU as an RCCL communicator over its socket transport (NCCL_HOSTID per
 * rank, as transport.rccl_net_env), graphs on, each exchange variant, an
 * Allreduce(SUM, INT) run three times on the same buffers (eager, captured,
 * replayed), blocking and stream-ordered, every result checked.  Linked
 * against the image's ROCm (/opt/rocm: HIP and RCCL), where the Python tests
 * run on torch's bundled copies -- so a failure only one of them shows points
 * at the runtime, not at the library.
 *
 *   gcc -O2 -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -Iinclude tools/graph_app.c -o tools/graph_app \
 *       -Lmvapich-cce_amd -lmvx -L/opt/rocm/lib -lamdhip64 -Wl,-rpath,$PWD/mvapich-cce_amd -Wl,-rpath,/opt/rocm/lib
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/wait.h>
#include <unistd.h>

#include <hip/hip_runtime_api.h>

#include "mvx_coll.h"

#define N 300000           /* the largest job */
/* job sizes: the first only by default; MVX_APP_SIZES=k runs k of them
 * (more distinct jobs: with MVX_GRAPH_CACHE small, more evictions) */
static const int g_sizes[] = {70001, 32768, 300000, 4096 * 8, 140001, 1000};

static int run(int rank, const char *id)
{
    MPI_Comm c;
    hipStream_t st;
    int *ds, *dr, *h, i, v, rep, via, st_g, err, z, nz = 1, n;
    const char *e = getenv("MVX_APP_SIZES");
    static const int modes[3][2] = {{MVX_EXCH_P2P, 0}, {MVX_EXCH_PIPE, 3}, {MVX_EXCH_COLL, 0}};
    if (hipSetDevice(0) != hipSuccess || hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) return 1;
    if (mvx_comm_init(&c, rank, 2, 0, id)) { fprintf(stderr, "rank %d: init\n", rank); return 1; }
    h = (int *)malloc(N * sizeof(int));
    hipMalloc((void **)&ds, N * sizeof(int));
    hipMalloc((void **)&dr, N * sizeof(int));
    for (i = 0; i < N; i++) h[i] = rank * 1000 + i % 977;
    hipMemcpy(ds, h, N * sizeof(int), hipMemcpyHostToDevice);
    if (e && atoi(e) > 1) nz = atoi(e) < 6 ? atoi(e) : 6;
    mvx_comm_set_graphs(c, 1);
    for (z = 0; z < nz; z++)
    for (v = 0; v < 3; v++) {
        n = g_sizes[z];
        mvx_comm_set_exchange(c, modes[v][0], modes[v][1]);
        for (via = 0; via < 2; via++)
            for (rep = 0; rep < 3; rep++) {
                hipMemset(dr, 0, N * sizeof(int));
                fprintf(stderr, "rank %d: n %d variant %d %s rep %d\n", rank, n, v, via ? "stream" : "blocking", rep);
                if (via == 0) {
                    if (MPI_Allreduce(ds, dr, n, MPI_INT, MPI_SUM, c)) return 1;
                } else {
                    if (mvx_allreduce_async(ds, dr, n, MPI_INT, MPI_SUM, c, st) || hipStreamSynchronize(st))
                        return 1;
                }
                mvx_comm_last_graph(c, &st_g, &err);
                hipMemcpy(h, dr, N * sizeof(int), hipMemcpyDeviceToHost);
                for (i = 0; i < n; i++)
                    if (h[i] != 1000 + 2 * (i % 977)) {
                        fprintf(stderr, "rank %d: wrong result at %d: %d\n", rank, i, h[i]);
                        return 1;
                    }
                fprintf(stderr, "rank %d:   ok, graph state %d error %d\n", rank, st_g, err);
            }
    }
    mvx_comm_free(&c);
    return 0;
}

int main(void)
{
    char id[MVX_UNIQUE_ID_BYTES];
    int fd[2], r, rc = 0, status;
    pid_t kid[2];
    setenv("NCCL_SOCKET_IFNAME", "lo", 0);
    setenv("NCCL_IB_DISABLE", "1", 0);
    if (pipe(fd)) return 1;
    for (r = 0; r < 2; r++) {
        kid[r] = fork();
        if (kid[r] == 0) {
            char hid[32];
            snprintf(hid, sizeof hid, "graph-app-rank-%d", r);
            setenv("NCCL_HOSTID", hid, 1);
            if (r == 0) {
                close(fd[0]);
                if (mvx_get_unique_id(id) || write(fd[1], id, sizeof id) != sizeof id) _exit(1);
            } else {
                close(fd[1]);
                if (read(fd[0], id, sizeof id) != sizeof id) _exit(1);
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
    printf("graph_app: %s\n", rc ? "FAILED" : "ok");
    return rc;
}
