/* lat_probe.c -- per-call latency of small device-buffer calls from C,
 * against the floor of a bare HIP launch + stream synchronisation:
 *   hipMemcpyAsync(D2D, 8 B) + sync, MPIR_SUM via mvx_op_apply + sync,
 *   MPI_Allreduce / MPI_Reduce on a 1-rank RCCL communicator (blocking),
 *   and the same Allreduce on a 4-rank virtual communicator.
 * Build: see tools/gpu_round.sh (stage lat). */
#include <stdio.h>
#include <stdlib.h>
#include <time.h>
#include <hip/hip_runtime_api.h>
#include "mvx_coll.h"
#include "mvx_hip.h"

static double now(void)
{
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + 1e-9 * t.tv_nsec;
}

#define REPS 20000
#define TIME(label, body) do {                                             \
        int i_; double t0_;                                                \
        for (i_ = 0; i_ < 200; i_++) { body; }                             \
        t0_ = now();                                                       \
        for (i_ = 0; i_ < REPS; i_++) { body; }                            \
        printf("{\"probe\": \"%s\", \"n\": %d, \"us_per_call\": %.2f}\n", \
               label, n, (now() - t0_) / REPS * 1e6);                      \
    } while (0)

int main(void)
{
    char id[MVX_UNIQUE_ID_BYTES];
    MPI_Comm comm, vcomm;
    float *a, *b, *va[4], *vb[4];
    int rcs[4], n, i;
    if (hipSetDevice(0) != hipSuccess) return 1;
    if (mvx_get_unique_id(id) || mvx_comm_init(&comm, 0, 1, 0, id)) return 2;
    if (mvx_comm_init_local(&vcomm, 4, 0)) return 3;
    if (hipMalloc((void **)&a, 1 << 24) || hipMalloc((void **)&b, 1 << 24)) return 4;
    for (i = 0; i < 4; i++)
        if (hipMalloc((void **)&va[i], 1 << 20) || hipMalloc((void **)&vb[i], 1 << 20)) return 5;
    hipMemset(a, 0, 1 << 24);
    hipMemset(b, 0, 1 << 24);
    for (n = 2; n <= 65536; n *= 32) {
        TIME("hipMemcpyAsync+sync (floor)", { hipMemcpyAsync(b, a, n * 4, hipMemcpyDeviceToDevice, 0); hipStreamSynchronize(0); });
        TIME("mvx_op_apply SUM f32 + sync", { mvx_op_apply(MPI_SUM, MPI_FLOAT, a, b, n, 0); hipStreamSynchronize(0); });
        TIME("MPI_Allreduce p=1 (RCCL comm)", { MPI_Allreduce(a, b, n, MPI_FLOAT, MPI_SUM, comm); });
        TIME("MPI_Reduce p=1 (RCCL comm)", { MPI_Reduce(a, b, n, MPI_FLOAT, MPI_SUM, 0, comm); });
        TIME("Allreduce p=4 virtual", { mvx_allreduce_multi((void *const *)va, (void *const *)vb, n < 65536 ? n : 65536, MPI_FLOAT, MPI_SUM, vcomm, rcs, NULL); hipStreamSynchronize(0); });
    }
    mvx_comm_free(&vcomm);
    mvx_comm_free(&comm);
    return 0;
}
