/* TEST HELPER: an MPI program in C against libmvx.so alone -- what a user
 * of the reference compiles when switching (include/mvx_coll.h; INTEGRATION.md
 * section 1).  One process, one GPU: a 1-rank RCCL world for the blocking MPI
 * calls on device and host buffers, and a 4-rank virtual communicator for
 * answers that depend on several ranks.  Known answers are computed here.
 * Exit status 0 = every check passed; prints the first failure otherwise. */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <hip/hip_runtime_api.h>
#include "mvx_coll.h"

#define N 4099
#define CHECK(c, ...) do { if (!(c)) { printf("FAIL %s:%d ", __FILE__, __LINE__); printf(__VA_ARGS__); printf("\n"); return 1; } } while (0)

static void my_prod(void *in, void *inout, int *len, MPI_Datatype *dt)   /* a user op, like coll9.c's addem */
{
    int i, *a = (int *)in, *b = (int *)inout;
    (void)dt;
    for (i = 0; i < *len; i++) b[i] = a[i] * b[i];
}

int main(void)
{
    char id[MVX_UNIQUE_ID_BYTES];
    MPI_Comm world, v4;
    int i, q, rcs[4], *hs, *hr, *ds, *dr, *vs[4], *vr[4];
    float *fs, *fr;
    MPI_Op op;
    hipSetDevice(0);
    CHECK(mvx_get_unique_id(id) == 0 && mvx_comm_init(&world, 0, 1, 0, id) == 0, "world");
    CHECK(world == MPI_COMM_WORLD, "first communicator is MPI_COMM_WORLD");
    hs = (int *)malloc(N * sizeof(int));
    hr = (int *)malloc(N * sizeof(int));
    for (i = 0; i < N; i++) hs[i] = i - 2000;
    /* host buffers: p = 1 Allreduce / Reduce / Scan are the input itself */
    CHECK(MPI_Allreduce(hs, hr, N, MPI_INT, MPI_SUM, MPI_COMM_WORLD) == MPI_SUCCESS, "allreduce");
    CHECK(memcmp(hs, hr, N * sizeof(int)) == 0, "allreduce p=1");
    memset(hr, 0, N * sizeof(int));
    CHECK(MPI_Reduce(hs, hr, N, MPI_INT, MPI_MAX, 0, MPI_COMM_WORLD) == MPI_SUCCESS, "reduce");
    CHECK(memcmp(hs, hr, N * sizeof(int)) == 0, "reduce p=1");
    memset(hr, 0, N * sizeof(int));
    CHECK(MPI_Scan(hs, hr, N, MPI_INT, MPI_MIN, MPI_COMM_WORLD) == MPI_SUCCESS, "scan");
    CHECK(memcmp(hs, hr, N * sizeof(int)) == 0, "scan p=1");
    /* the reference's error codes */
    CHECK(MPI_Allreduce(hs, hs, N, MPI_INT, MPI_SUM, MPI_COMM_WORLD) % 64 == MPI_ERR_BUFFER, "alias");
    CHECK(MPI_Allreduce(hs, hr, -1, MPI_INT, MPI_SUM, MPI_COMM_WORLD) % 64 == MPI_ERR_COUNT, "count");
    /* BAND on FLOAT at p = 1: no rank calls (*uop), so no error (intra_fns_new.c) */
    CHECK(MPI_Allreduce(hs, hr, N, MPI_FLOAT, MPI_BAND, MPI_COMM_WORLD) == MPI_SUCCESS, "BAND on FLOAT, p = 1");
    /* device buffers */
    CHECK(hipMalloc((void **)&ds, N * sizeof(int)) == hipSuccess && hipMalloc((void **)&dr, N * sizeof(int)) == hipSuccess, "hipMalloc");
    hipMemcpy(ds, hs, N * sizeof(int), hipMemcpyHostToDevice);
    CHECK(MPI_Allreduce(ds, dr, N, MPI_INT, MPI_SUM, MPI_COMM_WORLD) == MPI_SUCCESS, "device allreduce");
    hipMemcpy(hr, dr, N * sizeof(int), hipMemcpyDeviceToHost);
    CHECK(memcmp(hs, hr, N * sizeof(int)) == 0, "device allreduce p=1");
    /* a 4-rank virtual communicator: rank q holds q + 1 + i */
    CHECK(mvx_comm_init_local(&v4, 4, 0) == 0, "virtual comm");
    for (q = 0; q < 4; q++) {
        CHECK(hipMalloc((void **)&vs[q], N * sizeof(int)) == hipSuccess && hipMalloc((void **)&vr[q], N * sizeof(int)) == hipSuccess, "hipMalloc v");
        for (i = 0; i < N; i++) hs[i] = q + 1 + (i % 7);
        hipMemcpy(vs[q], hs, N * sizeof(int), hipMemcpyHostToDevice);
    }
    CHECK(mvx_allreduce_multi((void *const *)vs, (void *const *)vr, N, MPI_INT, MPI_SUM, v4, rcs, NULL) == 0, "multi");
    hipDeviceSynchronize();
    for (q = 0; q < 4; q++) {
        CHECK(rcs[q] == 0, "rank %d rc %d", q, rcs[q]);
        hipMemcpy(hr, vr[q], N * sizeof(int), hipMemcpyDeviceToHost);
        for (i = 0; i < N; i++) CHECK(hr[i] == 10 + 4 * (i % 7), "sum rank %d elem %d: %d", q, i, hr[i]);
    }
    /* BAND on FLOAT at p = 4: 329 on every rank that calls (*uop) -- all four */
    CHECK(mvx_allreduce_multi((void *const *)vs, (void *const *)vr, 64, MPI_FLOAT, MPI_BAND, v4, rcs, NULL) == 0, "band");
    for (q = 0; q < 4; q++) CHECK(rcs[q] == 329, "BAND on FLOAT rank %d: %d", q, rcs[q]);
    /* a user op (MPI_Op_create), run on the host in the reference's roles */
    CHECK(MPI_Op_create(my_prod, 1, &op) == MPI_SUCCESS, "op_create");
    CHECK(mvx_allreduce_multi((void *const *)vs, (void *const *)vr, N, MPI_INT, op, v4, rcs, NULL) == 0, "user op");
    hipDeviceSynchronize();
    for (q = 0; q < 4; q++) {
        hipMemcpy(hr, vr[q], N * sizeof(int), hipMemcpyDeviceToHost);
        for (i = 0; i < N; i++) {
            const int k = i % 7;
            CHECK(hr[i] == (1 + k) * (2 + k) * (3 + k) * (4 + k), "prod rank %d elem %d: %d", q, i, hr[i]);
        }
    }
    CHECK(MPI_Op_free(&op) == MPI_SUCCESS && op == MPI_OP_NULL, "op_free");
    /* MAXLOC on MPI_FLOAT_INT from host buffers: value ties keep the smaller loc */
    fs = (float *)malloc(2 * N * sizeof(float));
    fr = (float *)malloc(2 * N * sizeof(float));
    for (i = 0; i < N; i++) { fs[2 * i] = (float)(i % 5); ((int *)fs)[2 * i + 1] = i; }
    CHECK(MPI_Allreduce(fs, fr, N, MPI_FLOAT_INT, MPI_MAXLOC, MPI_COMM_WORLD) == MPI_SUCCESS, "maxloc");
    CHECK(memcmp(fs, fr, 2 * N * sizeof(float)) == 0, "maxloc p=1");
    for (q = 0; q < 4; q++) { hipFree(vs[q]); hipFree(vr[q]); }
    hipFree(ds); hipFree(dr);
    mvx_comm_free(&v4);
    mvx_comm_free(&world);
    free(hs); free(hr); free(fs); free(fr);
    printf("c_app ok\n");
    return 0;
}
