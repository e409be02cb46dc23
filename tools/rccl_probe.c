/* Can RCCL run 2 ranks on one GPU in one process?  (test-infrastructure probe) */
#include <stdio.h>
#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>
int main(void)
{
    ncclComm_t comms[2];
    int devs[2] = {0, 0};
    ncclResult_t r = ncclCommInitAll(comms, 2, devs);
    printf("ncclCommInitAll(2 ranks, dev 0): %d %s\n", (int)r, ncclGetErrorString(r));
    if (r != ncclSuccess) return 0;
    float *a, *b; hipStream_t s[2];
    hipSetDevice(0);
    hipMalloc((void **)&a, 1 << 20); hipMalloc((void **)&b, 1 << 20);
    hipMemset(a, 0, 1 << 20); hipMemset(b, 0, 1 << 20);
    hipStreamCreate(&s[0]); hipStreamCreate(&s[1]);
    ncclGroupStart();
    ncclSend(a, 1024, ncclFloat, 1, comms[0], s[0]);
    ncclRecv(b, 1024, ncclFloat, 0, comms[1], s[1]);
    r = ncclGroupEnd();
    printf("group send/recv: %d %s\n", (int)r, ncclGetErrorString(r));
    hipDeviceSynchronize();
    printf("done\n");
    return 0;
}
