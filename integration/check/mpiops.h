/* COMPILE-CHECK ONLY (integration/check/README.md): include/mpiops.h:4-9 */
#ifndef CHECK_MPIOPS_H
#define CHECK_MPIOPS_H
struct MPIR_OP {
    MPI_User_function *op;
    unsigned long cookie;
    int commute;
    int permanent;
};
#endif
