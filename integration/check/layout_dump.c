/* TEST INFRASTRUCTURE (integration/check/README.md): prints the offset and
 * size of every struct member integration/intra_mvx.c reads, one
 * "name value" line each, from whichever headers it is compiled against:
 *
 *   (default)    the compile-check headers of this directory
 *   REAL_HEADERS the reference's own include/ and mpid/ch2 headers, ch_shmem
 *                device (mpid.h pulls mpi.h, cookie.h, comm.h, datatype.h)
 *   REAL_GEN2    the same plus the _SMP_ devices' communicator,
 *                mpid/ch_gen2/comm.h (ch_smp / ch_psm / ch_hybrid carry the
 *                same struct), read under renamed tags beside ch2's
 *
 * tests/test_cpu_integration.py compares the lines (ref_layout.py makes the
 * real-header builds; nothing of the reference is copied or built). */
#include <stddef.h>
#include <stdio.h>

#if defined(REAL_HEADERS) || defined(REAL_GEN2)
#include "mpid.h"
#include "mpiops.h"
#include "mpicoll.h"
#else
#include "mpiimpl.h"
#include "mpiops.h"
#include "mpicoll.h"
#endif

#ifdef REAL_GEN2
/* mpid/ch_gen2/comm.h is guarded by the same macro as ch2's comm.h and
 * declares the same names: include it a second time under other tags */
#undef MPIR_GROUP_COOKIE
#define MPIR_GROUP g2_MPIR_GROUP
#define MPIR_Errhandler g2_MPIR_Errhandler
#define MPIR_COMMUNICATOR g2_MPIR_COMMUNICATOR
#define MPIR_INTRA g2_MPIR_INTRA
#define MPIR_INTER g2_MPIR_INTER
#define MPIR_COMM_TYPE g2_MPIR_COMM_TYPE
#define _MPIR_Comm_list g2__MPIR_Comm_list
#define MPIR_Comm_list g2_MPIR_Comm_list
#define MPIR_All_communicators g2_MPIR_All_communicators
#include "ch_gen2/comm.h"
typedef struct g2_MPIR_COMMUNICATOR comm_t;
#else
typedef struct MPIR_COMMUNICATOR comm_t;
#endif

#define OFF(T, m) printf("%s.%s %zu\n", #T, #m, offsetof(T, m))

typedef struct MPIR_DATATYPE dtype_t;
typedef struct MPIR_OP op_t;
typedef struct _MPIR_COLLOPS collops_t;

int main(void)
{
    OFF(comm_t, np);
    OFF(comm_t, local_rank);
    OFF(comm_t, self);
    OFF(comm_t, permanent);
    OFF(comm_t, collops);
#ifdef _SMP_
    OFF(comm_t, leader_comm);
    OFF(comm_t, shmem_coll_ok);
#endif
    printf("sizeof.comm_t %zu\n", sizeof(comm_t));
    OFF(dtype_t, dte_type);
    OFF(dtype_t, permanent);
    OFF(dtype_t, ub);
    OFF(dtype_t, lb);
    OFF(dtype_t, extent);
    OFF(dtype_t, size);
    OFF(dtype_t, count);
    OFF(dtype_t, stride);
    OFF(dtype_t, indices);
    OFF(dtype_t, blocklen);
    OFF(dtype_t, blocklens);
    OFF(dtype_t, old_type);
    OFF(dtype_t, old_types);
    OFF(dtype_t, self);
    printf("sizeof.dtype_t %zu\n", sizeof(dtype_t));
    OFF(op_t, op);
    OFF(op_t, commute);
    OFF(op_t, permanent);
    printf("sizeof.op_t %zu\n", sizeof(op_t));
    OFF(collops_t, Bcast);
    OFF(collops_t, Reduce);
    OFF(collops_t, Allreduce);
    OFF(collops_t, Reduce_scatter);
    OFF(collops_t, Scan);
    OFF(collops_t, ref_count);
    printf("sizeof.collops_t %zu\n", sizeof(collops_t));
    return 0;
}
