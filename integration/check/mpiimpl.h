/* COMPILE-CHECK ONLY (integration/check/README.md): the declarations of the
 * reference's mpi.h / mpiimpl.h / mpid/ch2/{comm,datatype}.h that
 * integration/intra_mvx.c uses, spelled as there.  Not the reference. */
#ifndef CHECK_MPIIMPL_H
#define CHECK_MPIIMPL_H

typedef int MPI_Datatype;                      /* mpi.h:29 */
typedef int MPI_Comm;
typedef int MPI_Op;
typedef long MPI_Aint;                         /* mpidefs.h.in (@MPI_AINT@, long on LP64) */
typedef int MPI_Fint;                          /* mpidefs.h.in:9 */

#define MPI_SUCCESS        0                   /* mpi_errno.h:22 */
#define MPI_ERR_TYPE       3                   /* :26 */
#define MPI_ERR_OP         9                   /* :35 */
#define MPI_ERR_OTHER     15                   /* :46 */
#define MPI_ERR_INTERN    16
#define MPI_ERR_EXHAUSTED (MPI_ERR_INTERN | (1 << 6))   /* mpi_error.h:249 */

#define MPI_BYTE          ((MPI_Datatype)3)    /* mpi.h:67 */
#define MPI_INT           ((MPI_Datatype)6)    /* mpi.h:70 */
#define MPI_MAX           (MPI_Op)(100)        /* mpi.h:129 */
#define MPI_MIN           (MPI_Op)(101)        /* mpi.h:130 */
#define MPI_MAXLOC        (MPI_Op)(111)        /* mpi.h:140 */
#define MPI_KEYVAL_INVALID 0                   /* mpi.h:170 */

typedef void (MPI_User_function)(void *, void *, int *, MPI_Datatype *);       /* mpi.h:206 */
typedef int (MPI_Copy_function)(MPI_Comm, int, void *, void *, void *, int *); /* :209 */
typedef int (MPI_Delete_function)(MPI_Comm, int, void *, void *);              /* :210 */
int MPIR_null_copy_fn(MPI_Comm, int, void *, void *, void *, int *);
#define MPI_NULL_COPY_FN MPIR_null_copy_fn                                      /* :194 */
int MPI_Keyval_create(MPI_Copy_function *, MPI_Delete_function *, int *, void *); /* :431 */
int MPI_Attr_put(MPI_Comm, int, void *);                                        /* :433 */
int MPI_Attr_get(MPI_Comm, int, void *, int *);                                 /* :434 */

typedef enum {                                 /* mpid/ch2/datatype.h:15-23 */
    MPIR_INT, MPIR_FLOAT, MPIR_DOUBLE, MPIR_COMPLEX, MPIR_LONG, MPIR_SHORT,
    MPIR_CHAR, MPIR_BYTE, MPIR_UCHAR, MPIR_USHORT, MPIR_ULONG, MPIR_UINT,
    MPIR_CONTIG, MPIR_VECTOR, MPIR_HVECTOR, MPIR_INDEXED,
    MPIR_HINDEXED, MPIR_STRUCT, MPIR_DOUBLE_COMPLEX, MPIR_PACKED,
    MPIR_UB, MPIR_LB, MPIR_LONGDOUBLE, MPIR_LONGLONGINT,
    MPIR_LOGICAL, MPIR_FORT_INT, MPIR_ULONGLONG
} MPIR_NODETYPE;

struct MPIR_DATATYPE {                         /* mpid/ch2/datatype.h:26-56 */
    MPIR_NODETYPE dte_type;
    unsigned long cookie;
    int committed, is_contig, basic, permanent;
    MPI_Aint ub, lb, real_ub, real_lb;
    int has_ub, has_lb;
    MPI_Aint extent;
    int size, elements, ref_count, align, count;
    MPI_Aint stride;
    MPI_Aint *indices;
    int blocklen;
    int *blocklens;
    struct MPIR_DATATYPE *old_type, **old_types, *flattened;
    MPI_Datatype self;
};

typedef struct _MPIR_COLLOPS *MPIR_COLLOPS;    /* mpid/ch2/comm.h:49 */

struct MPIR_COMMUNICATOR {                     /* mpid/ch2/comm.h:65-113 */
    unsigned long cookie;
    int np;
    int local_rank;
    int *lrank_to_grank;
    int send_context, recv_context;
    void *ADIctx;
    int comm_type;
    void *group, *local_group;
    struct MPIR_COMMUNICATOR *comm_coll;
    int self;
    int ref_count;
    void *comm_cache, *attr_cache;
    int use_return_handler;
    int error_handler;
    int permanent;
#ifdef _SMP_
    void *mutex;                               /* mpid/ch_gen2/comm.h:121 (ch2: an empty
                                                  MPID_THREAD_DS_LOCK_DECLARE, ch2/mpid.h:56) */
#endif
    int msgform;
    void *adiCollCtx;
    MPIR_COLLOPS collops;
    struct MPIR_COMMUNICATOR *comm_next;
    char *comm_name;
#ifdef _SMP_                                   /* mpid/ch_gen2/comm.h:139-181 (ch_smp, ch_psm and
                                                  ch_hybrid declare the same members) */
    struct Collbuf *collbuf;
    unsigned int is_mcast_enabled, is_alltoall_enabled, is_barrier_enabled, is_allgather_enabled;
    int rdma_barrier_id;
    int togle;
    MPI_Comm leader_comm, shmem_comm, parent_comm;
    int parent;
    int *leader_map, *leader_rank;
    int shmem_comm_rank, shmem_coll_ok, leader_group_size;
    int bcast_fd, bcast_index;
    void *bcast_mmap_ptr;
    char *bcast_shmem_file;
    int bcast_seg_size, allg_cyclic_ok;
    int new_group;                             /* MPI_Group */
    MPI_Comm new_comm;
    int *new_ranks;
#endif
};

void *MPIR_ToPointer(int);                     /* mpiimpl.h:329 */
#define MPIR_GET_DTYPE_PTR(idx) (struct MPIR_DATATYPE *)MPIR_ToPointer(idx)      /* datatype.h:60 */
#define MPIR_GET_COMM_PTR(idx) (struct MPIR_COMMUNICATOR *)MPIR_ToPointer(idx)   /* comm.h:126 */
#define MPIR_GET_OP_PTR(op) (struct MPIR_OP *)MPIR_ToPointer(op)                 /* mpiimpl.h:193 */
extern struct MPIR_COMMUNICATOR *MPIR_COMM_WORLD;                                 /* mpiimpl.h:171 */

#endif
