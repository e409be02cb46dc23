/* COMPILE-CHECK ONLY (integration/check/README.md): include/mpicoll.h:8-59,
 * the members intra_mvx.c touches plus placeholders keeping their order */
#ifndef CHECK_MPICOLL_H
#define CHECK_MPICOLL_H
struct _MPIR_COLLOPS {
    int (*Barrier)(struct MPIR_COMMUNICATOR *);
    int (*Bcast)(void *, int, struct MPIR_DATATYPE *, int, struct MPIR_COMMUNICATOR *);
    void *Gather, *Gatherv, *Scatter, *Scatterv, *Allgather, *Allgatherv, *Alltoall,
        *Alltoallv, *Alltoallw;
    int (*Reduce)(void *, void *, int, struct MPIR_DATATYPE *, MPI_Op, int,
                  struct MPIR_COMMUNICATOR *);
    int (*Allreduce)(void *, void *, int, struct MPIR_DATATYPE *, MPI_Op,
                     struct MPIR_COMMUNICATOR *);
    int (*Reduce_scatter)(void *, void *, int *, struct MPIR_DATATYPE *, MPI_Op,
                          struct MPIR_COMMUNICATOR *);
    int (*Scan)(void *, void *, int, struct MPIR_DATATYPE *, MPI_Op, struct MPIR_COMMUNICATOR *);
    int ref_count;
};
extern MPIR_COLLOPS MPIR_inter_collops;
extern MPIR_COLLOPS MPIR_intra_collops;
#endif
