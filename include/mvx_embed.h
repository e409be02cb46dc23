/*
 * mvx_embed.h -- the surface of libmvx_embed.so, the host library built to be
 * linked INTO an MPI implementation (integration/intra_mvx.c).  It declares
 * only mvx_* names with plain int handles, so it can be included next to the
 * host MPI's own mpi.h / mpiimpl.h without redefining MPI_Comm, MPI_SUM ...
 * (libmvx_embed.so exports nothing else, embed.map).  Every function here is
 * also in libmvx.so; mvx_coll.h includes this header so the compiler checks
 * the two declarations agree.
 *
 * Handles: datatypes and ops are libmvx's (include/mvx_mpi.h).  The
 * predefined ones have the reference's values (include/mpi.h:64-140), so a
 * permanent MPIR_DATATYPE's `self` and a predefined MPI_Op pass unchanged;
 * derived types are rebuilt with the mvx_type_* constructors of
 * include/mvx_hip.h and user ops registered with mvx_op_create.
 */
#ifndef MVX_EMBED_H
#define MVX_EMBED_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MVX_UNIQUE_ID_BYTES 128

/* communicators: one process per GPU, collective over `size` processes.
 * Creation and every call on a communicator run on its device and leave the
 * caller's current device as it was. */
int mvx_get_unique_id(void *id_out);
int mvx_comm_init(int *comm, int rank, int size, int device, const void *unique_id);
int mvx_comm_free(int *comm);
/* teardown without waiting for peers (ncclCommAbort; mvx_coll.h) */
int mvx_comm_abort(int *comm);
int mvx_device_count(void);
/* 0 if `device` can be selected and given a context -- what mvx_comm_init
 * needs of this rank before it enters RCCL's collective creation; 15
 * (MPI_ERR_OTHER) otherwise.  The current device is kept. */
int mvx_device_check(int device);
/* 1 if p is device (or managed) memory */
int mvx_buffer_is_device(const void *p);

/* the reduction collectives (reduce.c:62-96, allreduce.c:57-92,
 * red_scat.c:60-90, scan.c:55-95): same argument checks in the same order,
 * same return codes; device or host buffers */
int mvx_coll_reduce(void *sendbuf, void *recvbuf, int count, int datatype, int op, int root,
                    int comm);
int mvx_coll_allreduce(void *sendbuf, void *recvbuf, int count, int datatype, int op, int comm);
int mvx_coll_reduce_scatter(void *sendbuf, void *recvbuf, int *recvcnts, int datatype, int op,
                            int comm);
int mvx_coll_scan(void *sendbuf, void *recvbuf, int count, int datatype, int op, int comm);

/* user ops: MPI_User_function with int handles (include/mpi.h:282) */
typedef void(mvx_user_function)(void *invec, void *inoutvec, int *len, int *datatype);
int mvx_op_create(mvx_user_function *function, int commute, int *op);
int mvx_op_free(int *op);

/* The datatype handle a user function receives for libmvx type `type`
 * (default: `type` itself).  A binding that rebuilds the host MPI's derived
 * type as a libmvx type sets the host MPI's handle here, so the function
 * sees the handle its caller passed, as in the reference ((*uop)(..., &type),
 * intra_fns_new.c:5697).  handle == type removes the mapping.  Returns 0, or
 * MPI_ERR_OTHER (15) when the table (256 entries) is full. */
int mvx_type_set_handle(int type, int handle);

/* Registration cache for pageable host buffers (MVAPICH's dreg,
 * mpid/ch_gen2/dreg.c:774-832): with it on, a pageable range a call uses is
 * page-locked (hipHostRegister) on first use and kept, so later calls DMA
 * it directly.  A registration must never outlive its memory (a DMA through
 * one whose pages were freed and mapped again faults the GPU), so the cache
 * drops every registration inside a range before that range is released:
 *   on = 1  libmvx.so's release hooks report releases (free, realloc,
 *           munmap, mremap, madvise DONTNEED/FREE/REMOVE, negative sbrk are
 *           interposed, as the reference's mem_hooks.c interposes munmap and
 *           sbrk).  They are in effect when libmvx.so is in the program's
 *           global scope ahead of libc (a program linked with -lmvx);
 *           mvx_host_hooks_active says whether they are.  Without them
 *           on = 1 is refused (MPI_ERR_OTHER) and the cache stays off.
 *   on = 2  the caller reports releases: mvx_host_unregister(addr) before it
 *           frees a buffer it passed, or mvx_host_invalidate(addr, bytes)
 *           from its own memory hooks (a host MPI's mem_hooks.c;
 *           libmvx_embed.so has no hooks of its own).
 *   on = 0  off: every registration is dropped.
 * Env at first use: MVX_HOST_REGISTER=1|2 (1 only where the hooks are in
 * effect), MVX_HOST_REGISTER_MAX_MIB (16384) caps the registered bytes
 * (least recently used entries are dropped), MVX_HOST_REGISTER_MIN_KIB
 * (1024) is the smallest range registered.  max_bytes 0 keeps the cap. */
int mvx_host_register_enable(int on, size_t max_bytes);
int mvx_host_hooks_active(void);
/* Registers [addr, addr + bytes) now (as a call using it would): 0, or
 * MPI_ERR_OTHER (cache off, range below the minimum, refused). */
int mvx_host_register(const void *addr, size_t bytes);
/* Drops every registration containing addr: 0, or MPI_ERR_ARG if none.  A
 * registration a call in flight is using is unregistered when that call is
 * done. */
int mvx_host_unregister(const void *addr);
/* Drops every registration overlapping [addr, addr + bytes), which is about
 * to be released (the reference's find_and_free_dregs_inside, dreg.c:1063):
 * the number dropped.  Safe to call from inside a memory hook: it makes no
 * HIP call -- the registrations leave the cache at once and are unregistered
 * at the next libmvx entry, after the last call using them (dreg.c:678-767). */
int mvx_host_invalidate(const void *addr, size_t bytes);
int mvx_host_register_stats(long *entries, size_t *bytes, long *hits, long *misses);
/* registrations dropped by releases (hooks and mvx_host_invalidate) so far */
long mvx_host_register_invalidations(void);
/* dropped registrations not unregistered yet, registrations held by calls in
 * flight, hipHostUnregister calls made so far (in dry mode: that would have
 * been made), and ranges copied through the CPU because their pages were
 * partly under a registration in use by another call */
int mvx_host_register_deferred(long *deferred, long *held, long *unregisters, long *bounced);

/* The buffer kinds of every rank in the next blocking collective call on
 * `comm`, when the caller has agreed them across ranks (the MVAPICH shim
 * does, integration/intra_mvx.c): MVX_KINDS_DEVICE -- every rank passes
 * device memory: large calls keep the unsliced schedule and the exchange
 * variants; MVX_KINDS_HOST -- every rank passes host memory: host calls of
 * any size overlap their copies in slices; MVX_KINDS_UNKNOWN (the default,
 * also "mixed") -- the schedule that pairs with any kind.
 * Every rank must pass the same value; the next call consumes it.  Every
 * rank runs the schedule the hint names, so a rank whose own buffers
 * contradict it still pairs with its peers (host buffers under DEVICE go
 * through HBM mirrors; device buffers under HOST are used in place). */
#define MVX_KINDS_UNKNOWN 0
#define MVX_KINDS_DEVICE 1
#define MVX_KINDS_HOST 2
int mvx_comm_set_call_kinds(int comm, int kinds);

/* device flavour and collective knobs (the reference's _SMP_ collops) */
typedef struct mvx_tuning {
    int smp;                        /* 1: _SMP_ collops, 0: ch_shmem collops  */
    int enable_shmem_collectives;   /* initutil.c:146; VIADEV_USE_SHMEM_COLL=0,
                                       VIADEV_USE_BLOCKING=1, (MV|VIADEV)_USE_
                                       SHARED_MEM=0 clear it                  */
    int shmem_coll_ok;              /* the comm holds a shmem collective block
                                       (create_2level_comm.c:199-225, 274-279) */
    int disable_shmem_reduce;       /* !VIADEV_USE_SHMEM_REDUCE              */
    int disable_shmem_allreduce;    /* !VIADEV_USE_SHMEM_ALLREDUCE           */
    int shmem_coll_reduce_threshold;     /* bytes, default 1 << 10 (:70)    */
    int shmem_coll_allreduce_threshold;  /* bytes, default 1 << 15 (:71)    */
} mvx_tuning;
int mvx_tuning_from_env(mvx_tuning *t, int smp);
int mvx_comm_get_tuning(int comm, mvx_tuning *t);
int mvx_comm_set_tuning(int comm, const mvx_tuning *t);

#ifdef __cplusplus
}
#endif
#endif /* MVX_EMBED_H */
