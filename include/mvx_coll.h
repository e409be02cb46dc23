/*
 * mvx_coll.h -- libmvx.so, the C host library of the MI355X reduction path.
 *
 * Drop-in surface (same names, argument meaning and return codes as the
 * reference):
 *   MPI_Reduce / MPI_Allreduce / MPI_Reduce_scatter   include/mpi.h:400-404,
 *     bodies src/coll/reduce.c:62-96, allreduce.c:57-92, red_scat.c:60-90
 *   MPI_Op_create / MPI_Op_free                        src/coll/opcreate.c:62-76,
 *                                                      opfree.c:51-82
 *   MPIR_MAXF ... MPIR_MINLOC (MPI_User_function)      include/mpiimpl.h:201-212
 *   struct mvx_collops {Reduce, Allreduce, Reduce_scatter}
 *                                                      include/mpicoll.h:41-49
 * plus PMPI_ twins (include/mpi.h:589-593).
 *
 * Buffers may be device memory (the fast path: RCCL over xGMI moves shards,
 * libmvx_hip.so kernels do the arithmetic in the reference's combine order)
 * or host memory (staged through HBM; see DESIGN.md for the PCIe-inclusive
 * rate).  The blocking MPI_* calls return with the result in recvbuf; the
 * mvx_*_async variants are stream-ordered on the given HIP stream.
 */
#ifndef MVX_COLL_H
#define MVX_COLL_H

#include <stddef.h>
#include "mvx_mpi.h"
#include "mvx_embed.h"   /* mvx_tuning, mvx_type_set_handle; shared with libmvx_embed.so */

#ifdef __cplusplus
extern "C" {
#endif

/* ---- communicators ----------------------------------------------------- */

/* rank 0 creates the id, every rank passes the same bytes to mvx_comm_init.
 * Creation and every call on a communicator switch to its device for their
 * duration; the caller's current device is left as it was. */
int mvx_get_unique_id(void *id_out);
/* one process per GPU: collective over `size` processes (RCCL over xGMI);
 * the first communicator created becomes MPI_COMM_WORLD. */
int mvx_comm_init(MPI_Comm *comm, int rank, int size, int device,
                  const void *unique_id);
/* `size` virtual ranks in this process on one device (loopback transport,
 * device-to-device copies); use the *_multi entry points with it. */
int mvx_comm_init_local(MPI_Comm *comm, int size, int device);

/* One process per rank with a caller-supplied transport instead of RCCL
 * (e.g. several processes sharing one GPU, bytes moved by a host library).
 * A phase is start, then send / recv calls (device buffers, enqueued work on
 * `stream` must complete before the bytes are read), then end, which
 * performs them and returns once the received bytes are in place and
 * visible to later work on `stream`.  Sends and receives between one pair
 * of ranks pair up in call order.  Callbacks return 0 or an error. */
typedef struct mvx_transport {
    void *ctx;
    int (*start)(void *ctx);
    int (*send)(void *ctx, const void *buf, size_t bytes, int peer, void *stream);
    int (*recv)(void *ctx, void *buf, size_t bytes, int peer, void *stream);
    int (*end)(void *ctx, void *stream);
    /* Optional (both or neither; NULL = MVX_EXCH_COLL runs as MVX_EXCH_P2P
     * on this transport).  Same completion rules as a phase.
     *   alltoall:  block j of sendbuf (`bytes` each) goes to rank j; rank j's
     *              block for this rank lands in block j of recvbuf
     *   allgather: in place -- this rank's block is at buf + rank * bytes;
     *              on return block j holds rank j's block, for every j */
    int (*alltoall)(void *ctx, const void *sendbuf, void *recvbuf, size_t bytes, void *stream);
    int (*allgather)(void *ctx, void *buf, size_t bytes, void *stream);
} mvx_transport;
/* The table's base (ctx and the four phase callbacks): what every caller
 * has, whichever header it was compiled against. */
#define MVX_TRANSPORT_BASE_BYTES offsetof(mvx_transport, alltoall)
/* Reads the table's base only: a transport given here has no collective
 * hooks (MVX_EXCH_COLL runs as P2P). */
int mvx_comm_init_transport(MPI_Comm *comm, int rank, int size, int device,
                            const mvx_transport *transport);
/* Reads the first `bytes` of the table (pass sizeof(mvx_transport)): the
 * hooks when the caller's table has them, none when it is shorter.
 * MPI_ERR_ARG below MVX_TRANSPORT_BASE_BYTES. */
int mvx_comm_init_transport_ex(MPI_Comm *comm, int rank, int size, int device,
                               const mvx_transport *transport, size_t bytes);
/* helpers for transports: a blocking copy between any two pointers
 * (hipMemcpyDefault) and a stream synchronisation */
int mvx_copy(void *dst, const void *src, size_t bytes);
int mvx_stream_synchronize(void *stream);
int mvx_comm_free(MPI_Comm *comm);
int MPI_Comm_size(MPI_Comm comm, int *size);
int MPI_Comm_rank(MPI_Comm comm, int *rank);
/* stream the blocking calls run on (default: the null stream) */
int mvx_comm_set_stream(MPI_Comm comm, void *hip_stream);
/* pre-size the staging pool so no allocation happens inside a call */
int mvx_comm_reserve(MPI_Comm comm, size_t bytes);

/* How a communicator moves blocks between ranks (device buffers).  All
 * variants compute the same bits; they differ in how xGMI is driven.
 *   MVX_EXCH_P2P   phases as grouped ncclSend / ncclRecv (default)
 *   MVX_EXCH_PIPE  the exchange in `slices` slices, each combined on a
 *                  second stream as it arrives while the next is on the
 *                  links; one distribution group after the last combine
 *   MVX_EXCH_COLL  ncclAllToAll + in-place ncclAllGather when every rank
 *                  holds p equal blocks (Allreduce / Reduce_scatter with
 *                  count % p == 0, p a power of two); P2P otherwise
 * Env at creation: MVX_EXCHANGE = p2p | pipe[:slices] | coll. */
#define MVX_EXCH_P2P  0
#define MVX_EXCH_PIPE 1
#define MVX_EXCH_COLL 2
int mvx_comm_set_exchange(MPI_Comm comm, int mode, int slices);
int mvx_comm_get_exchange(MPI_Comm comm, int *mode, int *slices);
/* The variant the last collective call on `comm` actually ran: the one set,
 * or MVX_EXCH_P2P where it falls back (COLL on an irregular plan, a user op,
 * host buffers or a transport without collectives; PIPE on a plan too small
 * to slice); -1 when the call moved nothing between ranks. */
int mvx_comm_last_exchange(MPI_Comm comm, int *mode);
/* Device calls as HIP graphs (default off; env at creation MVX_GRAPH=1).
 * On an RCCL communicator, a device-buffer call with a predefined op whose
 * job (plan, buffers, stream, variant) was seen before is captured into a
 * graph once and replayed after: one hipGraphLaunch in place of the host
 * issue of every transfer group and kernel (the PIPE variant's slices
 * especially).  The first call of a job runs eagerly, the second captures
 * and launches, later ones replay.  Same bits as the eager calls.  A failed
 * capture turns graphs off on the communicator (mvx_comm_last_graph reports
 * the error).  A communicator holds at most 32 graphs (MVX_GRAPH_CACHE=n
 * fewer); when they are all taken the least recently used one is destroyed
 * for a new job, and graphs captured on a staging pool are destroyed before
 * the pool is reallocated -- any graph on HIP 7.2 and later, only graphs
 * without parallel branches on earlier runtimes, where destroying a forked
 * graph's exec crashes later launches (PIPE's graphs are kept there until
 * mvx_comm_free, and jobs past the cap run eagerly).  MVX_GRAPH_EVICT=0|1|2
 * overrides: none / single-branch only / all.  mvx_comm_set_graphs(comm, 0)
 * stops their use without destroying them. */
int mvx_comm_set_graphs(MPI_Comm comm, int on);
/* graphs the communicator holds (live: replayable; retired: kept, never
 * replayed again) and execs destroyed mid-life so far */
int mvx_comm_graph_stats(MPI_Comm comm, int *live, int *retired, long *destroyed);
/* The last call: *state 0 eager, 1 replayed, 2 captured and launched;
 * *error the failed capture's code that turned graphs off (0: none). */
int mvx_comm_last_graph(MPI_Comm comm, int *state, int *error);
/* Tear down a communicator without waiting for its outstanding transfers
 * (ncclCommAbort): the way out of a transfer that never completes.  The
 * handle is freed as by mvx_comm_free; the staging memory is not (work
 * queued behind the aborted transfers may still read it). */
int mvx_comm_abort(MPI_Comm *comm);
/* Frees the staging of aborted communicators whose queued work has drained
 * (an event recorded behind it on every stream they used has completed);
 * runs at every communicator creation and mvx_comm_reserve too.  Returns
 * how many aborted communicators' staging is still held. */
int mvx_comm_reap(void);
/* Host buffers at p > 1 on a one-rank-per-process communicator.  Default
 * (0): the call copies them into HBM mirrors and moves exactly what a
 * device-buffer call moves, so ranks may pass different buffer kinds in
 * one call, as MPI allows.  1: the sliced pipeline (H2D, collective and D2H
 * of successive slices overlap; faster) -- every rank must then pass host
 * buffers in every call.  Env at creation: MVX_HOST_PIPELINE=1. */
int mvx_comm_set_host_pipeline(MPI_Comm comm, int on);
/* Ablation only: RCCL's own ncclAllReduce (coll =
 * MVX_COLL_ALLREDUCE, count elements) or ncclReduceScatter (coll =
 * MVX_COLL_REDUCE_SCATTER, count elements per rank) with ncclSum on the
 * communicator's RCCL handle, stream-ordered.  RCCL's combine order is not
 * the reference's (floats differ in the last bits) and it has no BAND /
 * MAXLOC: never a substitute for MPI_Allreduce / MPI_Reduce_scatter.
 * MPI_FLOAT, MPI_DOUBLE, MPI_INT, MPI_LONG, MPI_LONG_LONG_INT; MPI_ERR_COMM
 * on a communicator without RCCL (virtual, caller transport). */
int mvx_comm_rccl_native(MPI_Comm comm, int coll, const void *sendbuf, void *recvbuf, size_t count,
                         MPI_Datatype dt, void *stream);
/* RCCL's own view of an RCCL communicator: ncclCommCount, ncclCommCuDevice
 * (this rank's device) and ncclGetVersion; any pointer may be NULL.
 * MPI_ERR_COMM on a communicator without RCCL (virtual, caller transport). */
int mvx_comm_rccl_info(MPI_Comm comm, int *nranks, int *device, int *version);
/* Per-phase timing (diagnostics): with timing on, each device-buffer call
 * records HIP events on its stream around phase A (exchange), B (combine)
 * and C (distribution).  mvx_comm_phase_times waits for the last timed call
 * and returns ms[0..2] = A, B, C (-1 for the pipelined variant, whose phases
 * overlap) and ms[3] = the whole call; MPI_ERR_OTHER if nothing was timed. */
int mvx_comm_set_phase_timing(MPI_Comm comm, int on);
int mvx_comm_phase_times(MPI_Comm comm, float *ms);

/* ---- MPI API (blocking) ------------------------------------------------ */
int MPI_Reduce(void *sendbuf, void *recvbuf, int count, MPI_Datatype datatype,
               MPI_Op op, int root, MPI_Comm comm);
int MPI_Allreduce(void *sendbuf, void *recvbuf, int count,
                  MPI_Datatype datatype, MPI_Op op, MPI_Comm comm);
int MPI_Reduce_scatter(void *sendbuf, void *recvbuf, int *recvcnts,
                       MPI_Datatype datatype, MPI_Op op, MPI_Comm comm);
/* MPI_Scan (src/coll/scan.c:55-95 -> MPIR_intra_Scan, intra_scan.c:46-150):
 * inclusive prefix in the reference's recursive-doubling order. */
int MPI_Scan(void *sendbuf, void *recvbuf, int count, MPI_Datatype datatype,
             MPI_Op op, MPI_Comm comm);
int MPI_Op_create(MPI_User_function *function, int commute, MPI_Op *op);
int MPI_Op_free(MPI_Op *op);

/* Derived datatypes (include/mpi.h:369-385; src/pt2pt/type_*.c; the type
 * engine is libmvx_hip.so's, include/mvx_hip.h): usable with every
 * collective here -- with MPI_Op_create ops (the user function gets the
 * derived handle and buffers laid out by extent, as in the reference), and
 * with MPI_MAXLOC / MPI_MINLOC on a count-2 contiguous pair type or on a
 * struct type read as its first member's C pair struct (global_ops.c:
 * 1280-1503, 1520-1740); any other predefined op on a derived type is the
 * reference's 329.  Types whose type map has holes move packed (type-map
 * bytes only) and are unpacked into recvbuf, so bytes outside the type map
 * are never written. */
int MPI_Type_contiguous(int count, MPI_Datatype oldtype, MPI_Datatype *newtype);
int MPI_Type_vector(int count, int blocklen, int stride, MPI_Datatype oldtype, MPI_Datatype *newtype);
int MPI_Type_hvector(int count, int blocklen, MPI_Aint stride, MPI_Datatype oldtype,
                     MPI_Datatype *newtype);
int MPI_Type_indexed(int count, int *blocklens, int *indices, MPI_Datatype oldtype,
                     MPI_Datatype *newtype);
int MPI_Type_hindexed(int count, int *blocklens, MPI_Aint *indices, MPI_Datatype oldtype,
                      MPI_Datatype *newtype);
int MPI_Type_struct(int count, int *blocklens, MPI_Aint *indices, MPI_Datatype *types,
                    MPI_Datatype *newtype);
int MPI_Type_commit(MPI_Datatype *datatype);
int MPI_Type_free(MPI_Datatype *datatype);
int MPI_Type_extent(MPI_Datatype datatype, MPI_Aint *extent);
int MPI_Type_size(MPI_Datatype datatype, int *size);
int MPI_Type_lb(MPI_Datatype datatype, MPI_Aint *displacement);
int MPI_Type_ub(MPI_Datatype datatype, MPI_Aint *displacement);

/* A user op whose function runs on the device: `function` enqueues
 * inoutvec[i] = invec[i] op inoutvec[i], i < len, on `stream` (a
 * hipStream_t) and returns 0, or nonzero to fail the call.  Collectives give
 * it the same operand roles and order as an MPI_Op_create op with the same
 * commute flag; no data leaves HBM.  (Extension: the reference has host
 * functions only.) */
typedef int (MVX_Device_function)(const void *invec, void *inoutvec, size_t len,
                                  MPI_Datatype datatype, void *stream);
int mvx_op_create_device(MVX_Device_function *function, int commute, MPI_Op *op);
/* MPI_Op_create / MPI_Op_free under names that cannot collide with a host
 * MPI library's (libmvx_embed.so exports only mvx_* names) */
int mvx_op_create(MPI_User_function *function, int commute, MPI_Op *op);
int mvx_op_free(MPI_Op *op);
/* GPUs visible to this process */
int mvx_device_count(void);
int MPI_Error_class(int errorcode, int *errorclass);

/* The same three calls under names that cannot collide with a host MPI
 * library's own MPI_* symbols: what an in-tree binding and
 * MVX_device_collops call. */
int mvx_coll_reduce(void *sendbuf, void *recvbuf, int count, MPI_Datatype datatype,
                    MPI_Op op, int root, MPI_Comm comm);
int mvx_coll_allreduce(void *sendbuf, void *recvbuf, int count,
                       MPI_Datatype datatype, MPI_Op op, MPI_Comm comm);
int mvx_coll_reduce_scatter(void *sendbuf, void *recvbuf, int *recvcnts,
                            MPI_Datatype datatype, MPI_Op op, MPI_Comm comm);
int mvx_coll_scan(void *sendbuf, void *recvbuf, int count, MPI_Datatype datatype,
                  MPI_Op op, MPI_Comm comm);
/* 1 if p is device (or managed) memory the device path can use directly */
int mvx_buffer_is_device(const void *p);

int PMPI_Reduce(void *, void *, int, MPI_Datatype, MPI_Op, int, MPI_Comm);
int PMPI_Allreduce(void *, void *, int, MPI_Datatype, MPI_Op, MPI_Comm);
int PMPI_Reduce_scatter(void *, void *, int *, MPI_Datatype, MPI_Op, MPI_Comm);
int PMPI_Scan(void *, void *, int, MPI_Datatype, MPI_Op, MPI_Comm);
int PMPI_Op_create(MPI_User_function *, int, MPI_Op *);
int PMPI_Op_free(MPI_Op *);

/* ---- stream-ordered variants (device buffers only) ---------------------
 * Calls on one communicator share its staging pool: issue them on one
 * stream (as MPI orders a communicator's collectives), or synchronise the
 * streams between calls -- RCCL does not order one communicator's transfers
 * issued on two streams against each other (round 4: such a schedule did
 * not finish at p = 8, tools/graph_cost.c).
 *
 * Buffer kinds may differ across ranks: a host buffer at p > 1 is mirrored
 * in HBM and its blocks move as a device buffer's do.  Only the opt-in
 * sliced host pipeline (mvx_comm_set_host_pipeline) moves host buffers in
 * slices, and then every rank of a call must pass host buffers. */
int mvx_reduce_async(const void *sendbuf, void *recvbuf, int count,
                     MPI_Datatype datatype, MPI_Op op, int root, MPI_Comm comm,
                     void *hip_stream);
int mvx_allreduce_async(const void *sendbuf, void *recvbuf, int count,
                        MPI_Datatype datatype, MPI_Op op, MPI_Comm comm,
                        void *hip_stream);
int mvx_scan_async(const void *sendbuf, void *recvbuf, int count,
                   MPI_Datatype datatype, MPI_Op op, MPI_Comm comm, void *hip_stream);
int mvx_reduce_scatter_async(const void *sendbuf, void *recvbuf,
                             const int *recvcnts, MPI_Datatype datatype,
                             MPI_Op op, MPI_Comm comm, void *hip_stream);

/* ---- virtual communicators: all ranks' buffers in this process ---------- */
/* rc[r] receives rank r's return code; the function returns MPI_SUCCESS or
 * the first argument error. */
int mvx_reduce_multi(void *const *sendbufs, void *const *recvbufs, int count,
                     MPI_Datatype datatype, MPI_Op op, int root, MPI_Comm comm,
                     int *rc, void *hip_stream);
int mvx_allreduce_multi(void *const *sendbufs, void *const *recvbufs,
                        int count, MPI_Datatype datatype, MPI_Op op,
                        MPI_Comm comm, int *rc, void *hip_stream);
int mvx_scan_multi(void *const *sendbufs, void *const *recvbufs, int count,
                   MPI_Datatype datatype, MPI_Op op, MPI_Comm comm, int *rc,
                   void *hip_stream);
int mvx_reduce_scatter_multi(void *const *sendbufs, void *const *recvbufs,
                             const int *recvcnts, MPI_Datatype datatype,
                             MPI_Op op, MPI_Comm comm, int *rc,
                             void *hip_stream);

/* ---- collective function table (mpicoll.h:41-51 members, by handle) ---- */
typedef struct mvx_collops {
    int (*Reduce)(void *, void *, int, MPI_Datatype, MPI_Op, int, MPI_Comm);
    int (*Allreduce)(void *, void *, int, MPI_Datatype, MPI_Op, MPI_Comm);
    int (*Reduce_scatter)(void *, void *, int *, MPI_Datatype, MPI_Op,
                          MPI_Comm);
    int (*Scan)(void *, void *, int, MPI_Datatype, MPI_Op, MPI_Comm);
} mvx_collops;
extern const mvx_collops MVX_device_collops;

/* ---- predefined ops as MPI_User_functions (global_ops.c) ---------------
 * invec / inoutvec may be device or host memory: when neither is pageable
 * (device, or page-locked: hipHostMalloc'd, hipHostRegister'ed, or pinned by
 * the registration cache) the kernel reads and writes them in place
 * (MVX_HOST_ZEROCOPY=0: through HBM instead); pageable operands are streamed
 * through HBM in chunks, H2D / kernel / D2H overlapped.  The call completes
 * before it returns.  An undefined (op, type) pair leaves the data alone and sets
 * mvx_op_errno() to 329, as MPIR_Op_errno (global_ops.c:41). */
void MPIR_MAXF(void *, void *, int *, MPI_Datatype *);
void MPIR_MINF(void *, void *, int *, MPI_Datatype *);
void MPIR_SUM(void *, void *, int *, MPI_Datatype *);
void MPIR_PROD(void *, void *, int *, MPI_Datatype *);
void MPIR_LAND(void *, void *, int *, MPI_Datatype *);
void MPIR_BAND(void *, void *, int *, MPI_Datatype *);
void MPIR_LOR(void *, void *, int *, MPI_Datatype *);
void MPIR_BOR(void *, void *, int *, MPI_Datatype *);
void MPIR_LXOR(void *, void *, int *, MPI_Datatype *);
void MPIR_BXOR(void *, void *, int *, MPI_Datatype *);
void MPIR_MAXLOC(void *, void *, int *, MPI_Datatype *);
void MPIR_MINLOC(void *, void *, int *, MPI_Datatype *);
int mvx_op_errno(void);

/* ---- plans (host logic, no device needed; exported for tests) ----------- */
#define MVX_MAXP 64
#define MVX_MAXK 64

#define MVX_COLL_ALLREDUCE      1
#define MVX_COLL_REDUCE         2
#define MVX_COLL_REDUCE_SCATTER 3
#define MVX_COLL_SCAN           4

#define MVX_ALG_NONE          0
#define MVX_ALG_RECDBL        1
#define MVX_ALG_RABENSEIFNER  2
#define MVX_ALG_BINOMIAL      3
#define MVX_ALG_RS_HALVING    4
#define MVX_ALG_RS_PAIRWISE   5
#define MVX_ALG_SCAN_RECDBL   6
#define MVX_ALG_RS_RECDBL     7   /* noncommutative Reduce_scatter < 512 bytes */
#define MVX_ALG_SMP_LEADER    8   /* _SMP_ builds: node leader's sequential fold
                                     (intra_shmem_Reduce / intra_shmem_Allreduce) */

/* ---- device flavour and collective knobs -------------------------------
 * The reference picks its collops at build time: the ch_shmem device (no
 * _SMP_, the flavour SURVEY.md's oracle was built as) installs intra_Reduce /
 * intra_Allreduce; the _SMP_ devices (ch_gen2, ch_smp, ch_gen2_ud) install
 * intra_shmem_Reduce / intra_shmem_Allreduce in front of them
 * (intra_fns_new.c:293-310), whose small-message path is a leader folding the
 * node's ranks in rank order (4992-5198, 5793-5940), with runtime knobs read
 * by MPIR_Init (initutil.c:230-293).  Here the flavour is per communicator. */
/* typedef struct mvx_tuning: include/mvx_embed.h */

/* The knobs of an `smp` build after MPIR_Init's environment parsing
 * (VIADEV_USE_SHMEM_REDUCE, VIADEV_USE_SHMEM_ALLREDUCE, VIADEV_USE_BLOCKING,
 * VIADEV_USE_SHMEM_COLL, VIADEV_USE_SHARED_MEM, MV_USE_SHARED_MEM,
 * VIADEV_SHMEM_COLL_MAX_MSG_SIZE, VIADEV_SHMEM_COLL_{REDUCE,ALLREDUCE}_
 * THRESHOLD); shmem_coll_ok = 1.  Returns MPI_ERR_OTHER where the reference
 * prints and exits (a threshold above the max message size, :289-293). */
int mvx_tuning_from_env(mvx_tuning *t, int smp);
/* Communicators take their flavour from MVX_DEVICE at creation: "ch_gen2",
 * "ch_smp" or "ch_gen2_ud" select the _SMP_ collops, anything else (default
 * "ch_shmem") the plain ones.  An _SMP_ communicator claims one of the
 * VIADEV_MAX_SHMEM_COLL_COMM (default 16) shmem blocks, as create_2level_comm
 * does; without one its shmem_coll_ok is 0. */
int mvx_comm_get_tuning(MPI_Comm comm, mvx_tuning *t);
int mvx_comm_set_tuning(MPI_Comm comm, const mvx_tuning *t);

/* What kind of op a plan is for: the reference's struct MPIR_OP
 * {permanent, commute} (include/mpiops.h:1-11) */
#define MVX_OPKIND_PREDEFINED      0   /* permanent, commutative          */
#define MVX_OPKIND_USER_COMMUTE    1   /* MPI_Op_create(f, 1, ...)        */
#define MVX_OPKIND_USER_NONCOMMUTE 2   /* MPI_Op_create(f, 0, ...)        */

typedef struct { long off, cnt; } mvx_range;   /* in elements */

/* What rank `rank` does for one collective call.  Phase A: send ranges of
 * its sendbuf, receive other ranks' sendbuf ranges into staging slot s.
 * Phase B: one k-leaf combine (leaf q = rank leaf[q]'s data, folded with
 * rank leaf_fold[q]'s data when >= 0) over elements [c_src_off, +c_cnt) of
 * the source vectors, written to recvbuf + c_dst_off (c_dst_tmp = 0) or to
 * a temporary (1).  Phase C: send the combine output to the ranks in
 * b_send (destination recvbuf coordinates), receive b_recv ranges into
 * recvbuf.
 *
 * The combine program is a chain of trees over the leaves (every order of
 * the reference's collectives has this form, k <= MVX_MAXK):
 *   bit q of seg_heads starts a segment (bit 0 is always set); each segment
 *   [q, next head) is reduced as a TREE (include/mvx_hip.h: level by level,
 *   y[q] = op(y[q], y[q + 2^l])) into its first leaf; then, for every later
 *   head q in ascending order, y[0] = op(y[0], y[q]).
 * TREE(k) is seg_heads = 1; CHAIN(k) is every leaf a head; MPI_Scan's
 * partial sums are a chain over [x_r, tree blocks].  The left operand of a
 * step is the reference's `inoutvec`.  Up to 8 leaves this is one kernel
 * launch (mvx_op_program masks); beyond, the executor evaluates trees in
 * groups of 8 and the chain in windows of 8 -- the same association. */
typedef struct mvx_plan {
    int coll, alg, p, rank, root, op, dtype, esize;
    int symmetric;      /* result independent of operand roles */
    int calls_uop;      /* the reference calls (*uop) on this rank */
    long count;         /* vector elements (Reduce_scatter: total) */
    mvx_range a_send[MVX_MAXP];
    mvx_range a_recv[MVX_MAXP];
    int has_combine, k, shape, c_dst_tmp;   /* shape: MVX_SHAPE_* or -1 (mixed) */
    unsigned long long seg_heads;           /* the combine program, see above */
    int leaf[MVX_MAXK];
    int leaf_fold[MVX_MAXK];
    long c_src_off, c_cnt, c_dst_off;
    mvx_range b_send[MVX_MAXP];
    mvx_range b_recv[MVX_MAXP];
    int opkind;                       /* MVX_OPKIND_* */
    /* steps whose operand roles are exchanged: the step is
     * y = uop(in = y_left, inout = y_right), the reference's noncommutative
     * "order is not right" branch.  tree_swap: every tree step; chain_swap
     * bit q: the chain step at head q.  Only user ops set them (the device
     * kernels never see a swap). */
    int tree_swap;
    unsigned long long chain_swap;
    /* the datatype's type map has holes (mvx_type_layout dense == 0): every
     * range moves packed type-map bytes, esize = MPI_Type_size; the combine
     * unpacks its leaves to the extent layout the op sees */
    int packed;
} mvx_plan;

/* The single-launch masks (mvx_op_program) of a plan's program when
 * k <= MVX_COMBINE_KMAX; returns 0, or MPI_ERR_ARG for a larger k. */
int mvx_plan_masks(const mvx_plan *plan, unsigned *tree_mask, unsigned *chain_mask);

/* Builds rank `rank`'s plan; returns 0 or an MPI error class. */
int mvx_plan_build(mvx_plan *plan, int coll, int p, int rank, long count,
                   const int *recvcnts, int dtype, int op, int root);
/* The same for a user op (opkind MVX_OPKIND_*): permanent == 0 forces
 * recursive doubling / the binomial tree (intra_fns_new.c:5590, 4620), and a
 * noncommutative op takes the reference's order-preserving branches. */
int mvx_plan_build_kind(mvx_plan *plan, int coll, int p, int rank, long count,
                        const int *recvcnts, int dtype, int op, int root, int opkind);
/* The same under a device flavour (NULL = ch_shmem). */
int mvx_plan_build_tuned(mvx_plan *plan, int coll, int p, int rank, long count,
                         const int *recvcnts, int dtype, int op, int root, int opkind,
                         const mvx_tuning *t);
/* The reference's algorithm for (coll, p, total elements, dtype[, opkind]). */
int mvx_plan_algorithm(int coll, int p, long total_count, int dtype);
int mvx_plan_algorithm_kind(int coll, int p, long total_count, int dtype, int opkind);
int mvx_plan_algorithm_tuned(int coll, int p, long total_count, int dtype, int opkind,
                             const mvx_tuning *t);
/* Datatype facts: extent and MPI_Type_size; returns 0 or MPI_ERR_TYPE. */
int mvx_dtype_info(int dtype, int *extent, int *type_size);

#ifdef __cplusplus
}
#endif
#endif /* MVX_COLL_H */
