/*
 * mvx_internal.h -- declarations shared by libmvx.so's C sources (not part
 * of the drop-in surface; that is include/mvx_coll.h).
 *
 * libmvx.so is split by concern; every table a call works in belongs to the
 * communicator it runs on (mvx_comm_t.w), so two communicators alternating
 * calls never share staging, slice plans or transport state:
 *
 *   mvx_comm.c     communicators: creation, teardown (deferred release of an
 *                  aborted one's staging), knobs, phase timing, RCCL queries
 *   mvx_opreg.c    MPI_Op registry, datatype constructors and handles
 *   mvx_combine.c  phase B: the combine program (kernels, > 8 leaves, user
 *                  functions, datatypes with holes)
 *   mvx_xport.c    transports: RCCL, caller-supplied, loopback (virtual)
 *   mvx_exec.c     one rank's plan on device buffers: phases A-C and the
 *                  exchange variants P2P / PIPE / COLL
 *   mvx_stage.c    host buffers (sliced pipeline, HBM mirrors) and packed
 *                  datatypes
 *   mvx_api.c      the MPI entry points: argument checks, one call's job
 *   mvx_hostop.c   MPIR_SUM ... as MPI_User_functions on any memory
 *   mvx_host.c     buffer kinds, the host copy pool, the registration cache
 *   mvx_plan.c     the reference's schedules as per-rank plans
 */
#ifndef MVX_INTERNAL_H
#define MVX_INTERNAL_H

#include <stddef.h>
#include <stdint.h>

#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include "mvx_coll.h"
#include "mvx_hip.h"

/* internal linkage across the library's objects, never exported */
#define MVXI __attribute__((visibility("hidden")))

/* ---- mvx_host.c ---------------------------------------------------------- */
#define MVX_BUF_PAGEABLE 0   /* host memory the DMA engines cannot address */
#define MVX_BUF_PINNED   1   /* page-locked host memory */
#define MVX_BUF_DEVICE   2   /* device or managed memory */
/* pageable memory whose pages a registration of the cache partly covers
 * (a neighbour's, in use by another call): HIP refuses a copy that starts
 * inside a registration and runs past it (hipErrorInvalidValue,
 * tools/shadow_probe.c), so such memory is copied by the CPU through pinned
 * bounce slots, never handed to HIP (mvx_host.c) */
#define MVX_BUF_BOUNCE   3
int mvx_buf_kind(const void *p);   /* one pointer-attribute query */
int mvx_host_pinned(const void *p);
int mvxi_host_drain_lag(void);
void mvx_pcopy(void *dst, const void *src, size_t bytes);
int mvx_copy_threads(void);
/* the kind of [p, p + bytes): as mvx_buf_kind, except that with the
 * registration cache on a pageable range of at least its minimum is
 * registered (or found registered) and reads as MVX_BUF_PINNED */
MVXI int mvxi_buf_kind_range(const void *p, size_t bytes);
/* the same, for a call that will DMA the range: a range the cache hands out
 * as registered is held for the call (*hold its id, 0 if none) until
 * mvxi_buf_release(hold) after the call's last DMA on it -- a release of its
 * memory meanwhile defers the unregistration (mvx_host.c).  mine[0..nmine)
 * point at the holds this call took already, before any of its DMA: a
 * registration only this call holds may still be merged with the new range
 * (its operands sharing a page), and the ids there are updated if it is. */
MVXI int mvxi_buf_kind_hold(const void *p, size_t bytes, unsigned long *hold, unsigned long *const *mine,
                            int nmine);
MVXI void mvxi_buf_release(unsigned long hold);
MVXI hipError_t mvxi_queue_stream(hipStream_t *s, const char *env, const char *dflt);

/* ---- errors (mvx_comm.c) ----------------------------------------------- */
#define ERR_KIND_DEFAULT 1      /* MPIR_ERR_DEFAULT, mpi_error.h:119 */
#define ERR_KIND_ALIAS 7        /* MPIR_ERR_BUFFER_ALIAS, mpi_error.h:127 */
#define ERR_KIND_ROOT_TOOBIG 3  /* mpi_error.h:169 */
#define ERR_TYPE_NULL_CODE MVX_ERRCLASS_TO_CODE(MPI_ERR_TYPE, 5)  /* 323 */
#define ERR_COMM_NULL_CODE MVX_ERRCLASS_TO_CODE(MPI_ERR_COMM, 3)  /* 197 */
/* MPIR_Err_setmsg's return value (nerrmsg.c:111-182) */
MVXI int mvxi_setmsg_code(int cls, int kind);

/* ---- staging geometry ---------------------------------------------------- */
/* Consecutive staging slots are 4 KiB apart beyond their size: back-to-back
 * equal-size shards put the same chunk of every leaf at the same DRAM
 * interleave position, and the k-leaf combine then ran 5-6 % slower
 * (tools/tune_combine_layout.py, profiles/r01/tune_combine_layout.jsonl:
 * 53.9 vs 51.2 us for 8 x 32 MiB).  Re-swept in round 6 with the body
 * kernel: 4 KiB still among the best (47.8-48.7 us; 0 / 512 B 51.6-52.6,
 * 1.5-3 KiB 48.9-50.0, 3.5-12 KiB within 48.3-49.2:
 * profiles/r06/tune_combine_layout_fine.jsonl). */
#define SLOT_STAGGER 4096

static inline size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }

/* staging slot base with the same alignment mod 16 as `like`, so the
 * combine kernel keeps its 16-byte vector path */
static inline size_t slot_at(size_t cur, const void *like)
{
    return al256(cur) + ((uintptr_t)like & 15);
}

/* ---- transports (mvx_xport.c) -------------------------------------------- */
/* A phase is a group of point-to-point transfers.  RCCL issues them as one
 * ncclGroupStart/End; the loopback transport (virtual communicators) records
 * every rank's sends and receives of a phase and, once all ranks have
 * issued theirs, pairs them and copies device-to-device. */
#define LB_MAX (MVX_MAXP * MVX_MAXP)
typedef struct { int from, to; const void *src; void *dst; size_t bytes; int used; } lb_msg;
typedef struct { lb_msg send[LB_MAX], recv[LB_MAX]; int ns, nr; } loopback_t;

typedef struct mvx_xport {
    int (*start)(struct mvx_xport *);
    int (*end)(struct mvx_xport *);
    int (*send)(struct mvx_xport *, const void *, size_t, int, hipStream_t);
    int (*recv)(struct mvx_xport *, void *, size_t, int, hipStream_t);
    /* whole-communicator exchanges of the COLL variant (NULL: none) */
    int (*alltoall)(struct mvx_xport *, const void *, void *, size_t, hipStream_t);
    int (*allgather)(struct mvx_xport *, void *, size_t, hipStream_t);
    ncclComm_t nccl;
    loopback_t *lb;
    const mvx_transport *ops;   /* caller-supplied transport */
    hipStream_t st;             /* the stream its phases end on */
    int depth;                  /* nesting of start / end (one group) */
    int me;
} mvx_xport;

MVXI void mvxi_xport_loopback(mvx_xport *t, loopback_t *lb, int me);
/* pair every receive with its send (same from/to, issue order) and copy */
MVXI int mvxi_lb_flush(loopback_t *lb, hipStream_t st);

/* ---- one rank's execution of its plan (mvx_exec.c) ----------------------- */
typedef struct mvx_comm_t mvx_comm_t;

typedef struct {
    const mvx_plan *P;              /* the plan, or the current slice of it */
    mvx_comm_t *c;
    const char *sendbuf;            /* device */
    char *recvbuf;                  /* device */
    char *pool;                     /* this rank's staging region */
    size_t slot[MVX_MAXP], tmp_off;
    size_t wide_off, wide_slot;     /* scratch of a > 8-leaf combine */
    int wide_n;
} rank_exec_t;

/* a job: this process's ranks of one collective call */
typedef struct {
    int nr;                          /* local ranks: 1 (RCCL) or p (virtual) */
    const mvx_plan *P;               /* nr plans */
    const char *send[MVX_MAXP];      /* the caller's buffers */
    char *recv[MVX_MAXP];
    long nsend[MVX_MAXP], nrecv[MVX_MAXP];   /* elements */
    mvx_xport *t;                    /* nr transports */
    int kinds;                       /* 1: skind / rkind are filled (mvxi_job_kinds) */
    int skind[MVX_MAXP], rkind[MVX_MAXP];   /* MVX_BUF_* of send / recv (empty: DEVICE) */
    unsigned long shold[MVX_MAXP], rhold[MVX_MAXP];   /* registration holds (mvxi_buf_kind_hold) */
} job_t;

MVXI int mvxi_job_kinds(job_t *J);
/* the job is over (rc: its result; on failure the device is drained first,
 * as copies of a failed pipeline may still be in flight): drop its holds */
MVXI void mvxi_job_release(job_t *J, int rc);
MVXI void mvxi_graphs_clear(mvx_comm_t *c);
MVXI int mvxi_run_device(mvx_comm_t *c, const job_t *J, hipStream_t st);
MVXI int mvxi_exec_group(rank_exec_t *X, mvx_xport *t, int nr, hipStream_t st, mvx_comm_t *timed);
MVXI size_t mvxi_region_layout(mvx_comm_t *c, rank_exec_t *X, const job_t *J, const mvx_plan *Q, size_t *off);
MVXI int mvxi_job_layout(mvx_comm_t *c, rank_exec_t *X, const job_t *J, const mvx_plan *Q);
MVXI void mvxi_plan_slice(const mvx_plan *P, long i, long cs, mvx_plan *Q);
MVXI long mvxi_plan_span(const mvx_plan *P);
/* the slice schedule's slice length for a call's plan, 0 = unsliced (mvx_stage.c) */
MVXI long mvxi_slice_elems(const mvx_plan *P);
MVXI int mvxi_send_ranges(const mvx_plan *Q, mvx_range *v);
MVXI int mvxi_recv_ranges(const mvx_plan *Q, mvx_range *v);

/* ---- host buffers and packed datatypes (mvx_stage.c) --------------------- */
typedef struct {
    const char *sorg[MVX_MAXP];   /* device origins of the send vectors */
    char *rorg[MVX_MAXP];         /* device origins of the recv vectors */
    char *smir[MVX_MAXP], *rmir[MVX_MAXP], *psend[MVX_MAXP], *precv[MVX_MAXP];
} packed_bufs_t;

#define STAGE_NB 4         /* >= the drain lag + 2 (mvxi_host_drain_lag) */
#define STAGE_LAG_MAX 2
typedef struct {                  /* a communicator's host-staging resources */
    int ready;
    hipStream_t sh, sd;
    char *bin[STAGE_NB], *bout[STAGE_NB];
    size_t bbytes;
    hipEvent_t ein[STAGE_NB], eout[STAGE_NB], ex[STAGE_NB];
} stage_res_t;

MVXI int mvxi_run_job(mvx_comm_t *c, job_t *J, hipStream_t st, int blocking);
MVXI int mvxi_run_job_packed(mvx_comm_t *c, job_t *J, hipStream_t st, int blocking);
MVXI int mvxi_job_packed_host(const job_t *J);
MVXI int mvxi_copy_any(mvx_comm_t *c, void *dst, const void *src, size_t bytes, hipStream_t st, int sync);
MVXI int mvxi_run_staged(mvx_comm_t *c, const job_t *J, hipStream_t st);
MVXI int mvxi_typed_copy(mvx_comm_t *c, int dt, long n, const char *send, char *recv, hipStream_t st, int sync);
MVXI void mvxi_stage_release(stage_res_t *S);

/* ---- graphs of device calls (mvx_exec.c) ---------------------------------
 * With graphs on (mvx_comm_set_graphs), a device-buffer call whose job was
 * seen before is captured once into a HIP graph -- RCCL's transfer groups,
 * the combine launches, the cross-stream events of PIPE -- and replayed:
 * one hipGraphLaunch instead of the host issue of every group and kernel.
 * The key is everything the captured work depends on: the plan, the
 * buffers, the stream, the staging pool and the variant. */
#define GRAPH_CACHE 32
typedef struct {
    int state;                  /* 0 free, 1 seen once (ran eagerly; mvx_work.seen), 2 captured, 3 retired (mvx_exec.c) */
    unsigned long long hash;
    mvx_plan plan;
    const char *send;
    char *recv;
    hipStream_t st;
    char *pool;
    int exch, slices, keep;
    hipGraphExec_t exec;
    int ran_exch;
    int forked;                 /* the graph has parallel branches (graph_forked) */
    hipEvent_t done;            /* recorded after each launch: the exec is idle once it completes */
    unsigned long stamp;
} graph_ent_t;
/* the communicator's staging pool grows to `need` bytes; graphs captured on
 * the old pool are destroyed (or retired) before it is freed (mvx_exec.c) */
MVXI int mvxi_grow_pool(struct mvx_comm_t *c, size_t need);
/* which graph execs may be destroyed mid-life on this HIP runtime (mvx_comm.c) */
#define MVX_GRAPH_EVICT_NONE 0       /* none: retired, destroyed with the communicator */
#define MVX_GRAPH_EVICT_SERIAL 1     /* those without parallel branches (HIP < 7.2) */
#define MVX_GRAPH_EVICT_ALL 2        /* any (HIP >= 7.2) */
MVXI int mvxi_graph_evict_default(void);

/* a capture is open on this thread: staging must not be reallocated */
extern __thread int mvxi_capturing MVXI;

/* ---- communicators (mvx_comm.c) ------------------------------------------ */
/* The tables one call works in: formerly process statics, now owned by the
 * communicator (allocated at its first call, freed with it). */
typedef struct mvx_work {
    graph_ent_t graphs[GRAPH_CACHE];           /* captured device calls (live or retired) */
    graph_ent_t seen[GRAPH_CACHE];             /* jobs seen once (ran eagerly), the capture candidates */
    unsigned long graph_clock;
    long graphs_destroyed;                     /* execs destroyed mid-life so far */
    mvx_plan call_plan;                        /* mvx_api.c run(): this rank's plan */
    mvx_plan pipe[2][MVX_MAXP];                /* PIPE: slice plans, by slice parity */
    rank_exec_t px0[MVX_MAXP], px[2][MVX_MAXP];
    mvx_plan slice[STAGE_LAG_MAX + 1][MVX_MAXP];   /* staged: the slice being issued and the ones not drained yet */
    job_t pk_job;                              /* packed datatypes */
    packed_bufs_t pk_bufs;
    job_t tc_job;                              /* typed copy */
    packed_bufs_t tc_bufs;
    mvx_plan tc_plan;
    mvx_plan multi_plans[MVX_MAXP];            /* virtual communicators */
    mvx_xport multi_t[MVX_MAXP];
    loopback_t lb;
    job_t multi_job;
    stage_res_t stage;                         /* host staging streams / bounce slots */
} mvx_work;

struct mvx_comm_t {
    int used, rank, size, device, local;
    MPI_Comm handle;
    ncclComm_t nccl;
    hipStream_t stream;
    char *pool;          /* plan staging (received shards, temporaries) */
    size_t pool_bytes;
    char *hpool;         /* host-buffer staging */
    size_t hpool_bytes;
    char *upool;         /* user-op scratch: device (device functions) */
    size_t upool_bytes;
    char *uhost;         /* user-op scratch: pinned host (MPI_User_functions) */
    size_t uhost_bytes;
    char *xpool;         /* extent-layout scratch of packed (holey) datatypes */
    size_t xpool_bytes;
    mvx_tuning tune;     /* device flavour + knobs (mvx_coll.h) */
    int shmem_block;     /* claimed shmem collective block, -1 = none */
    int exch, exch_slices;      /* exchange variant, MVX_EXCH_* (mvx_coll.h) */
    int host_sliced;            /* host buffers at p > 1: sliced pipeline (all ranks' kinds agree) */
    int call_kinds;             /* the next blocking call's agreed kinds (MVX_KINDS_*), then 0 */
    int has_ops;                /* caller-supplied transport instead of RCCL */
    mvx_transport ops;
    hipStream_t cstream;        /* combine stream of the pipelined exchange */
    hipEvent_t pev[4];          /* its exchange-done / combine-done events */
    int timing;                 /* mvx_comm_set_phase_timing: events around phases A / B / C */
    int tev_ready, tev_kind;    /* events created; what the last timed call recorded (TEV_*) */
    hipEvent_t tev[4];          /* start, after A, after B, after C */
    int keep;                   /* this call's (op, type) is undefined: every combine keeps its inout */
    int ran_exch;               /* the variant the last call ran (mvx_comm_last_exchange), -1 none */
    hipStream_t last_st;        /* the stream of the last call (an abort's drain check) */
    int graphs;                 /* mvx_comm_set_graphs: capture / replay device calls */
    int graph_cap;              /* graphs it may hold (MVX_GRAPH_CACHE, <= GRAPH_CACHE) */
    int graph_evict;            /* graphs destroyed mid-life (LRU, pool change): MVX_GRAPH_EVICT_* */
    int graph_error;            /* a capture failed: graphs stay off on this communicator */
    int last_graph;             /* the last call: 0 eager, 1 replayed, 2 captured and launched */
    hipStream_t gstream;        /* graphs of null-stream calls run here (fork / join) */
    hipEvent_t gev[2];
    mvx_work *w;                /* per-call tables, NULL until the first call */
};

MVXI mvx_comm_t *mvxi_get_comm(MPI_Comm h);
MVXI mvx_work *mvxi_work(mvx_comm_t *c);
MVXI int mvxi_grow(char **buf, size_t *have, size_t need);
MVXI int mvxi_grow_host(char **buf, size_t *have, size_t need);
MVXI void mvxi_xport_comm(mvx_xport *t, mvx_comm_t *c, hipStream_t st);
/* switch to `device` for a call and back: enter returns the caller's device
 * (-1 unknown), or MVXI_DEV_FAILED when `device` cannot be selected */
#define MVXI_DEV_FAILED (-2)
MVXI int mvxi_dev_enter(int device);
MVXI void mvxi_dev_leave(int device, int prev);

/* per-phase timing: event i of a timed call (no-op when timing is off) */
#define TEV_NONE 0
#define TEV_PHASES 1
#define TEV_TOTAL 2
MVXI int mvxi_tev(mvx_comm_t *c, int i, hipStream_t st);

/* ---- ops (mvx_opreg.c) ---------------------------------------------------- */
typedef struct {           /* struct MPIR_OP, include/mpiops.h:1-11 */
    MPI_User_function *op;     /* host function (MPI_Op_create) */
    MVX_Device_function *dop;  /* stream-ordered device function */
    unsigned cookie;
    int commute, permanent;
} mvx_op_t;

MVXI int mvxi_predefined(MPI_Op op);
MVXI mvx_op_t *mvxi_user_op(MPI_Op op);
MVXI int mvxi_op_kind(MPI_Op op);
MVXI int mvxi_op_verdict(MPI_Op op, MPI_Datatype dt);
MVXI MPI_Datatype mvxi_user_handle(MPI_Datatype dt);
MVXI int mvxi_is_device_ptr(const void *p);

/* ---- phase B (mvx_combine.c) ---------------------------------------------- */
typedef struct { char *base; size_t slot; int used, cap; } scratch_t;
/* scratch slots a > 8-leaf program can take (0 up to MVX_COMBINE_KMAX) */
MVXI int mvxi_wide_temps(const mvx_plan *P);
MVXI int mvxi_combine(mvx_comm_t *c, const mvx_plan *P, const char *const *leafp, void *dst,
                      scratch_t *S, hipStream_t st);

#endif
