/*
 * oracle.h -- CPU restatement of the reference reduction path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load liboracle.so; the product library
 * (mvapich-cce_amd/) never links or calls it.
 *
 * What it restates:
 *   orc_op()              the 12 predefined MPI_Op kernels,
 *                         reference src/coll/global_ops.c:56-1745
 *   orc_allreduce()       intra_Allreduce, src/coll/intra_fns_new.c:5453-5790
 *   orc_reduce()          intra_Reduce,    src/coll/intra_fns_new.c:4519-4989
 *   orc_reduce_scatter()  intra_Reduce_scatter, src/coll/intra_fns_new.c:
 *                         6191-6720 (all four branches)
 *   orc_scan()            MPIR_intra_Scan, src/coll/intra_scan.c:91-150
 * The collectives are simulated with p in-memory ranks stepping in lockstep
 * through the reference's own send/recv schedule (every round snapshots the
 * senders before any receiver combines), so the combine order, the operand
 * roles (which rank's data is `inout`) and the per-rank op error codes are
 * the reference's, not a derived formula.
 *
 * Pinning: the reference cannot be compiled here without its configure step
 * (global_ops.c needs the generated mpichconf.h), so
 * this restatement is pinned by the reference's own known-answer tests
 * (examples/test/coll/ allred.c, redscat.c, coll12.c, redtst.c, shortint.c;
 * fixtures in tests/golden/) and by the reference
 * outputs recorded in SURVEY.md Appendix A.3/A.5.
 */
#ifndef MVX_ORACLE_H
#define MVX_ORACLE_H

#ifdef __cplusplus
extern "C" {
#endif

/* Datatype facts as the reference build registers them (initdte.c:106-280).
 * Returns 0 and fills extent / type_size (MPI_Type_size: bytes of the type
 * map, excluding padding), or MPI_ERR_TYPE (3) for an unregistered handle. */
int orc_dtype_info(int dtype, int *extent, int *type_size);

/* Derived types (cpu_types.c): the reference's constructors, bounds and
 * type maps; handles 256.. usable everywhere a datatype is.  Codes as the
 * reference (0, 2, 3, 12, 16, 323); a negative code -(class | kind << 6) is
 * one the reference makes with MPIR_Err_setmsg. */
int orc_type_contiguous(int count, int oldtype, int *newtype);
int orc_type_vector(int count, int blocklen, int stride, int oldtype, int *newtype);
int orc_type_hvector(int count, int blocklen, long stride, int oldtype, int *newtype);
int orc_type_indexed(int count, const int *blocklens, const int *indices, int oldtype, int *newtype);
int orc_type_hindexed(int count, const int *blocklens, const long *indices, int oldtype, int *newtype);
int orc_type_struct(int count, const int *blocklens, const long *indices, const int *types, int *newtype);
int orc_type_commit(int dtype);
int orc_type_free(int *dtype);
int orc_type_bounds(int dtype, long *lb, long *ub, long *extent, long *size);
/* kind: 1 contig, 2 hvector, 3 hindexed, 4 struct; old: the flattened old
 * type (contig), the old type, or old_types[0] (struct) */
int orc_derived_info(int dtype, int *kind, int *old, int *count, long *extent, long *size);
int orc_type_parts(int dtype, int *old, int *count);
/* n elements, type-map bytes only (what a message moves); 3 if not derived */
int orc_type_copy(void *dst, const void *src, long n, int dtype);
long orc_type_nblocks(int dtype);
int orc_type_block(int dtype, long i, long *off, long *len);

/* One predefined op: inout[i] = in[i] op inout[i] for i < len.
 * Returns 0, or 329 (MPIR_ERR_OP_NOT_DEFINED) for an undefined (op, type)
 * pair (the data is left untouched), or 9 (MPI_ERR_OP) for a bad handle. */
int orc_op(int op, int dtype, const void *in, void *inout, int len);
/* MPIR_F_TRUE / MPIR_F_FALSE for MPI_LOGICAL (default 1 / 0, gfortran) */
void orc_set_flog(int true_value, int false_value);

/* Collectives over p simulated ranks.  send[r]/recv[r] are rank r's
 * buffers; rc[r] receives rank r's return code.  Returns 0. */
int orc_allreduce(int p, const void *const *send, void *const *recv,
                  int count, int dtype, int op, int *rc);
int orc_reduce(int p, const void *const *send, void *const *recv,
               int count, int dtype, int op, int root, int *rc);
int orc_reduce_scatter(int p, const void *const *send, void *const *recv,
                       const int *recvcnts, int dtype, int op, int *rc);

/* User-defined ops (MPI_Op_create, opcreate.c:62-76): handles 200..263
 * name an MPI_User_function with its commute flag; the replays then take the
 * reference's permanent == 0 and noncommutative branches.  fn = NULL frees. */
typedef void orc_user_fn(void *invec, void *inoutvec, int *len, int *dtype);
int orc_user_op_set(int handle, orc_user_fn *fn, int commute);
/* orc_op for any handle, user ops included */
int orc_call(int op, int dtype, const void *in, void *inout, int len);

/* Device flavour of the replays.  smp = 0 (default): the ch_shmem build's
 * collops (intra_Reduce / intra_Allreduce).  smp = 1: the _SMP_ builds'
 * intra_shmem_Reduce / intra_shmem_Allreduce (intra_fns_new.c:4992-5198,
 * 5793-5940) on one node -- the len = 0 op test on every rank, then the
 * leader's rank-order fold below the thresholds (bytes, `count*extent`),
 * with the knobs enable_shmem_collectives, shmem_coll_ok,
 * disable_shmem_reduce / _allreduce. */
int orc_smp_set(int smp, int enable, int ok, int dis_red, int dis_ar, int thr_red,
                int thr_ar);

/* MPI_Scan, the default MPIR_intra_Scan (intra_scan.c:91-150) */
int orc_scan(int p, const void *const *send, void *const *recv, int count,
             int dtype, int op, int *rc);

/* Which algorithm the reference picks (same thresholds, intra_fns_new.c:
 * 30-40, 123-132, 4619, 5589, 6248, 6450).  Values: see ORC_ALG_*. */
#define ORC_ALG_NONE          0
#define ORC_ALG_RECDBL        1  /* Allreduce recursive doubling          */
#define ORC_ALG_RABENSEIFNER  2  /* RS (recursive halving) + AG / gather  */
#define ORC_ALG_BINOMIAL      3  /* Reduce binomial tree                  */
#define ORC_ALG_RS_HALVING    4  /* Reduce_scatter recursive halving      */
#define ORC_ALG_RS_PAIRWISE   5  /* Reduce_scatter pairwise exchange      */
#define ORC_ALG_RS_RECDBL     7  /* Reduce_scatter recursive doubling
                                    (noncommutative, < 512 bytes)         */
int orc_algorithm(int coll, int p, long total_count, int dtype);
int orc_algorithm_op(int coll, int p, long total_count, int dtype, int op);
#define ORC_COLL_ALLREDUCE      1
#define ORC_COLL_REDUCE         2
#define ORC_COLL_REDUCE_SCATTER 3

/* CPU baseline: the reference's schedules run by p
 * host threads over shared memory (oracle/cpu_coll.c), p a power of two;
 * Reduce: binomial tree only.  Returns seconds per collective. */
double orc_threads_coll(int coll, int p, void *const *send, void *const *recv, void *const *tmp,
                        int count, const int *recvcnts, int dtype, int op, int root, int reps);

/* Synthetic input generator: xorshift64 seeded
 * 0x9E3779B97F4A7C15 ^ (rank*1000003 + 1).  dist: 0 mixed-sign f32,
 * 1 U[0,1) f32, 2 int64 with P(bit)=0.953, 3 FLOAT_INT v=u%1024 l=rank,
 * 4 FLOAT_INT v=u%1024 l=rank*n+i, 5 raw 64-bit words (any type). */
void orc_fill(void *buf, long n, int dist, int rank);

#ifdef __cplusplus
}
#endif
#endif
