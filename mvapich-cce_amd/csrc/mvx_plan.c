/*
 * mvx_plan.c -- host logic of the device collectives: which algorithm the
 * reference would run, and, for one rank, what it sends, what it combines in
 * which order, and what it receives.  Pure C, no device calls.
 *
 * The reference runs each collective as log2(p) (or p-1) rounds of
 * MPI_Sendrecv + (*uop) over shrinking halves of the vector
 * (src/coll/intra_fns_new.c).  On MI355X all p contributions to a block can
 * be made co-resident in one exchange over xGMI, after which one kernel
 * replays the reference's whole combine tree for that block in registers.
 * The plan therefore reduces every algorithm to three phases:
 *   A  exchange of sendbuf ranges (all-to-all of blocks, or full vectors)
 *   B  one k-leaf combine whose leaf permutation and shape reproduce the
 *      reference's combine order and operand roles bit for bit
 *   C  distribution of the combined blocks (all-gather / gather to root)
 *
 * Order derivations (intra_fns_new.c line numbers):
 *  - Allreduce / Reduce recursive halving with distance 1, 2, 4 ...
 *    (5653-5710, 4697-4751): newrank o's value after level l is
 *    T(o,l) = op(T(o,l-1), T(o^2^(l-1), l-1)); newrank o ends owning block
 *    bitrev(o) (send_idx/recv_idx arithmetic 5668-5680).  With leaves
 *    y[q] = leaf(o ^ q) this is the TREE shape.
 *  - Recursive doubling (5592-5629): the same T(o, log2 pof2) over the whole
 *    vector, o = the rank's own newrank (rank-dependent for NaN / signed-zero
 *    MAX/MIN; identical on all ranks for symmetric ops).
 *  - Reduce_scatter recursive halving, distance pof2/2 ... 1 (6341-6407):
 *    H(o,m) = op(H(o,2m), H(o^m,2m)); leaves y[q] = leaf(o ^ bitrev(q)).
 *  - Reduce_scatter pairwise (6473-6500): chain over x_r, x_{r-1}, ...
 *  - Reduce binomial (4907-4954): relative-rank tree truncated at p,
 *    leaves y[q] = x_{(q+root)%p}.
 *  - Non-power-of-two folds: Allreduce / Reduce_scatter leaf(n) =
 *    op(x_{2n+1}, x_{2n}) (5548-5577, 6283-6312), Reduce leaf(n) =
 *    op(x_{2n}, x_{2n+1}) (4641-4671); leaf(n) = x_{n+rem} past the fold.
 */
#include <string.h>
#include "mvx_coll.h"
#include "mvx_hip.h"

/* coll_table, intra_fns_new.c:129-132, flattened: the reference reads
 * row[-1] (the previous row's last entry) when p = 1. */
static const int coll_table_flat[3 * 5] = {
    -1, -1, -1, 16384, 16384,
    -1, 65536, 8192, 4096, 4096,
    -1, 65536, 4096, 4096, 4096 };
#define ALLREDUCE_IDX 1
#define REDUCE_IDX 2
#define REDSCAT_COMMUTATIVE_LONG_MSG 524288   /* intra_fns_new.c:39-40 */
#define REDSCAT_NONCOMMUTATIVE_SHORT_MSG 512

/* Extent and MPI_Type_size of a handle, basic or derived: the datatype table
 * lives with the kernels that resolve it (mvx_type_describe, libmvx_hip.so;
 * initdte.c:106-280 for the basic and pair types -- pair structs carry an
 * MPI_UB, so their extent includes padding and their size does not --
 * type_contig.c for MPI_Type_contiguous).  MPI_LB / MPI_UB hold no data and
 * cannot be reduced. */
int mvx_dtype_info(int dtype, int *extent, int *type_size)
{
    long e, s;
    if (mvx_type_describe(dtype, NULL, NULL, &e, &s)) return MPI_ERR_TYPE;
    if (e > 0x7fffffffL || s > 0x7fffffffL) return MPI_ERR_TYPE;
    if (extent) *extent = (int)e;
    if (type_size) *type_size = (int)s;
    return MPI_SUCCESS;
}

static int pof2_lgn(int size, int *lgn_out)
{
    int pof2 = 1, lgn = -1;
    while (pof2 <= size) { pof2 <<= 1; lgn++; }
    pof2 >>= 1;
    lgn--;
    if (lgn > 4) lgn = 4;
    if (lgn_out) *lgn_out = lgn;
    return pof2;
}

static int log2i(int pof2)
{
    int l = 0;
    while ((1 << l) < pof2) l++;
    return l;
}

static int bitrev(int x, int bits)
{
    int r = 0, i;
    for (i = 0; i < bits; i++) r |= ((x >> i) & 1) << (bits - 1 - i);
    return r;
}

/* count * type_size as the reference's int arithmetic produces it */
static int imul32(long a, long b)
{
    return (int)(unsigned int)((unsigned long)a * (unsigned long)b);
}

int mvx_plan_algorithm_kind(int coll, int p, long total, int dtype, int kind)
{
    int e, ts, lgn, pof2, tv;
    const int permanent = kind == MVX_OPKIND_PREDEFINED;
    const int commute = kind != MVX_OPKIND_USER_NONCOMMUTE;
    if (mvx_dtype_info(dtype, &e, &ts) || p < 1 || total <= 0) return MVX_ALG_NONE;
    pof2 = pof2_lgn(p, &lgn);
    switch (coll) {
    case MVX_COLL_ALLREDUCE:     /* intra_fns_new.c:5589-5591 */
        tv = coll_table_flat[ALLREDUCE_IDX * 5 + lgn];
        if (tv == -1 || imul32(total, ts) < tv || !permanent || total < pof2)
            return MVX_ALG_RECDBL;
        return MVX_ALG_RABENSEIFNER;
    case MVX_COLL_REDUCE:        /* intra_fns_new.c:4619-4620 */
        tv = coll_table_flat[REDUCE_IDX * 5 + lgn];
        if (tv != -1 && imul32(total, ts) > tv && permanent && total >= pof2)
            return MVX_ALG_RABENSEIFNER;
        return MVX_ALG_BINOMIAL;
    case MVX_COLL_REDUCE_SCATTER: /* intra_fns_new.c:6248, 6450-6452, 6505 */
        if (commute && imul32(total, ts) < REDSCAT_COMMUTATIVE_LONG_MSG) return MVX_ALG_RS_HALVING;
        if (!commute && imul32(total, ts) < REDSCAT_NONCOMMUTATIVE_SHORT_MSG) return MVX_ALG_RS_RECDBL;
        return MVX_ALG_RS_PAIRWISE;
    case MVX_COLL_SCAN:          /* MPIR_intra_Scan, intra_scan.c:46-150 */
        return MVX_ALG_SCAN_RECDBL;
    default:
        return MVX_ALG_NONE;
    }
}

int mvx_plan_algorithm(int coll, int p, long total, int dtype)
{
    return mvx_plan_algorithm_kind(coll, p, total, dtype, MVX_OPKIND_PREDEFINED);
}

/* intra_shmem_Allreduce / intra_shmem_Reduce take their leader path when
 * (5849-5854, 5066-5070) the comm holds a shmem block, the message is short
 * (`int stride = count*extent`, the reference's int product, 5847 / 5064),
 * the path is not disabled, the op commutes and shmem collectives are on. */
static int smp_leader_path(int coll, long total, int extent, int kind, const mvx_tuning *t)
{
    int stride;
    if (!t || !t->smp || !t->enable_shmem_collectives || !t->shmem_coll_ok) return 0;
    if (kind == MVX_OPKIND_USER_NONCOMMUTE) return 0;
    stride = imul32(total, extent);
    if (coll == MVX_COLL_ALLREDUCE)
        return !t->disable_shmem_allreduce && stride < t->shmem_coll_allreduce_threshold;
    if (coll == MVX_COLL_REDUCE)
        return !t->disable_shmem_reduce && stride < t->shmem_coll_reduce_threshold;
    return 0;
}

int mvx_plan_algorithm_tuned(int coll, int p, long total, int dtype, int kind,
                             const mvx_tuning *t)
{
    int e, ts;
    if (mvx_dtype_info(dtype, &e, &ts) || p < 1 || total <= 0) return MVX_ALG_NONE;
    if (smp_leader_path(coll, total, e, kind, t)) return MVX_ALG_SMP_LEADER;
    return mvx_plan_algorithm_kind(coll, p, total, dtype, kind);
}

/* Does the op's result depend on which operand is inout?  For the IEEE
 * compare-select ops, where NaN and +-0 pick an operand by role (coll.h:14-19,
 * global_ops.c:1297-1309), and for every op on the x87 types: an x87 store
 * writes 10 bytes, so the 6 padding bytes of the 16-byte slot, which
 * MPI_LONG_DOUBLE's type map moves, stay those of the inout operand. */
static int is_ieee(int t)
{
    return t == MPI_FLOAT || t == MPI_DOUBLE || t == MPI_LONG_DOUBLE || t == MPI_REAL ||
           t == MPI_DOUBLE_PRECISION;
}

static int op_symmetric(int op, int dtype)
{
    int old = dtype, cnt = 1;
    /* an undefined pair leaves every inout operand as it is (global_ops.c's
     * default branches): the result is the inout leaf's, so roles matter */
    if (!mvx_op_supported(op, dtype)) return 0;
    if (dtype == MPI_LONG_DOUBLE || dtype == MPI_LONG_DOUBLE_INT) return 0;
    if (dtype >= MVX_TYPE_DERIVED_BASE || dtype == MPI_2REAL || dtype == MPI_2DOUBLE_PRECISION) {
        /* count-2 contiguous {value, loc} pairs of one base type: the IEEE /
         * x87 ones pick operands by role (NaN, +-0, slot padding) */
        mvx_type_describe(dtype, &old, &cnt, NULL, NULL);
        if (op != MPI_MAXLOC && op != MPI_MINLOC) return 0;
        return !is_ieee(old);
    }
    switch (op) {
    case MPI_SUM: case MPI_PROD: case MPI_LAND: case MPI_LOR: case MPI_LXOR:
    case MPI_BAND: case MPI_BOR: case MPI_BXOR:
        return 1;
    case MPI_MAX: case MPI_MIN:
        return !is_ieee(dtype);
    case MPI_MAXLOC: case MPI_MINLOC:
        return !(dtype == MPI_FLOAT_INT || dtype == MPI_DOUBLE_INT ||
                 dtype == MPI_LONG_DOUBLE_INT);
    default:
        return 0;
    }
}

/* the single-launch masks of a chain-of-trees program (include/mvx_coll.h,
 * include/mvx_hip.h): tree steps of every segment at its leaf offset, a
 * chain bit at every later segment head */
int mvx_plan_masks(const mvx_plan *P, unsigned *tree_mask, unsigned *chain_mask)
{
    unsigned t = 0, c = 0;
    int s, e, l, q;
    if (!P || P->k < 1 || P->k > MVX_COMBINE_KMAX) return MPI_ERR_ARG;
    for (s = 0; s < P->k; s = e) {
        for (e = s + 1; e < P->k && !(P->seg_heads >> e & 1ull); e++) ;
        if (s) c |= 1u << s;
        for (l = 0; (1 << l) < e - s; l++)
            for (q = 0; q + (1 << l) < e - s; q += 2 << l) t |= 1u << (l * 8 + s + q);
    }
    if (tree_mask) *tree_mask = t;
    if (chain_mask) *chain_mask = c;
    return MPI_SUCCESS;
}

static unsigned long long all_heads(int k)
{
    return k >= 64 ? ~0ull : (1ull << k) - 1;
}

static void set_range(mvx_range *r, long off, long cnt)
{
    r->off = cnt > 0 ? off : 0;
    r->cnt = cnt > 0 ? cnt : 0;
}

/* leaf n of a folded power-of-two tree.  a_odd: the odd rank is the inout
 * operand (Allreduce, Reduce_scatter); otherwise the even one (Reduce). */
static void fold_leaf(int n, int rem, int a_odd, int *a, int *b)
{
    if (n < rem) {
        *a = a_odd ? 2 * n + 1 : 2 * n;
        *b = a_odd ? 2 * n : 2 * n + 1;
    } else {
        *a = n + rem;
        *b = -1;
    }
}

/* blocks of the Rabenseifner reduce-scatter: cnts[i] = count/pof2, the last
 * block takes the remainder (intra_fns_new.c:5645-5651) */
static void rab_blocks(long count, int pof2, long *cnts, long *disps)
{
    int i;
    for (i = 0; i < pof2 - 1; i++) cnts[i] = count / pof2;
    cnts[pof2 - 1] = count - (count / pof2) * (pof2 - 1);
    disps[0] = 0;
    for (i = 1; i < pof2; i++) disps[i] = disps[i - 1] + cnts[i - 1];
}

/* Reduce_scatter recursive halving: does `rank` call (*uop) at least once?
 * Replays the index arithmetic of intra_fns_new.c:6283-6407. */
static int rs_halving_calls(int p, int rank, const int *recvcnts)
{
    int lgn, pof2 = pof2_lgn(p, &lgn), rem = p - pof2, i, mask;
    int newrank, send_idx = 0, recv_idx = 0, last_idx = pof2;
    long newcnts[MVX_MAXP];
    if (rank < 2 * rem) {
        if (rank % 2 == 0) return 0;
        return 1;   /* the fold combine over total_count > 0 elements */
    }
    newrank = rank - rem;
    for (i = 0; i < pof2; i++) {
        int old_i = (i < rem) ? i * 2 + 1 : i + rem;
        newcnts[i] = (old_i < 2 * rem) ? (long)recvcnts[old_i] + recvcnts[old_i - 1]
                                       : recvcnts[old_i];
    }
    for (mask = pof2 >> 1; mask > 0; mask >>= 1) {
        int newdst = newrank ^ mask;
        long recv_cnt = 0;
        if (newrank < newdst) {
            send_idx = recv_idx + mask;
            for (i = recv_idx; i < send_idx; i++) recv_cnt += newcnts[i];
        } else {
            recv_idx = send_idx + mask;
            for (i = recv_idx; i < last_idx; i++) recv_cnt += newcnts[i];
        }
        if (recv_cnt != 0) return 1;
        send_idx = recv_idx;
        last_idx = recv_idx + mask;
    }
    return 0;
}

static int plan_body(mvx_plan *P, int coll, int p, int rank, long count,
                     const int *recvcnts, int dtype, int op, int root, int kind,
                     const mvx_tuning *t)
{
    /* noncommutative user ops: every combine is uop(in = lower ranks,
     * inout = higher ranks) (5610-5624, 4922-4936, 6660-6682,
     * intra_scan.c:124-137), the same tree on every rank */
    const int canon = kind == MVX_OPKIND_USER_NONCOMMUTE;
    int e, ts, lgn, pof2, rem, L, i, s, q;
    long cnts[MVX_MAXP], disps[MVX_MAXP];

    memset(P, 0, sizeof *P);
    if (p < 1 || p > MVX_MAXP || rank < 0 || rank >= p) return MPI_ERR_COMM;
    if (mvx_dtype_info(dtype, &e, &ts)) return MPI_ERR_TYPE;
    for (i = 0; i < MVX_MAXK; i++) P->leaf_fold[i] = -1;
    P->coll = coll; P->p = p; P->rank = rank; P->root = root;
    P->op = op; P->dtype = dtype; P->esize = e;
    {   /* a type map with holes moves packed: MPI_Type_size bytes per element */
        int dense = 1;
        mvx_type_layout(dtype, NULL, &dense, NULL, NULL, NULL, NULL);
        if (!dense) { P->packed = 1; P->esize = ts; }
    }
    P->symmetric = kind == MVX_OPKIND_PREDEFINED && op_symmetric(op, dtype);
    P->opkind = kind;
    P->shape = MVX_SHAPE_TREE;

    if (coll == MVX_COLL_REDUCE_SCATTER) {
        long total = 0;
        if (!recvcnts) return MPI_ERR_ARG;
        for (i = 0; i < p; i++) { disps[i] = total; total += recvcnts[i]; }
        count = total;
    }
    P->count = count;
    P->alg = mvx_plan_algorithm_tuned(coll, p, count, dtype, kind, t);
    if (P->alg == MVX_ALG_NONE) return MPI_SUCCESS;   /* nothing to do */

    pof2 = pof2_lgn(p, &lgn);
    rem = p - pof2;
    L = log2i(pof2);

    if (P->alg == MVX_ALG_SMP_LEADER) {
        /* One node: the shmem group is the whole comm in rank order and its
         * leader is rank 0 (create_2level_comm.c:125-138).  The leader copies
         * its vector and folds local ranks 1 .. p-1 into it,
         * (*uop)(in = x_i, inout = acc) (5872-5888, 5089-5112): a left chain
         * x0 o x1 o ... o x_{p-1}, the same for every element.  Allreduce
         * broadcasts it (5926): every rank gets every vector in one exchange
         * and evaluates the chain itself.  Reduce: root gets the vectors
         * (the leader's hand-off to root, 5127-5181, moves the same bits). */
        if (coll == MVX_COLL_REDUCE && rank != root) {
            set_range(&P->a_send[root], 0, count);
            return MPI_SUCCESS;
        }
        for (s = 0; s < p; s++) {
            if (s == rank) continue;
            if (coll == MVX_COLL_ALLREDUCE) set_range(&P->a_send[s], 0, count);
            set_range(&P->a_recv[s], 0, count);
        }
        P->shape = MVX_SHAPE_CHAIN;
        P->has_combine = 1;
        P->k = p;
        for (q = 0; q < p; q++) P->leaf[q] = q;
        P->c_src_off = 0; P->c_cnt = count; P->c_dst_off = 0;
        return MPI_SUCCESS;
    }

    if (coll == MVX_COLL_ALLREDUCE) {
        const int newrank = rank < 2 * rem ? (rank % 2 ? rank / 2 : -1) : rank - rem;
        P->calls_uop = (rank < 2 * rem && rank % 2) || (newrank != -1 && pof2 > 1);
        if (P->alg == MVX_ALG_RECDBL && !P->symmetric && !canon) {
            /* every rank needs every vector: its own-rooted tree differs */
            const int o = rank < 2 * rem ? rank / 2 : rank - rem;
            for (s = 0; s < p; s++) {
                if (s == rank) continue;
                set_range(&P->a_send[s], 0, count);
                set_range(&P->a_recv[s], 0, count);
            }
            P->has_combine = 1;
            P->k = pof2;
            for (q = 0; q < pof2; q++) fold_leaf(o ^ q, rem, 1, &P->leaf[q], &P->leaf_fold[q]);
            P->c_src_off = 0; P->c_cnt = count; P->c_dst_off = 0;
            return MPI_SUCCESS;
        }
        /* Rabenseifner blocks: block j combined on rank j, then all-gathered */
        rab_blocks(count, pof2, cnts, disps);
        for (s = 0; s < p; s++) {
            if (s == rank) continue;
            if (s < pof2) set_range(&P->a_send[s], disps[s], cnts[s]);
            if (rank < pof2) set_range(&P->a_recv[s], disps[rank], cnts[rank]);
        }
        if (rank < pof2) {
            /* Rabenseifner: newrank o ends owning block bitrev(o); recursive
             * doubling with a rank-independent tree (symmetric or
             * noncommutative user op): any rank can combine any block */
            const int o = (P->symmetric || canon) ? 0 : bitrev(rank, L);
            P->has_combine = 1;
            P->k = pof2;
            for (q = 0; q < pof2; q++) fold_leaf(o ^ q, rem, 1, &P->leaf[q], &P->leaf_fold[q]);
            P->c_src_off = disps[rank]; P->c_cnt = cnts[rank]; P->c_dst_off = disps[rank];
            for (s = 0; s < p; s++)
                if (s != rank) set_range(&P->b_send[s], disps[rank], cnts[rank]);
        }
        for (s = 0; s < pof2; s++)
            if (s != rank) set_range(&P->b_recv[s], disps[s], cnts[s]);
        return MPI_SUCCESS;
    }

    if (coll == MVX_COLL_REDUCE) {
        if (root < 0 || root >= p) return MPI_ERR_ROOT;
        if (P->alg == MVX_ALG_RABENSEIFNER) {
            const int newrank = rank < 2 * rem ? (rank % 2 ? -1 : rank / 2) : rank - rem;
            P->calls_uop = (rank < 2 * rem && rank % 2 == 0) || (newrank != -1 && pof2 > 1);
            rab_blocks(count, pof2, cnts, disps);
            for (s = 0; s < p; s++) {
                if (s == rank) continue;
                if (s < pof2) set_range(&P->a_send[s], disps[s], cnts[s]);
                if (rank < pof2) set_range(&P->a_recv[s], disps[rank], cnts[rank]);
            }
            if (rank < pof2) {
                const int o = P->symmetric ? 0 : bitrev(rank, L);
                P->has_combine = 1;
                P->k = pof2;
                for (q = 0; q < pof2; q++) fold_leaf(o ^ q, rem, 0, &P->leaf[q], &P->leaf_fold[q]);
                P->c_src_off = disps[rank]; P->c_cnt = cnts[rank];
                if (rank == root) P->c_dst_off = disps[rank];
                else { P->c_dst_tmp = 1; set_range(&P->b_send[root], disps[rank], cnts[rank]); }
            }
            if (rank == root)
                for (s = 0; s < pof2; s++)
                    if (s != root) set_range(&P->b_recv[s], disps[s], cnts[s]);
            return MPI_SUCCESS;
        }
        /* binomial tree: gather every vector at root, combine there.  A
         * noncommutative op runs the tree relative to 0 and hands the result
         * to root (4908-4909, 4956-4966): the same leaves from 0. */
        const int lroot = canon ? 0 : root;
        {
            const int rel = (rank - lroot + p) % p;
            int m;
            for (m = 1; m < p; m <<= 1) {
                if (rel & m) break;
                if ((rel | m) < p) { P->calls_uop = 1; break; }
            }
        }
        if (rank != root) {
            set_range(&P->a_send[root], 0, count);
            return MPI_SUCCESS;
        }
        for (s = 0; s < p; s++)
            if (s != root) set_range(&P->a_recv[s], 0, count);
        P->has_combine = 1;
        P->k = p;
        for (q = 0; q < p; q++) P->leaf[q] = (q + lroot) % p;
        P->c_src_off = 0; P->c_cnt = count; P->c_dst_off = 0;
        return MPI_SUCCESS;
    }

    if (coll == MVX_COLL_SCAN) {
        /* rank r: recv = x_r; for l = 0.. : if bit l of r is set,
         * recv = op(recv, T(r - 2^l, l)), T(d, l) the partial of d's aligned
         * 2^l-block, T(d,l) = op(T(d,l-1), T(d^2^(l-1), l-1))
         * (intra_scan.c:118-147; every member of a block below r exists).
         * Leaves: [x_r | block l = 0 | block l = 1 | ...] for the set bits,
         * each block in the tree order x_{dst ^ q}; tree steps inside each
         * block, then a chain over the block heads. */
        int pos = 1, l;
        P->shape = -1;
        P->calls_uop = 0;          /* MPIR_intra_Scan never reports MPIR_Op_errno */
        for (s = 0; s < p; s++) {
            if (s > rank) set_range(&P->a_send[s], 0, count);
            if (s < rank) set_range(&P->a_recv[s], 0, count);
        }
        P->has_combine = 1;
        P->leaf[0] = rank;
        P->seg_heads = 1ull;
        /* noncommutative: dst's partial is the aligned block in rank order,
         * lower ranks as `in` at every tree level; the chain keeps recv as
         * inout (intra_scan.c:124-137) */
        P->tree_swap = canon;
        for (l = 0; (1 << l) <= rank; l++) {
            const int dst = rank ^ (1 << l), size_l = 1 << l;
            int q;
            if (!(rank & (1 << l))) continue;
            for (q = 0; q < size_l; q++) P->leaf[pos + q] = canon ? ((dst >> l) << l) + q : dst ^ q;
            P->seg_heads |= 1ull << pos;
            pos += size_l;
        }
        P->k = pos;                /* = rank + 1 */
        P->c_src_off = 0; P->c_cnt = count; P->c_dst_off = 0;
        return MPI_SUCCESS;
    }

    if (coll == MVX_COLL_REDUCE_SCATTER) {
        const long my = recvcnts[rank];
        for (s = 0; s < p; s++) {
            if (s == rank) continue;
            set_range(&P->a_send[s], disps[s], recvcnts[s]);
            set_range(&P->a_recv[s], disps[rank], my);
        }
        P->has_combine = 1;
        P->c_src_off = disps[rank]; P->c_cnt = my; P->c_dst_off = 0;
        if (P->alg == MVX_ALG_RS_PAIRWISE) {
            P->calls_uop = p > 1;
            P->shape = MVX_SHAPE_CHAIN;
            P->k = p;
            for (q = 0; q < p; q++) P->leaf[q] = (rank - q + p) % p;
            /* noncommutative: src = rank - q above rank swaps (6487-6498) */
            for (q = 1; q < p; q++)
                if (canon && q > rank) P->chain_swap |= 1ull << q;
        } else if (P->alg == MVX_ALG_RS_RECDBL) {
            /* noncommutative recursive doubling (6505-6706): block r ends as
             * the rank-ordered tree, lower ranks as `in` */
            P->k = p;
            for (q = 0; q < p; q++) P->leaf[q] = q;
        } else {
            const int o = rank < 2 * rem ? rank / 2 : rank - rem;
            P->calls_uop = rs_halving_calls(p, rank, recvcnts);
            P->k = pof2;
            for (q = 0; q < pof2; q++)
                fold_leaf(o ^ bitrev(q, L), rem, 1, &P->leaf[q], &P->leaf_fold[q]);
        }
        return MPI_SUCCESS;
    }
    return MPI_ERR_ARG;
}

int mvx_plan_build_tuned(mvx_plan *P, int coll, int p, int rank, long count,
                         const int *recvcnts, int dtype, int op, int root, int kind,
                         const mvx_tuning *t)
{
    int rc;
    if (kind < MVX_OPKIND_PREDEFINED || kind > MVX_OPKIND_USER_NONCOMMUTE) return MPI_ERR_ARG;
    rc = plan_body(P, coll, p, rank, count, recvcnts, dtype, op, root, kind, t);
    if (rc == MPI_SUCCESS && P->has_combine && P->shape >= 0) {
        P->seg_heads = P->shape == MVX_SHAPE_TREE ? 1ull : all_heads(P->k);
        if (kind == MVX_OPKIND_USER_NONCOMMUTE && P->shape == MVX_SHAPE_TREE)
            P->tree_swap = 1;
    }
    /* the _SMP_ collops test a predefined op with len = 0 on every rank
     * before choosing a path (5054-5058, 5841-5845): an undefined pair
     * fails on all ranks, p = 1 included */
    if (rc == MPI_SUCCESS && t && t->smp && kind == MVX_OPKIND_PREDEFINED &&
        P->alg != MVX_ALG_NONE && (coll == MVX_COLL_ALLREDUCE || coll == MVX_COLL_REDUCE))
        P->calls_uop = 1;
    return rc;
}

int mvx_plan_build_kind(mvx_plan *P, int coll, int p, int rank, long count,
                        const int *recvcnts, int dtype, int op, int root, int kind)
{
    return mvx_plan_build_tuned(P, coll, p, rank, count, recvcnts, dtype, op, root, kind, NULL);
}

int mvx_plan_build(mvx_plan *P, int coll, int p, int rank, long count,
                   const int *recvcnts, int dtype, int op, int root)
{
    return mvx_plan_build_kind(P, coll, p, rank, count, recvcnts, dtype, op, root,
                               MVX_OPKIND_PREDEFINED);
}
