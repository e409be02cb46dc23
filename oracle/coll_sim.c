/*
 * coll_sim.c -- TEST INFRASTRUCTURE: lockstep simulation of the reference's
 * Reduce / Allreduce / Reduce_scatter schedules over p in-memory ranks.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use
 * this (via oracle/liboracle.so).  Every message of the reference algorithm
 * is replayed as a copy from the sender's buffer state at the start of the
 * round (MPI_Sendrecv pairs are symmetric inside a round), and every (*uop)
 * call is replayed with the same (in, inout, len) arguments, so combine
 * order, operand roles and per-rank error codes follow the reference.
 *
 *   orc_allreduce       intra_fns_new.c:5453-5790
 *     self copy 5521, pof2/lgn 5527-5538, non-pof2 fold (even -> rank+1)
 *     5548-5577, algorithm choice 5589-5591, recursive doubling 5592-5629,
 *     reduce-scatter by recursive halving 5632-5710, allgather 5712-5754,
 *     non-pof2 tail 5764-5776, MPIR_Op_errno return 5783-5786.
 *   orc_reduce          intra_fns_new.c:4519-4989
 *     Rabenseifner 4619-4874 (odd -> rank-1 fold 4641-4671, halving
 *     4697-4751, odd-root hand-off 4760-4789, binomial gather 4791-4870);
 *     binomial tree 4876-4954.
 *   orc_reduce_scatter  intra_fns_new.c:6191-6503
 *     recursive halving 6248-6448 (fold 6283-6312, counts 6325-6339,
 *     mask pof2/2 -> 1 6341-6407), pairwise 6450-6503 (noncommutative
 *     operand swap 6487-6498), noncommutative recursive doubling 6505-6706.
 * User ops (orc_user_op_set) take the permanent == 0 choices (recursive
 * doubling 5590, binomial 4620) and every `commute` branch: 5610-5624,
 * 4908-4936 / 4956-4966, 6487, 6660-6682, intra_scan.c:124-137.
 */
#include <stdlib.h>
#include <string.h>
#include "oracle.h"

#define ERR_OP 9
#define ERR_TYPE 3
#define ERR_COUNT 2

/* coll_table, intra_fns_new.c:129-132, flattened so that the reference's
 * lgn = -1 read at p = 1 (row[-1] = previous row's last entry) is kept. */
static const int coll_table_flat[3 * 5] = {
    -1, -1, -1, 16384, 16384,
    -1, 65536, 8192, 4096, 4096,
    -1, 65536, 4096, 4096, 4096 };
#define ALLREDUCE_IDX 1
#define REDUCE_IDX 2
#define REDSCAT_COMMUTATIVE_LONG_MSG 524288   /* intra_fns_new.c:39-40 */
#define REDSCAT_NONCOMMUTATIVE_SHORT_MSG 512

static int pof2_lgn(int size, int *lgn_out)
{
    int pof2 = 1, lgn = -1;
    while (pof2 <= size) { pof2 <<= 1; lgn++; }
    pof2 >>= 1;
    lgn--;
    if (lgn > 4) lgn = 4;
    *lgn_out = lgn;
    return pof2;
}

/* 32-bit int product as the reference computes count*type_size */
static int imul32(long a, long b)
{
    return (int)(unsigned int)((unsigned long)a * (unsigned long)b);
}

#define NUOPS 64
static struct { orc_user_fn *fn; int commute; } g_uops[NUOPS];

int orc_user_op_set(int handle, orc_user_fn *fn, int commute)
{
    if (handle < 200 || handle >= 200 + NUOPS) return 12;
    g_uops[handle - 200].fn = fn;
    g_uops[handle - 200].commute = commute;
    return 0;
}

static int permanent(int op) { return op >= 100 && op <= 111; }
static int op_valid(int op)
{
    return permanent(op) || (op >= 200 && op < 200 + NUOPS && g_uops[op - 200].fn);
}
static int commute(int op) { return permanent(op) ? 1 : g_uops[op - 200].commute; }

/* copy n elements, only the bytes in the datatype's type map (MPI message
 * semantics: padding of the destination is left alone) */
static void tm_copy(void *dst, const void *src, long n, int dtype)
{
    int e, s;
    long i;
    if (orc_type_copy(dst, src, n, dtype) == 0) return;   /* derived: its type map */
    orc_dtype_info(dtype, &e, &s);
    if (e == s) { memcpy(dst, src, (size_t)(n * e)); return; }
    for (i = 0; i < n; i++) {
        char *d = (char *)dst + i * e;
        const char *x = (const char *)src + i * e;
        switch (dtype) {
        case 18: case 19: memcpy(d, x, 8); memcpy(d + 8, x + 8, 4); break;
        case 20: memcpy(d, x, 2); memcpy(d + 4, x + 4, 4); break;
        default: memcpy(d, x, (size_t)s); break; /* LONG_DOUBLE_INT: v,l */
        }
    }
}

/* Data buffers (temporaries, snapshots) hold every byte the type map of
 * their elements touches relative to the origin, [lo, hi): for a derived
 * type whose map reaches past count * extent (e.g. displacements from 1 with
 * extent 14 and map bytes up to 14) that is wider than count * extent --
 * the bytes the reference's MPI_Sendrecv of the type moves and its
 * MALLOC(count * extent) - lb temporaries hold.  The allocation's base is
 * kept in a small table so data_free can find it from the origin. */
typedef struct { long lo, hi; } span_t;

static span_t span_of(int dtype, long n)
{
    int E, TS;
    long nb, i, off, len;
    span_t s = {0, 0};
    if (orc_dtype_info(dtype, &E, &TS) || n <= 0) return s;
    s.hi = n * E;
    nb = orc_type_nblocks(dtype);
    for (i = 0; i < nb; i++) {
        if (orc_type_block(dtype, i, &off, &len)) continue;
        if (off < s.lo) s.lo = off;
        if ((n - 1) * E + off + len > s.hi) s.hi = (n - 1) * E + off + len;
    }
    return s;
}

#define DATA_SLOTS 8192
static struct { char *origin, *base; } g_data[DATA_SLOTS];

/* zeroed buffer for `bytes` (= n * extent) bytes of dtype; returns the origin */
static char *data_calloc(long bytes, int dtype)
{
    int E, TS, i;
    long n;
    span_t s;
    char *b;
    orc_dtype_info(dtype, &E, &TS);
    n = E > 0 ? bytes / E : 0;
    s = span_of(dtype, n);
    if (s.hi < bytes) s.hi = bytes;
    b = (char *)calloc((size_t)(s.hi - s.lo) + 1, 1);
    for (i = 0; i < DATA_SLOTS; i++)
        if (!g_data[i].origin) {
            g_data[i].origin = b - s.lo;
            g_data[i].base = b;
            return b - s.lo;
        }
    abort();      /* more live buffers than any schedule here needs */
}

static void data_free(void *origin)
{
    int i;
    if (!origin) return;
    for (i = 0; i < DATA_SLOTS; i++)
        if (g_data[i].origin == origin) {
            free(g_data[i].base);
            g_data[i].origin = g_data[i].base = NULL;
            return;
        }
    abort();
}

/* a snapshot of `bytes` (= n * extent) bytes of dtype at src: the whole span */
static char *dup_buf(const void *src, long bytes, int dtype)
{
    int E, TS;
    char *b = data_calloc(bytes, dtype);
    span_t s;
    orc_dtype_info(dtype, &E, &TS);
    s = span_of(dtype, E > 0 ? bytes / E : 0);
    if (s.hi < bytes) s.hi = bytes;
    if (s.hi > s.lo) memcpy(b + s.lo, (const char *)src + s.lo, (size_t)(s.hi - s.lo));
    return b;
}

static void uop(int op, int dtype, const void *in, void *inout, int len,
                int *err)
{
    int e;
    if (!permanent(op)) {     /* user functions report nothing */
        int l = len, t = dtype;
        g_uops[op - 200].fn((void *)in, inout, &l, &t);
        return;
    }
    e = orc_op(op, dtype, in, inout, len);
    if (e) *err = e;
}

int orc_call(int op, int dtype, const void *in, void *inout, int len)
{
    int err = 0;
    if (!op_valid(op)) return ERR_OP;
    uop(op, dtype, in, inout, len, &err);
    return err;
}

/* the noncommutative "order is not right" step: uop(mine, theirs) into a
 * copy of theirs, copied back into mine (5615-5624 and its siblings) */
static void uop_swapped(int op, int dtype, const void *theirs, void *mine, int len,
                        int *err)
{
    int E, TS;
    char *tmp;
    orc_dtype_info(dtype, &E, &TS);
    tmp = dup_buf(theirs, (long)len * E, dtype);
    uop(op, dtype, mine, tmp, len, err);
    tm_copy(mine, tmp, len, dtype);
    data_free(tmp);
}

int orc_algorithm_op(int coll, int p, long total_count, int dtype, int op)
{
    int e, ts, lgn, pof2, tv;
    const int perm = permanent(op), comm = op_valid(op) ? commute(op) : 1;
    if (orc_dtype_info(dtype, &e, &ts)) return ORC_ALG_NONE;
    pof2 = pof2_lgn(p, &lgn);
    if (coll == ORC_COLL_ALLREDUCE) {
        if (total_count == 0) return ORC_ALG_NONE;
        tv = coll_table_flat[ALLREDUCE_IDX * 5 + lgn];
        if (tv == -1 || imul32(total_count, ts) < tv || !perm || total_count < pof2)
            return ORC_ALG_RECDBL;
        return ORC_ALG_RABENSEIFNER;
    }
    if (coll == ORC_COLL_REDUCE) {
        if (total_count == 0) return ORC_ALG_NONE;
        tv = coll_table_flat[REDUCE_IDX * 5 + lgn];
        if (tv != -1 && imul32(total_count, ts) > tv && perm && total_count >= pof2)
            return ORC_ALG_RABENSEIFNER;
        return ORC_ALG_BINOMIAL;
    }
    if (coll == ORC_COLL_REDUCE_SCATTER) {
        const int nbytes = imul32(total_count, ts);
        if (total_count == 0) return ORC_ALG_NONE;
        if (comm && nbytes < REDSCAT_COMMUTATIVE_LONG_MSG) return ORC_ALG_RS_HALVING;
        if (!comm && nbytes < REDSCAT_NONCOMMUTATIVE_SHORT_MSG) return ORC_ALG_RS_RECDBL;
        return ORC_ALG_RS_PAIRWISE;
    }
    return ORC_ALG_NONE;
}

int orc_algorithm(int coll, int p, long total_count, int dtype)
{
    return orc_algorithm_op(coll, p, total_count, dtype, 102);
}

/* ---------------------------------------------------------------------- */
/* _SMP_ builds (ch_gen2 / ch_smp / ch_gen2_ud): collops->Reduce and
 * ->Allreduce are intra_shmem_Reduce / intra_shmem_Allreduce
 * (intra_fns_new.c:293-310).  One node: the shmem group is every rank in
 * rank order, its leader rank 0 (create_2level_comm.c:125-138). */
static struct {
    int smp, enable, ok, dis_red, dis_ar, thr_red, thr_ar;
} g_smp = {0, 1, 1, 0, 0, 1 << 10, 1 << 15};

int orc_smp_set(int smp, int enable, int ok, int dis_red, int dis_ar, int thr_red,
                int thr_ar)
{
    g_smp.smp = smp; g_smp.enable = enable; g_smp.ok = ok;
    g_smp.dis_red = dis_red; g_smp.dis_ar = dis_ar;
    g_smp.thr_red = thr_red; g_smp.thr_ar = thr_ar;
    return 0;
}

/* the leader-path test of 5066-5070 / 5849-5854 (`int stride = count*extent`) */
static int smp_leader(int thr, int disabled, int count, int E, int op)
{
    return g_smp.ok && imul32(count, E) < thr && !disabled && commute(op) && g_smp.enable;
}

/* The leader's gather-and-fold: tmpbuf = a copy of its own sendbuf (5872),
 * every other local rank copies its sendbuf into its shmem slot (5918), and
 * the leader calls (*uop)(slot i, tmpbuf) for i = 1 .. local_size-1
 * (5885-5888; Reduce 5089-5112). */
static char *smp_fold(int p, const void *const *send, int count, int dtype, int op)
{
    int E, TS, i, dummy = 0;
    long bytes;
    char *tmp;
    orc_dtype_info(dtype, &E, &TS);
    bytes = (long)count * E;
    tmp = data_calloc(bytes, dtype);
    tm_copy(tmp, send[0], count, dtype);
    for (i = 1; i < p; i++) {
        char *slot = data_calloc(bytes, dtype);
        tm_copy(slot, send[i], count, dtype);
        uop(op, dtype, slot, tmp, count, &dummy);
        data_free(slot);
    }
    return tmp;
}

/* the len = 0 test every rank makes first for a predefined op (5841-5845,
 * 5054-5058); returns its MPIR_Op_errno */
static int smp_precheck(int op, int dtype, const void *send, void *recv)
{
    return permanent(op) ? orc_op(op, dtype, send, recv, 0) : 0;
}

/* ---------------------------------------------------------------------- */

int orc_allreduce(int p, const void *const *send, void *const *recv,
                  int count, int dtype, int op, int *rc)
{
    int E, TS, r, lgn, pof2, rem, mask, i, alg;
    int *newrank, *err;
    char **snap;
    long bytes;

    if (p <= 0) return 0;
    if (orc_dtype_info(dtype, &E, &TS)) {
        for (r = 0; r < p; r++) rc[r] = ERR_TYPE;
        return 0;
    }
    for (r = 0; r < p; r++) rc[r] = 0;
    if (count < 0) { for (r = 0; r < p; r++) rc[r] = ERR_COUNT; return 0; }
    if (count == 0) return 0;
    if (!op_valid(op)) { for (r = 0; r < p; r++) rc[r] = ERR_OP; return 0; }

    if (g_smp.smp) {   /* intra_shmem_Allreduce, intra_fns_new.c:5793-5940 */
        int e = smp_precheck(op, dtype, send[0], recv[0]);
        if (e) { for (r = 0; r < p; r++) rc[r] = e; return 0; }
        if (smp_leader(g_smp.thr_ar, g_smp.dis_ar, count, E, op)) {
            if (p == 1) tm_copy(recv[0], send[0], count, dtype);          /* 5909-5911 */
            else {
                char *tmp = smp_fold(p, send, count, dtype, op);
                tm_copy(recv[0], tmp, count, dtype);                       /* 5904-5906 */
                data_free(tmp);
                for (r = 1; r < p; r++) tm_copy(recv[r], recv[0], count, dtype);  /* Bcast 5926 */
            }
            return 0;
        }
    }

    bytes = (long)count * E;
    newrank = (int *)calloc((size_t)p, sizeof(int));
    err = (int *)calloc((size_t)p, sizeof(int));
    snap = (char **)calloc((size_t)p, sizeof(char *));

    for (r = 0; r < p; r++) tm_copy(recv[r], send[r], count, dtype);
    pof2 = pof2_lgn(p, &lgn);
    rem = p - pof2;

    /* non-pof2 fold: even ranks < 2*rem hand their data to rank+1 */
    for (r = 0; r < p; r++) {
        if (r < 2 * rem) {
            if (r % 2 == 0) newrank[r] = -1;
            else {
                char *tmp = dup_buf(recv[r - 1], bytes, dtype);
                uop(op, dtype, tmp, recv[r], count, &err[r]);
                data_free(tmp);
                newrank[r] = r / 2;
            }
        } else newrank[r] = r - rem;
    }

    alg = orc_algorithm_op(ORC_COLL_ALLREDUCE, p, count, dtype, op);
#define REAL(nd) (((nd) < rem) ? (nd) * 2 + 1 : (nd) + rem)
    if (alg == ORC_ALG_RECDBL) {
        for (mask = 1; mask < pof2; mask <<= 1) {
            for (r = 0; r < p; r++)
                if (newrank[r] != -1) snap[r] = dup_buf(recv[r], bytes, dtype);
            for (r = 0; r < p; r++) {
                int dst;
                if (newrank[r] == -1) continue;
                dst = REAL(newrank[r] ^ mask);
                if (commute(op) || dst < r) uop(op, dtype, snap[dst], recv[r], count, &err[r]);
                else uop_swapped(op, dtype, snap[dst], recv[r], count, &err[r]);
            }
            for (r = 0; r < p; r++) { data_free(snap[r]); snap[r] = NULL; }
        }
    } else {
        int *cnts = (int *)malloc(sizeof(int) * (size_t)pof2);
        int *disps = (int *)malloc(sizeof(int) * (size_t)pof2);
        int *sidx = (int *)calloc((size_t)p, sizeof(int));
        int *ridx = (int *)calloc((size_t)p, sizeof(int));
        int *lidx = (int *)calloc((size_t)p, sizeof(int));
        int *rcnt = (int *)calloc((size_t)p, sizeof(int));
        for (i = 0; i < pof2 - 1; i++) cnts[i] = count / pof2;
        cnts[pof2 - 1] = count - (count / pof2) * (pof2 - 1);
        disps[0] = 0;
        for (i = 1; i < pof2; i++) disps[i] = disps[i - 1] + cnts[i - 1];
        for (r = 0; r < p; r++) lidx[r] = pof2;

        /* reduce-scatter, recursive halving with distance 1, 2, 4, ... */
        for (mask = 1; mask < pof2; mask <<= 1) {
            for (r = 0; r < p; r++) {
                int nr = newrank[r], nd;
                if (nr == -1) continue;
                nd = nr ^ mask;
                rcnt[r] = 0;
                if (nr < nd) {
                    sidx[r] = ridx[r] + pof2 / (mask * 2);
                    for (i = ridx[r]; i < sidx[r]; i++) rcnt[r] += cnts[i];
                } else {
                    ridx[r] = sidx[r] + pof2 / (mask * 2);
                    for (i = ridx[r]; i < lidx[r]; i++) rcnt[r] += cnts[i];
                }
                snap[r] = dup_buf(recv[r], bytes, dtype);
            }
            for (r = 0; r < p; r++) {
                int dst;
                long off;
                if (newrank[r] == -1) continue;
                dst = REAL(newrank[r] ^ mask);
                off = (long)disps[ridx[r]] * E;
                uop(op, dtype, snap[dst] + off, (char *)recv[r] + off,
                    rcnt[r], &err[r]);
            }
            for (r = 0; r < p; r++) {
                data_free(snap[r]); snap[r] = NULL;
                if (newrank[r] == -1) continue;
                sidx[r] = ridx[r];
                if ((mask << 1) < pof2) lidx[r] = ridx[r] + pof2 / (mask << 1);
            }
        }
        /* allgather by recursive doubling back up */
        for (mask = pof2 >> 1; mask > 0; mask >>= 1) {
            for (r = 0; r < p; r++) {
                int nr = newrank[r], nd;
                if (nr == -1) continue;
                nd = nr ^ mask;
                rcnt[r] = 0;
                if (nr < nd) {
                    if (mask != pof2 / 2) lidx[r] = lidx[r] + pof2 / (mask * 2);
                    ridx[r] = sidx[r] + pof2 / (mask * 2);
                    for (i = ridx[r]; i < lidx[r]; i++) rcnt[r] += cnts[i];
                } else {
                    ridx[r] = sidx[r] - pof2 / (mask * 2);
                    for (i = ridx[r]; i < sidx[r]; i++) rcnt[r] += cnts[i];
                }
                snap[r] = dup_buf(recv[r], bytes, dtype);
            }
            for (r = 0; r < p; r++) {
                int dst;
                long off;
                if (newrank[r] == -1) continue;
                dst = REAL(newrank[r] ^ mask);
                off = (long)disps[ridx[r]] * E;
                tm_copy((char *)recv[r] + off, snap[dst] + off, rcnt[r], dtype);
            }
            for (r = 0; r < p; r++) {
                data_free(snap[r]); snap[r] = NULL;
                if (newrank[r] == -1) continue;
                if (newrank[r] > (newrank[r] ^ mask)) sidx[r] = ridx[r];
            }
        }
        free(cnts); free(disps); free(sidx); free(ridx); free(lidx);
        free(rcnt);
    }
#undef REAL
    /* non-pof2 tail: odd ranks < 2*rem return the result to rank-1 */
    for (r = 0; r < 2 * rem; r += 2) tm_copy(recv[r], recv[r + 1], count, dtype);

    for (r = 0; r < p; r++) rc[r] = err[r];
    free(newrank); free(err); free(snap);
    return 0;
}

/* ---------------------------------------------------------------------- */

int orc_reduce(int p, const void *const *send, void *const *recv,
               int count, int dtype, int op, int root, int *rc)
{
    int E, TS, r, lgn, pof2, rem, mask, i, alg;
    int *err;
    char **wb, **snap;
    long bytes;

    if (p <= 0) return 0;
    if (orc_dtype_info(dtype, &E, &TS)) {
        for (r = 0; r < p; r++) rc[r] = ERR_TYPE;
        return 0;
    }
    for (r = 0; r < p; r++) rc[r] = 0;
    if (count < 0) { for (r = 0; r < p; r++) rc[r] = ERR_COUNT; return 0; }
    if (count == 0) return 0;
    if (root < 0 || root >= p) { for (r = 0; r < p; r++) rc[r] = 7; return 0; }
    if (!op_valid(op)) { for (r = 0; r < p; r++) rc[r] = ERR_OP; return 0; }

    if (g_smp.smp) {   /* intra_shmem_Reduce, intra_fns_new.c:4992-5198 */
        int e = smp_precheck(op, dtype, send[0], recv[0]);
        if (e) { for (r = 0; r < p; r++) rc[r] = e; return 0; }
        if (smp_leader(g_smp.thr_red, g_smp.dis_red, count, E, op)) {
            if (p == 1) tm_copy(recv[root], send[0], count, dtype);       /* 5135-5137 */
            else {
                /* root 0: the leader copies tmpbuf into recvbuf (5129-5131);
                 * otherwise it sends tmpbuf to root (5168-5171, 5179-5181) */
                char *tmp = smp_fold(p, send, count, dtype, op);
                tm_copy(recv[root], tmp, count, dtype);
                data_free(tmp);
            }
            return 0;
        }
    }

    bytes = (long)count * E;
    err = (int *)calloc((size_t)p, sizeof(int));
    wb = (char **)calloc((size_t)p, sizeof(char *));
    snap = (char **)calloc((size_t)p, sizeof(char *));
    /* non-roots reduce into a private buffer (4590-4594) */
    for (r = 0; r < p; r++) {
        wb[r] = (r == root) ? (char *)recv[r] : data_calloc(bytes, dtype);
        tm_copy(wb[r], send[r], count, dtype);
    }
    pof2 = pof2_lgn(p, &lgn);
    alg = orc_algorithm_op(ORC_COLL_REDUCE, p, count, dtype, op);

    if (alg == ORC_ALG_RABENSEIFNER) {
        int *newrank = (int *)calloc((size_t)p, sizeof(int));
        int *cnts = (int *)malloc(sizeof(int) * (size_t)pof2);
        int *disps = (int *)malloc(sizeof(int) * (size_t)pof2);
        int *sidx = (int *)calloc((size_t)p, sizeof(int));
        int *ridx = (int *)calloc((size_t)p, sizeof(int));
        int *lidx = (int *)calloc((size_t)p, sizeof(int));
        int *rcnt = (int *)calloc((size_t)p, sizeof(int));
        int *active = (int *)calloc((size_t)p, sizeof(int));
        int *jj = (int *)calloc((size_t)p, sizeof(int));
        int newroot;
        rem = p - pof2;
#define RREAL(nd) (((nd) < rem) ? (nd) * 2 : (nd) + rem)
        /* fold: odd ranks < 2*rem hand their data to rank-1 */
        for (r = 0; r < p; r++) {
            if (r < 2 * rem) {
                if (r % 2 != 0) newrank[r] = -1;
                else {
                    char *tmp = dup_buf(wb[r + 1], bytes, dtype);
                    uop(op, dtype, tmp, wb[r], count, &err[r]);
                    data_free(tmp);
                    newrank[r] = r / 2;
                }
            } else newrank[r] = r - rem;
        }
        for (i = 0; i < pof2 - 1; i++) cnts[i] = count / pof2;
        cnts[pof2 - 1] = count - (count / pof2) * (pof2 - 1);
        disps[0] = 0;
        for (i = 1; i < pof2; i++) disps[i] = disps[i - 1] + cnts[i - 1];
        for (r = 0; r < p; r++) lidx[r] = pof2;

        for (mask = 1; mask < pof2; mask <<= 1) {
            for (r = 0; r < p; r++) {
                int nr = newrank[r], nd;
                if (nr == -1) continue;
                nd = nr ^ mask;
                rcnt[r] = 0;
                if (nr < nd) {
                    sidx[r] = ridx[r] + pof2 / (mask * 2);
                    for (i = ridx[r]; i < sidx[r]; i++) rcnt[r] += cnts[i];
                } else {
                    ridx[r] = sidx[r] + pof2 / (mask * 2);
                    for (i = ridx[r]; i < lidx[r]; i++) rcnt[r] += cnts[i];
                }
                snap[r] = dup_buf(wb[r], bytes, dtype);
            }
            for (r = 0; r < p; r++) {
                int dst;
                long off;
                if (newrank[r] == -1) continue;
                dst = RREAL(newrank[r] ^ mask);
                off = (long)disps[ridx[r]] * E;
                uop(op, dtype, snap[dst] + off, wb[r] + off, rcnt[r], &err[r]);
            }
            for (r = 0; r < p; r++) {
                data_free(snap[r]); snap[r] = NULL;
                if (newrank[r] == -1) continue;
                sidx[r] = ridx[r];
                if ((mask << 1) < pof2) lidx[r] = ridx[r] + pof2 / (mask << 1);
            }
        }

        /* gather to root */
        if (root < 2 * rem) {
            if (root % 2 != 0) {
                /* root was excluded: newrank 0 (rank 0) hands block 0 over */
                tm_copy(wb[root], wb[0], cnts[0], dtype);
                newrank[root] = 0;
                sidx[root] = 0;
                lidx[root] = 2;
                newrank[0] = -1;
                newroot = 0;
            } else newroot = root / 2;
        } else newroot = root - rem;

        {
            int j0 = 0;
            mask = 1;
            while (mask < pof2) { mask <<= 1; j0++; }
            mask >>= 1;
            j0--;
            for (r = 0; r < p; r++) { active[r] = newrank[r] != -1; jj[r] = j0; }
        }
        for (; mask > 0; mask >>= 1) {
            int *sender = (int *)calloc((size_t)p, sizeof(int));
            int *peer = (int *)calloc((size_t)p, sizeof(int));
            for (r = 0; r < p; r++) {
                int nr, nd, dst, ndtr, nrtr;
                if (!active[r]) continue;
                nr = newrank[r];
                nd = nr ^ mask;
                dst = RREAL(nd);
                if (nd == 0 && root < 2 * rem && root % 2 != 0) dst = root;
                ndtr = (nd >> jj[r]) << jj[r];
                nrtr = (newroot >> jj[r]) << jj[r];
                rcnt[r] = 0;
                if (nr < nd) {
                    if (mask != pof2 / 2) lidx[r] = lidx[r] + pof2 / (mask * 2);
                    ridx[r] = sidx[r] + pof2 / (mask * 2);
                    for (i = ridx[r]; i < lidx[r]; i++) rcnt[r] += cnts[i];
                } else {
                    ridx[r] = sidx[r] - pof2 / (mask * 2);
                    for (i = ridx[r]; i < sidx[r]; i++) rcnt[r] += cnts[i];
                }
                sender[r] = (ndtr == nrtr);
                peer[r] = dst;
            }
            for (r = 0; r < p; r++)
                if (active[r]) snap[r] = dup_buf(wb[r], bytes, dtype);
            for (r = 0; r < p; r++) {
                long off;
                if (!active[r] || sender[r]) continue;
                off = (long)disps[ridx[r]] * E;
                tm_copy(wb[r] + off, snap[peer[r]] + off, rcnt[r], dtype);
            }
            for (r = 0; r < p; r++) {
                data_free(snap[r]); snap[r] = NULL;
                if (!active[r]) continue;
                if (sender[r]) { active[r] = 0; continue; }
                if (newrank[r] > (newrank[r] ^ mask)) sidx[r] = ridx[r];
                jj[r]--;
            }
            free(sender); free(peer);
        }
#undef RREAL
        free(newrank); free(cnts); free(disps); free(sidx); free(ridx);
        free(lidx); free(rcnt); free(active); free(jj);
    } else {
        /* binomial tree relative to lroot: root if commutative, else 0
         * and the result is sent on to root (4908-4909, 4956-4966) */
        const int lroot = commute(op) ? root : 0;
        for (mask = 1; mask < p; mask <<= 1) {
            int *recv_from = (int *)malloc(sizeof(int) * (size_t)p);
            for (r = 0; r < p; r++) {
                int rel = (r - lroot + p) % p, src;
                recv_from[r] = -1;
                /* a rank that already sent has exited: its low bits hold a 1 */
                if (rel & (mask - 1)) continue;
                if ((mask & rel) == 0) {
                    src = rel | mask;
                    if (src < p) recv_from[r] = (src + lroot) % p;
                }
            }
            for (r = 0; r < p; r++)
                if (recv_from[r] >= 0)
                    snap[recv_from[r]] = dup_buf(wb[recv_from[r]], bytes, dtype);
            for (r = 0; r < p; r++) {
                if (recv_from[r] < 0) continue;
                if (commute(op)) uop(op, dtype, snap[recv_from[r]], wb[r], count, &err[r]);
                else uop_swapped(op, dtype, snap[recv_from[r]], wb[r], count, &err[r]);
            }
            for (r = 0; r < p; r++) { data_free(snap[r]); snap[r] = NULL; }
            free(recv_from);
        }
        if (lroot != root) tm_copy(wb[root], wb[0], count, dtype);
    }
    for (r = 0; r < p; r++) {
        rc[r] = err[r];
        if (r != root) data_free(wb[r]);
    }
    free(err); free(wb); free(snap);
    return 0;
}

/* ---------------------------------------------------------------------- */

/* Noncommutative short-message Reduce_scatter, intra_fns_new.c:6505-6706:
 * recursive doubling over the whole vector; each step moves every block but
 * the sender's subtree's (an indexed type of two runs), the subtrees that
 * lack a partner in the non-power-of-two case get the received data
 * forwarded down a halving tree (6598-6650), and the combine is done after
 * the forwarding (6652-6682).  Lockstep: every message of a round is read
 * from the sender's state at the start of that round. */
typedef struct { int len0, len1, dis1; } twoblk;

static twoblk except_subtree(const int *recvcnts, int p, int root, int mask)
{
    twoblk t;
    int j;
    t.len0 = t.len1 = 0;
    for (j = 0; j < root && j < p; j++) t.len0 += recvcnts[j];
    for (j = root + mask; j < p; j++) t.len1 += recvcnts[j];
    t.dis1 = t.len0;
    for (j = root; j < root + mask && j < p; j++) t.dis1 += recvcnts[j];
    return t;
}

static void copy_two(char *dst, const char *src, twoblk t, int E, int dtype)
{
    tm_copy(dst, src, t.len0, dtype);
    tm_copy(dst + (long)t.dis1 * E, src + (long)t.dis1 * E, t.len1, dtype);
}

static void rs_recdbl(int p, const void *const *send, void *const *recv,
                      const int *recvcnts, const int *disps, int total, int dtype,
                      int op, int *err)
{
    int E, TS, r, mask, i;
    long bytes;
    char **res, **tmp, **snap;
    int *received, *dtr, *mtr;
    orc_dtype_info(dtype, &E, &TS);
    bytes = (long)total * E;
    res = (char **)calloc((size_t)p, sizeof(char *));
    tmp = (char **)calloc((size_t)p, sizeof(char *));
    snap = (char **)calloc((size_t)p, sizeof(char *));
    received = (int *)calloc((size_t)p, sizeof(int));
    dtr = (int *)calloc((size_t)p, sizeof(int));
    mtr = (int *)calloc((size_t)p, sizeof(int));
    for (r = 0; r < p; r++) {
        res[r] = data_calloc(bytes, dtype);
        tmp[r] = data_calloc(bytes, dtype);
        tm_copy(res[r], send[r], total, dtype);
    }
    for (mask = 1, i = 0; mask < p; mask <<= 1, i++) {
        int tmask, k, kk;
        for (r = 0; r < p; r++) {
            dtr[r] = ((r ^ mask) >> i) << i;
            mtr[r] = (r >> i) << i;
            received[r] = 0;
        }
        /* the exchange: rank r receives dst's tmp_results minus r's
         * partner subtree (dst's sendtype = r's recvtype) */
        for (r = 0; r < p; r++) snap[r] = dup_buf(res[r], bytes, dtype);
        for (r = 0; r < p; r++) {
            const int dst = r ^ mask;
            if (dst >= p) continue;
            copy_two(tmp[r], snap[dst], except_subtree(recvcnts, p, dtr[r], mask), E, dtype);
            received[r] = 1;
        }
        for (r = 0; r < p; r++) { data_free(snap[r]); snap[r] = NULL; }
        /* forwarding inside subtrees that had no partner */
        for (kk = mask, k = 0; kk; kk >>= 1) k++;
        k--;
        for (tmask = mask >> 1; tmask; tmask >>= 1, k--) {
            for (r = 0; r < p; r++) snap[r] = dup_buf(tmp[r], bytes, dtype);
            for (r = 0; r < p; r++) {
                int dst = r ^ tmask, tree_root, done;
                if (dtr[r] + mask <= p) continue;
                done = p - mtr[r] - mask;
                tree_root = (r >> k) << k;
                if (dst < r && dst < tree_root + done && r >= tree_root + done) {
                    copy_two(tmp[r], snap[dst], except_subtree(recvcnts, p, dtr[r], mask), E, dtype);
                    received[r] = 1;
                }
            }
            for (r = 0; r < p; r++) { data_free(snap[r]); snap[r] = NULL; }
        }
        /* the combine, over the two runs of the recvtype */
        for (r = 0; r < p; r++) {
            twoblk t;
            if (!received[r]) continue;
            t = except_subtree(recvcnts, p, dtr[r], mask);
            if (commute(op) || dtr[r] < mtr[r]) {
                uop(op, dtype, tmp[r], res[r], t.len0, &err[r]);
                uop(op, dtype, tmp[r] + (long)t.dis1 * E, res[r] + (long)t.dis1 * E, t.len1, &err[r]);
            } else {
                uop(op, dtype, res[r], tmp[r], t.len0, &err[r]);
                uop(op, dtype, res[r] + (long)t.dis1 * E, tmp[r] + (long)t.dis1 * E, t.len1, &err[r]);
                copy_two(res[r], tmp[r], t, E, dtype);
            }
        }
    }
    for (r = 0; r < p; r++) {
        if (recvcnts[r]) tm_copy(recv[r], res[r] + (long)disps[r] * E, recvcnts[r], dtype);
        data_free(res[r]); data_free(tmp[r]);
    }
    free(res); free(tmp); free(snap); free(received); free(dtr); free(mtr);
}

int orc_reduce_scatter(int p, const void *const *send, void *const *recv,
                       const int *recvcnts, int dtype, int op, int *rc)
{
    int E, TS, r, i, alg, total = 0;
    int *disps, *err;

    if (p <= 0) return 0;
    if (orc_dtype_info(dtype, &E, &TS)) {
        for (r = 0; r < p; r++) rc[r] = ERR_TYPE;
        return 0;
    }
    for (r = 0; r < p; r++) rc[r] = 0;
    if (!op_valid(op)) { for (r = 0; r < p; r++) rc[r] = ERR_OP; return 0; }
    disps = (int *)malloc(sizeof(int) * (size_t)p);
    err = (int *)calloc((size_t)p, sizeof(int));
    for (i = 0; i < p; i++) { disps[i] = total; total += recvcnts[i]; }
    if (total == 0) { free(disps); free(err); return 0; }

    alg = orc_algorithm_op(ORC_COLL_REDUCE_SCATTER, p, total, dtype, op);
    if (alg == ORC_ALG_RS_HALVING) {
        int lgn, pof2 = pof2_lgn(p, &lgn), rem = p - pof2, mask;
        long bytes = (long)total * E;
        char **res = (char **)calloc((size_t)p, sizeof(char *));
        char **snap = (char **)calloc((size_t)p, sizeof(char *));
        int *newrank = (int *)calloc((size_t)p, sizeof(int));
        int *newcnts = (int *)malloc(sizeof(int) * (size_t)pof2);
        int *newdisps = (int *)malloc(sizeof(int) * (size_t)pof2);
        int *sidx = (int *)calloc((size_t)p, sizeof(int));
        int *ridx = (int *)calloc((size_t)p, sizeof(int));
        int *lidx = (int *)calloc((size_t)p, sizeof(int));
        int *rcnt = (int *)calloc((size_t)p, sizeof(int));
        for (r = 0; r < p; r++) {
            res[r] = data_calloc(bytes, dtype);
            tm_copy(res[r], send[r], total, dtype);
        }
        for (r = 0; r < p; r++) {
            if (r < 2 * rem) {
                if (r % 2 == 0) newrank[r] = -1;
                else {
                    char *tmp = dup_buf(res[r - 1], bytes, dtype);
                    uop(op, dtype, tmp, res[r], total, &err[r]);
                    data_free(tmp);
                    newrank[r] = r / 2;
                }
            } else newrank[r] = r - rem;
        }
        for (i = 0; i < pof2; i++) {
            int old_i = (i < rem) ? i * 2 + 1 : i + rem;
            newcnts[i] = (old_i < 2 * rem) ? recvcnts[old_i] + recvcnts[old_i - 1]
                                           : recvcnts[old_i];
        }
        newdisps[0] = 0;
        for (i = 1; i < pof2; i++) newdisps[i] = newdisps[i - 1] + newcnts[i - 1];
        for (r = 0; r < p; r++) lidx[r] = pof2;

        for (mask = pof2 >> 1; mask > 0; mask >>= 1) {
            for (r = 0; r < p; r++) {
                int nr = newrank[r], nd;
                if (nr == -1) continue;
                nd = nr ^ mask;
                rcnt[r] = 0;
                if (nr < nd) {
                    sidx[r] = ridx[r] + mask;
                    for (i = ridx[r]; i < sidx[r]; i++) rcnt[r] += newcnts[i];
                } else {
                    ridx[r] = sidx[r] + mask;
                    for (i = ridx[r]; i < lidx[r]; i++) rcnt[r] += newcnts[i];
                }
                snap[r] = dup_buf(res[r], bytes, dtype);
            }
            for (r = 0; r < p; r++) {
                int nd, dst;
                long off;
                if (newrank[r] == -1) continue;
                nd = newrank[r] ^ mask;
                dst = (nd < rem) ? nd * 2 + 1 : nd + rem;
                off = (long)newdisps[ridx[r]] * E;
                if (rcnt[r] != 0)
                    uop(op, dtype, snap[dst] + off, res[r] + off, rcnt[r], &err[r]);
            }
            for (r = 0; r < p; r++) {
                data_free(snap[r]); snap[r] = NULL;
                if (newrank[r] == -1) continue;
                sidx[r] = ridx[r];
                lidx[r] = ridx[r] + mask;
            }
        }
        for (r = 0; r < p; r++)
            if (newrank[r] != -1 && recvcnts[r])
                tm_copy(recv[r], res[r] + (long)disps[r] * E, recvcnts[r], dtype);
        for (r = 0; r < 2 * rem; r += 2)
            if (recvcnts[r])
                tm_copy(recv[r], res[r + 1] + (long)disps[r] * E, recvcnts[r], dtype);
        for (r = 0; r < p; r++) data_free(res[r]);
        free(res); free(snap); free(newrank); free(newcnts); free(newdisps);
        free(sidx); free(ridx); free(lidx); free(rcnt);
    } else if (alg == ORC_ALG_RS_PAIRWISE) {
        /* pairwise: rank r folds in block r of rank r-1, r-2, ... */
        for (r = 0; r < p; r++)
            tm_copy(recv[r], (const char *)send[r] + (long)disps[r] * E,
                    recvcnts[r], dtype);
        for (r = 0; r < p; r++) {
            for (i = 1; i < p; i++) {
                int src = (r - i + p) % p;
                long n = recvcnts[r];
                char *tmp = data_calloc(n * E, dtype);
                tm_copy(tmp, (const char *)send[src] + (long)disps[r] * E, n, dtype);
                if (commute(op) || src < r) uop(op, dtype, tmp, recv[r], recvcnts[r], &err[r]);
                else uop_swapped(op, dtype, tmp, recv[r], recvcnts[r], &err[r]);
                data_free(tmp);
            }
        }
    } else {
        rs_recdbl(p, send, recv, recvcnts, disps, total, dtype, op, err);
    }
    for (r = 0; r < p; r++) rc[r] = err[r];
    free(disps); free(err);
    return 0;
}

/* ---------------------------------------------------------------------- */
/* MPIR_intra_Scan, src/coll/intra_scan.c:91-150 (the configured default,
 * intra_fns_new.c:323-331): recursive doubling over partial scans.  Never
 * returns MPIR_Op_errno (no check after the loop). */
int orc_scan(int p, const void *const *send, void *const *recv, int count,
             int dtype, int op, int *rc)
{
    int E, TS, r, mask;
    char **partial, **snap;
    long bytes;
    if (p <= 0) return 0;
    if (orc_dtype_info(dtype, &E, &TS)) { for (r = 0; r < p; r++) rc[r] = ERR_TYPE; return 0; }
    for (r = 0; r < p; r++) rc[r] = 0;
    if (count < 0) { for (r = 0; r < p; r++) rc[r] = ERR_COUNT; return 0; }
    if (count == 0) return 0;
    if (!op_valid(op)) { for (r = 0; r < p; r++) rc[r] = ERR_OP; return 0; }
    bytes = (long)count * E;
    partial = (char **)calloc((size_t)p, sizeof(char *));
    snap = (char **)calloc((size_t)p, sizeof(char *));
    for (r = 0; r < p; r++) {
        tm_copy(recv[r], send[r], count, dtype);
        partial[r] = data_calloc(bytes, dtype);
        tm_copy(partial[r], send[r], count, dtype);
    }
    for (mask = 1; mask < p; mask <<= 1) {
        for (r = 0; r < p; r++) snap[r] = dup_buf(partial[r], bytes, dtype);
        for (r = 0; r < p; r++) {
            int dst = r ^ mask, dummy = 0;
            if (dst >= p) continue;
            if (r > dst) {
                uop(op, dtype, snap[dst], partial[r], count, &dummy);
                uop(op, dtype, snap[dst], recv[r], count, &dummy);
            } else if (commute(op)) {
                uop(op, dtype, snap[dst], partial[r], count, &dummy);
            } else {
                uop_swapped(op, dtype, snap[dst], partial[r], count, &dummy);
            }
        }
        for (r = 0; r < p; r++) { data_free(snap[r]); snap[r] = NULL; }
    }
    for (r = 0; r < p; r++) data_free(partial[r]);
    free(partial); free(snap);
    return 0;
}
