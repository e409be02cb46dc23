/*
 * cpu_coll.c -- TEST INFRASTRUCTURE / CPU BASELINE: the reference's
 * collective schedules run by p host threads (one core per rank) over shared
 * memory, for the CPU baseline of BASELINE.md section 4 (C1 on 2 ranks, the
 * collective analogues on p ranks).  Never linked by the product.
 *
 * Each rank is a thread with its own send / recv / tmp buffers.  A round of
 * the reference's MPI_Sendrecv + (*uop) becomes: every rank copies what it
 * would receive from its partner's buffer into its own tmp (one copy, as a
 * shared-memory device moves a message), a barrier, the (*uop) on its own
 * data (orc_op, the restated global_ops.c loop), a barrier.  Orders, ranges
 * and operand roles are those of intra_fns_new.c (the same as
 * coll_sim.c's lockstep replay, which the tests compare against):
 *   Allreduce  recursive doubling 5592-5629, Rabenseifner 5632-5758
 *   Reduce     binomial tree 4876-4954
 *   Reduce_scatter  recursive halving 6341-6419, pairwise 6450-6503
 * Power-of-two p only (the BASELINE configs: 2, 4, 8).
 */
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include "oracle.h"

#define MAXP 64

typedef struct {
    int p, coll, count, dtype, op, root, reps, alg;
    const int *recvcnts;
    char **send, **recv, **tmp;
    pthread_barrier_t bar;
    int E;
} job_t;

typedef struct { job_t *j; int rank; } arg_t;

static void bar(job_t *j) { pthread_barrier_wait(&j->bar); }

static void allreduce_rank(job_t *j, int r)
{
    const int p = j->p, n = j->count, E = j->E;
    char *rv = j->recv[r], *tp = j->tmp[r];
    int mask;
    memcpy(rv, j->send[r], (size_t)n * E);
    bar(j);
    if (j->alg == ORC_ALG_RECDBL) {
        for (mask = 1; mask < p; mask <<= 1) {
            const int dst = r ^ mask;
            memcpy(tp, j->recv[dst], (size_t)n * E);
            bar(j);
            orc_op(j->op, j->dtype, tp, rv, n);
            bar(j);
        }
        return;
    }
    {   /* Rabenseifner: halving with distance 1, 2, ..., then doubling back */
        int cnts[MAXP], disps[MAXP], i, sidx = 0, ridx = 0, lidx = p;
        for (i = 0; i < p - 1; i++) cnts[i] = n / p;
        cnts[p - 1] = n - (n / p) * (p - 1);
        disps[0] = 0;
        for (i = 1; i < p; i++) disps[i] = disps[i - 1] + cnts[i - 1];
        for (mask = 1; mask < p; mask <<= 1) {
            const int dst = r ^ mask;
            int rc = 0;
            if (r < dst) {
                sidx = ridx + p / (mask * 2);
                for (i = ridx; i < sidx; i++) rc += cnts[i];
            } else {
                ridx = sidx + p / (mask * 2);
                for (i = ridx; i < lidx; i++) rc += cnts[i];
            }
            memcpy(tp + (size_t)disps[ridx] * E, j->recv[dst] + (size_t)disps[ridx] * E, (size_t)rc * E);
            bar(j);
            orc_op(j->op, j->dtype, tp + (size_t)disps[ridx] * E, rv + (size_t)disps[ridx] * E, rc);
            bar(j);
            sidx = ridx;
            if ((mask << 1) < p) lidx = ridx + p / (mask << 1);
        }
        for (mask = p >> 1; mask > 0; mask >>= 1) {
            const int dst = r ^ mask;
            int rc = 0;
            if (r < dst) {
                if (mask != p / 2) lidx = lidx + p / (mask * 2);
                ridx = sidx + p / (mask * 2);
                for (i = ridx; i < lidx; i++) rc += cnts[i];
            } else {
                ridx = sidx - p / (mask * 2);
                for (i = ridx; i < sidx; i++) rc += cnts[i];
            }
            memcpy(tp, j->recv[dst] + (size_t)disps[ridx] * E, (size_t)rc * E);
            bar(j);
            memcpy(rv + (size_t)disps[ridx] * E, tp, (size_t)rc * E);
            bar(j);
            if (r > dst) sidx = ridx;
        }
    }
}

static void reduce_rank(job_t *j, int r)   /* binomial tree, commutative, root-relative */
{
    const int p = j->p, n = j->count, E = j->E, rel = (r - j->root + p) % p;
    char *rv = j->recv[r], *tp = j->tmp[r];
    int mask, done = 0;
    memcpy(rv, j->send[r], (size_t)n * E);
    bar(j);
    for (mask = 1; mask < p; mask <<= 1) {
        int src = -1;
        if (!done) {
            if (rel & mask) done = 1;                  /* sent to the parent: idle */
            else if ((rel | mask) < p) src = ((rel | mask) + j->root) % p;
        }
        if (src >= 0) memcpy(tp, j->recv[src], (size_t)n * E);
        bar(j);
        if (src >= 0) orc_op(j->op, j->dtype, tp, rv, n);
        bar(j);
    }
}

static void reduce_scatter_rank(job_t *j, int r)
{
    const int p = j->p, E = j->E;
    int disps[MAXP], i, total = 0;
    for (i = 0; i < p; i++) { disps[i] = total; total += j->recvcnts[i]; }
    if (j->alg == ORC_ALG_RS_PAIRWISE) {           /* 6450-6503 */
        const int my = j->recvcnts[r];
        memcpy(j->recv[r], j->send[r] + (size_t)disps[r] * E, (size_t)my * E);
        for (i = 1; i < p; i++) {
            const int src = (r - i + p) % p;
            memcpy(j->tmp[r], j->send[src] + (size_t)disps[r] * E, (size_t)my * E);
            orc_op(j->op, j->dtype, j->tmp[r], j->recv[r], my);
        }
        bar(j);
        return;
    }
    {   /* recursive halving, distance p/2 ... 1, on a full-size copy */
        char *res = j->tmp[r] + (size_t)total * E;     /* tmp holds 2 x total */
        int mask, sidx = 0, ridx = 0, lidx = p;
        memcpy(res, j->send[r], (size_t)total * E);
        bar(j);
        for (mask = p >> 1; mask > 0; mask >>= 1) {
            const int dst = r ^ mask;
            char *dres = j->tmp[dst] + (size_t)total * E;
            int rc = 0;
            if (r < dst) {
                sidx = ridx + mask;
                for (i = ridx; i < sidx; i++) rc += j->recvcnts[i];
            } else {
                ridx = sidx + mask;
                for (i = ridx; i < lidx; i++) rc += j->recvcnts[i];
            }
            memcpy(j->tmp[r], dres + (size_t)disps[ridx] * E, (size_t)rc * E);
            bar(j);
            if (rc) orc_op(j->op, j->dtype, j->tmp[r], res + (size_t)disps[ridx] * E, rc);
            bar(j);
            sidx = ridx;
            lidx = ridx + mask;
        }
        memcpy(j->recv[r], res + (size_t)disps[r] * E, (size_t)j->recvcnts[r] * E);
    }
}

static void *thread_main(void *v)
{
    arg_t *a = (arg_t *)v;
    job_t *j = a->j;
    int k;
    for (k = 0; k < j->reps; k++) {
        if (j->coll == ORC_COLL_ALLREDUCE) allreduce_rank(j, a->rank);
        else if (j->coll == ORC_COLL_REDUCE) reduce_rank(j, a->rank);
        else reduce_scatter_rank(j, a->rank);
        bar(j);
    }
    return NULL;
}

/* Runs `reps` back-to-back collectives with p threads; returns seconds per
 * collective (wall clock), or a negative value on a bad argument.  recv[r]
 * receives rank r's result.  tmp[r] must hold 2 x total elements. */
double orc_threads_coll(int coll, int p, void *const *send, void *const *recv, void *const *tmp,
                        int count, const int *recvcnts, int dtype, int op, int root, int reps)
{
    job_t j;
    arg_t args[MAXP];
    pthread_t th[MAXP];
    struct timespec t0, t1;
    int r, e, s, total = count;
    if (p < 1 || p > MAXP || (p & (p - 1)) || reps < 1 || orc_dtype_info(dtype, &e, &s)) return -1.0;
    memset(&j, 0, sizeof j);
    j.p = p; j.coll = coll; j.count = count; j.dtype = dtype; j.op = op; j.root = root;
    j.reps = reps; j.recvcnts = recvcnts; j.E = e;
    j.send = (char **)send; j.recv = (char **)recv; j.tmp = (char **)tmp;
    if (coll == ORC_COLL_REDUCE_SCATTER) {
        total = 0;
        for (r = 0; r < p; r++) total += recvcnts[r];
    }
    j.alg = orc_algorithm(coll, p, total, dtype);
    if (coll == ORC_COLL_REDUCE && j.alg != ORC_ALG_BINOMIAL) return -2.0;   /* not restated here */
    pthread_barrier_init(&j.bar, NULL, (unsigned)p);
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (r = 0; r < p; r++) {
        args[r].j = &j; args[r].rank = r;
        pthread_create(&th[r], NULL, thread_main, &args[r]);
    }
    for (r = 0; r < p; r++) pthread_join(th[r], NULL);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    pthread_barrier_destroy(&j.bar);
    return ((double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec)) / reps;
}
