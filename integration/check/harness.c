/* harness.c -- TEST HELPER: a stand-in for the MPICH runtime calls
 * integration/intra_mvx.c makes (MPIR_ToPointer, attributes,
 * MPIR_intra_collops, MPIR_COMM_WORLD), so tests/test_cpu_integration.py and
 * tests/test_gpu_integration.py can drive the shim's collops table through
 * ctypes.  Compile-check headers: integration/check/README.md.
 *
 * Datatype nodes are built the way the reference's constructors store them
 * (field values supplied by the test from the oracle's restated bounds);
 * MPIR_intra_collops, standing for MVAPICH's own (host) path, counts its
 * calls and, for a one-rank communicator, copies sendbuf to recvbuf.
 *
 * World of np processes (h_init_world): each process is one rank of
 * MPI_COMM_WORLD; the stand-in's Bcast and its Allreduce of a few MPI_INTs
 * (the shim's route and creation agreements, counted apart from the data
 * calls) move their bytes through a board in a file every rank maps, with a
 * time limit so a rank that never arrives fails the call instead of hanging
 * the test.  The route agreement's ints are kept for the test to read
 * (h_last_route), and a CPU test may declare ranges device memory
 * (h_fake_device: the build routes the shim's device test here). */
#include <stdlib.h>
#include <string.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <time.h>
#include <unistd.h>

#include "mpiimpl.h"
#include "mpiops.h"
#include "mpicoll.h"

/* the build renames the shim's device test to h_buffer_is_device (Makefile);
 * libmvx's own test under its real name */
#undef mvx_buffer_is_device
int mvx_buffer_is_device(const void *p);

extern MPIR_COLLOPS MPIR_mvx_collops;
void MPIR_mvx_collops_init(void);
int mvx_shim_type(struct MPIR_DATATYPE *d, int *out);
int mvx_shim_op(MPI_Op op, int *out);

/* ---- handles ------------------------------------------------------------ */
#define NPTR 4096
static void *g_ptr[NPTR];
static int g_next = 1000;          /* above every predefined handle */

void *MPIR_ToPointer(int idx) { return idx >= 0 && idx < NPTR ? g_ptr[idx] : NULL; }

static int new_handle(void *p)
{
    if (g_next >= NPTR) return -1;
    g_ptr[g_next] = p;
    return g_next++;
}

/* ---- attributes (one value per (comm, keyval)) -------------------------- */
#define NATTR 64
static struct { int comm, key; void *val; } g_attr[NATTR];
static int g_nattr, g_nkey;
static MPI_Delete_function *g_del[16];

int MPIR_null_copy_fn(MPI_Comm c, int k, void *e, void *in, void *out, int *flag)
{
    (void)c; (void)k; (void)e; (void)in; (void)out;
    *flag = 0;
    return MPI_SUCCESS;
}

int MPI_Keyval_create(MPI_Copy_function *copy, MPI_Delete_function *del, int *keyval, void *extra)
{
    (void)copy; (void)extra;
    if (g_nkey >= 15) return MPI_ERR_OTHER;
    g_del[++g_nkey] = del;
    *keyval = g_nkey;
    return MPI_SUCCESS;
}

int MPI_Attr_put(MPI_Comm comm, int key, void *val)
{
    int i;
    for (i = 0; i < g_nattr; i++)
        if (g_attr[i].comm == comm && g_attr[i].key == key) break;
    if (i == g_nattr) {
        if (g_nattr == NATTR) return MPI_ERR_OTHER;
        g_nattr++;
    }
    g_attr[i].comm = comm;
    g_attr[i].key = key;
    g_attr[i].val = val;
    return MPI_SUCCESS;
}

int MPI_Attr_get(MPI_Comm comm, int key, void *val, int *flag)
{
    int i;
    *flag = 0;
    for (i = 0; i < g_nattr; i++)
        if (g_attr[i].comm == comm && g_attr[i].key == key) {
            *(void **)val = g_attr[i].val;
            *flag = 1;
        }
    return MPI_SUCCESS;
}

/* MPI_Comm_free's attribute deletion (attr_util.c): run the delete callbacks */
int h_comm_free_attrs(int comm)
{
    int i, n = 0;
    for (i = 0; i < g_nattr; i++)
        if (g_attr[i].comm == comm && g_del[g_attr[i].key]) {
            g_del[g_attr[i].key](comm, g_attr[i].key, g_attr[i].val, NULL);
            g_attr[i] = g_attr[--g_nattr];
            i--;
            n++;
        }
    return n;
}

/* ---- the host path ("MVAPICH's own") ------------------------------------ */
static int g_host_calls, g_agree_calls;
static struct MPIR_COMMUNICATOR g_world;
struct MPIR_COMMUNICATOR *MPIR_COMM_WORLD = &g_world;

/* the board: slot[r][g & 1] holds rank r's bytes of exchange g; arrive[r] =
 * the last exchange rank r has written.  Double-buffered by parity: a rank
 * writing exchange g + 2 has seen every rank arrive at g + 1, so each has
 * read exchange g. */
#define BOARD_RANKS 16
#define BOARD_SLOT 256
typedef struct {
    volatile long arrive[BOARD_RANKS];
    char slot[BOARD_RANKS][2][BOARD_SLOT];
} board_t;
static board_t *g_board;
static long g_gen;
static double g_limit_s = 60.0;

static double now_s(void)
{
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

/* every rank's `bytes` (<= BOARD_SLOT) of this exchange into out[r * bytes] */
static int board_allgather(const void *mine, int bytes, void *out)
{
    const int np = g_world.np, me = g_world.local_rank;
    const long g = ++g_gen;
    const double t0 = now_s();
    int r;
    if (!g_board || bytes > BOARD_SLOT) return MPI_ERR_OTHER;
    memcpy(g_board->slot[me][g & 1], mine, (size_t)bytes);
    __atomic_store_n(&g_board->arrive[me], g, __ATOMIC_RELEASE);
    for (r = 0; r < np; r++) {
        while (__atomic_load_n(&g_board->arrive[r], __ATOMIC_ACQUIRE) < g) {
            /* poll: spin for the first 100 us (a peer that is about to
             * arrive), then sleep 20 us between looks */
            struct timespec ts = {0, 20000};
            const double waited = now_s() - t0;
            if (waited > g_limit_s) return MPI_ERR_OTHER;
            if (waited > 1e-4) nanosleep(&ts, NULL);
        }
        memcpy((char *)out + (size_t)r * bytes, g_board->slot[r][g & 1], (size_t)bytes);
    }
    return MPI_SUCCESS;
}

static void host_copy(void *s, void *r, long n, struct MPIR_DATATYPE *d)
{
    if (s != r && n > 0) memcpy(r, s, (size_t)(n * d->extent));
}
static int host_bcast(void *b, int n, struct MPIR_DATATYPE *d, int root, struct MPIR_COMMUNICATOR *c)
{
    char all[BOARD_RANKS * BOARD_SLOT];
    const long bytes = (long)n * d->extent;
    if (c->np == 1) return MPI_SUCCESS;
    if (bytes > BOARD_SLOT || board_allgather(b, (int)bytes, all)) return MPI_ERR_OTHER;
    memcpy(b, all + (size_t)root * (size_t)bytes, (size_t)bytes);
    return MPI_SUCCESS;
}

/* the shim's agreements: an Allreduce of at most 4 MPI_INTs with MPI_MAX or
 * MPI_MIN, reduced for real across the world's ranks */
static int agreement(int n, struct MPIR_DATATYPE *d, MPI_Op op)
{
    return d->self == MPI_INT && n >= 1 && n <= 4 && (op == MPI_MAX || op == MPI_MIN);
}

/* the last route agreement (three ints): this rank's and the reduced ones */
static int g_route_n, g_route_mine[4], g_route_all[4];

static int host_agree(const int *s, int *r, int n, MPI_Op op, struct MPIR_COMMUNICATOR *c)
{
    int all[BOARD_RANKS * 4], i, q;
    g_agree_calls++;
    if (c->np == 1) {
        memcpy(r, s, (size_t)n * sizeof(int));
    } else {
        if (board_allgather(s, n * (int)sizeof(int), all)) return MPI_ERR_OTHER;
        for (i = 0; i < n; i++) {
            r[i] = all[i];
            for (q = 1; q < c->np; q++) {
                const int v = all[q * n + i];
                if (op == MPI_MAX ? v > r[i] : v < r[i]) r[i] = v;
            }
        }
    }
    if (n == 3) {
        g_route_n++;
        memcpy(g_route_mine, s, 3 * sizeof(int));
        memcpy(g_route_all, r, 3 * sizeof(int));
    }
    return MPI_SUCCESS;
}

/* the last route agreement's ints (mine[3], all[3]); returns how many route
 * agreements there have been */
int h_last_route(int *mine, int *all)
{
    memcpy(mine, g_route_mine, 3 * sizeof(int));
    memcpy(all, g_route_all, 3 * sizeof(int));
    return g_route_n;
}

/* ---- buffer kinds ------------------------------------------------------- */
/* ranges a CPU test declares device memory (no GPU here); anything else is
 * what libmvx says */
#define NFAKE 16
static struct { const char *p; long n; } g_fake[NFAKE];

int h_fake_device(const void *p, long bytes)
{
    int i;
    for (i = 0; i < NFAKE; i++)
        if (!g_fake[i].p) {
            g_fake[i].p = (const char *)p;
            g_fake[i].n = bytes;
            return 0;
        }
    return 1;
}

void h_fake_device_clear(void) { memset(g_fake, 0, sizeof g_fake); }

int h_buffer_is_device(const void *p)
{
    int i;
    for (i = 0; i < NFAKE; i++)
        if (g_fake[i].p && (const char *)p >= g_fake[i].p && (const char *)p < g_fake[i].p + g_fake[i].n) return 1;
    return mvx_buffer_is_device(p);
}
static int host_reduce(void *s, void *r, int n, struct MPIR_DATATYPE *d, MPI_Op op, int root,
                    struct MPIR_COMMUNICATOR *c)
{
    (void)op; (void)root; (void)c;
    g_host_calls++;
    host_copy(s, r, n, d);
    return MPI_SUCCESS;
}
static int host_allreduce(void *s, void *r, int n, struct MPIR_DATATYPE *d, MPI_Op op,
                       struct MPIR_COMMUNICATOR *c)
{
    if (agreement(n, d, op)) return host_agree((const int *)s, (int *)r, n, op, c);
    g_host_calls++;
    host_copy(s, r, n, d);
    return MPI_SUCCESS;
}
static int host_reduce_scatter(void *s, void *r, int *cnts, struct MPIR_DATATYPE *d, MPI_Op op,
                            struct MPIR_COMMUNICATOR *c)
{
    (void)op; (void)c;
    g_host_calls++;
    host_copy(s, r, cnts[0], d);
    return MPI_SUCCESS;
}
static struct _MPIR_COLLOPS g_intra = {
    .Bcast = host_bcast, .Reduce = host_reduce, .Allreduce = host_allreduce,
    .Reduce_scatter = host_reduce_scatter, .Scan = host_allreduce, .ref_count = 1,
};
MPIR_COLLOPS MPIR_intra_collops = &g_intra;
MPIR_COLLOPS MPIR_inter_collops = &g_intra;

int h_host_calls(void) { return g_host_calls; }
int h_agree_calls(void) { return g_agree_calls; }

#ifdef HARNESS_SMP
int enable_shmem_collectives = 1;     /* src/env/initutil.c:146 */
#endif
MPI_Fint MPIR_F_TRUE = 1, MPIR_F_FALSE = 0;   /* initfutil.c:100, gfortran's literals */

static int the_world(int rank, int np);

/* one-rank world, the shim's table installed */
int h_init(void) { return the_world(0, 1); }

/* rank `rank` of an np-process world whose board is the file `path` (every
 * rank passes the same path; the test creates it, zero-filled, beforehand);
 * limit_s bounds each board exchange */
int h_init_world(int rank, int np, const char *path, double limit_s)
{
    int fd;
    void *m;
    if (np < 1 || np > BOARD_RANKS || rank < 0 || rank >= np) return 1;
    fd = open(path, O_RDWR);
    if (fd < 0) return 1;
    if (ftruncate(fd, sizeof(board_t))) { close(fd); return 1; }
    m = mmap(NULL, sizeof(board_t), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (m == MAP_FAILED) return 1;
    g_board = (board_t *)m;
    if (limit_s > 0) g_limit_s = limit_s;
    return the_world(rank, np);
}

static int the_world(int rank, int np)
{
    /* the predefined types the shim's own calls name (MPI_INT, MPI_BYTE) */
    static struct MPIR_DATATYPE t_int, t_byte;
    t_int.dte_type = MPIR_INT; t_int.basic = t_int.permanent = 1; t_int.self = MPI_INT;
    t_int.extent = t_int.ub = t_int.size = 4;
    t_byte.dte_type = MPIR_BYTE; t_byte.basic = t_byte.permanent = 1; t_byte.self = MPI_BYTE;
    t_byte.extent = t_byte.ub = t_byte.size = 1;
    if (!g_ptr[MPI_INT]) g_ptr[MPI_INT] = &t_int;
    if (!g_ptr[MPI_BYTE]) g_ptr[MPI_BYTE] = &t_byte;
    g_world.np = np;
    g_world.local_rank = rank;
    g_world.self = 91;             /* MPI_COMM_WORLD, mpi.h:119 */
    g_world.comm_type = 1;         /* MPIR_INTRA */
    g_world.comm_coll = &g_world;
    g_ptr[91] = &g_world;
    MPIR_mvx_collops_init();
    g_world.collops = MPIR_mvx_collops;
    return MPIR_mvx_collops != NULL && MPIR_mvx_collops->Bcast == g_intra.Bcast ? 0 : 1;
}

/* ---- datatype nodes, as type_*.c store them ----------------------------- */
static struct MPIR_DATATYPE *node(MPIR_NODETYPE k, long lb, long ub, long extent, long size)
{
    struct MPIR_DATATYPE *d = (struct MPIR_DATATYPE *)calloc(1, sizeof *d);
    d->dte_type = k;
    d->lb = lb;
    d->ub = ub;
    d->extent = extent;
    d->size = (int)size;
    d->self = new_handle(d);
    return d;
}

/* a predefined type (permanent, handle = the reference's) */
void *h_basic(int handle, long lb, long ub, long extent, long size)
{
    struct MPIR_DATATYPE *d = (struct MPIR_DATATYPE *)calloc(1, sizeof *d);
    d->dte_type = MPIR_INT;
    d->basic = d->permanent = 1;
    d->lb = lb;
    d->ub = ub;
    d->extent = extent;
    d->size = (int)size;
    d->self = handle;
    g_ptr[handle] = d;
    return d;
}

void *h_contig(int count, void *old, long lb, long ub, long extent, long size)
{
    struct MPIR_DATATYPE *d = node(MPIR_CONTIG, lb, ub, extent, size);
    d->count = count;
    d->old_type = (struct MPIR_DATATYPE *)old;
    return d;
}

void *h_hvector(int count, int blocklen, long stride, void *old, long lb, long ub, long extent,
                long size)
{
    struct MPIR_DATATYPE *d = node(MPIR_HVECTOR, lb, ub, extent, size);
    d->count = count;
    d->blocklen = blocklen;
    d->stride = stride;
    d->old_type = (struct MPIR_DATATYPE *)old;
    return d;
}

void *h_hindexed(int count, const int *bl, const long *idx, void *old, long lb, long ub,
                 long extent, long size)
{
    struct MPIR_DATATYPE *d = node(MPIR_HINDEXED, lb, ub, extent, size);
    int i;
    d->count = count;
    d->blocklens = (int *)malloc((size_t)(count ? count : 1) * sizeof(int));
    d->indices = (MPI_Aint *)malloc((size_t)(count ? count : 1) * sizeof(MPI_Aint));
    for (i = 0; i < count; i++) {
        d->blocklens[i] = bl[i];
        d->indices[i] = idx[i];
    }
    d->old_type = (struct MPIR_DATATYPE *)old;
    return d;
}

void *h_struct(int count, const int *bl, const long *idx, void *const *olds, long lb, long ub,
               long extent, long size)
{
    struct MPIR_DATATYPE *d = node(MPIR_STRUCT, lb, ub, extent, size);
    int i;
    d->count = count;
    d->blocklens = (int *)malloc((size_t)(count ? count : 1) * sizeof(int));
    d->indices = (MPI_Aint *)malloc((size_t)(count ? count : 1) * sizeof(MPI_Aint));
    d->old_types = (struct MPIR_DATATYPE **)malloc((size_t)(count ? count : 1) * sizeof(void *));
    for (i = 0; i < count; i++) {
        d->blocklens[i] = bl[i];
        d->indices[i] = idx[i];
        d->old_types[i] = (struct MPIR_DATATYPE *)olds[i];
    }
    return d;
}

int h_self(void *d) { return ((struct MPIR_DATATYPE *)d)->self; }
int h_translate(void *d, int *out) { return mvx_shim_type((struct MPIR_DATATYPE *)d, out); }

/* ---- ops ---------------------------------------------------------------- */
static int g_seen_type;
int h_seen_type(void) { return g_seen_type; }

/* int sum that records the datatype handle it was given */
static void uop_isum(void *in, void *inout, int *len, MPI_Datatype *dt)
{
    int i;
    g_seen_type = *dt;
    for (i = 0; i < *len; i++) ((int *)inout)[i] += ((int *)in)[i];
}

int h_op_create(int commute)
{
    struct MPIR_OP *o = (struct MPIR_OP *)calloc(1, sizeof *o);
    o->op = uop_isum;
    o->commute = commute;
    return new_handle(o);
}

int h_op_translate(int op, int *out) { return mvx_shim_op(op, out); }

/* ---- the collops members, as MPI_Allreduce & co. call them -------------- */
int h_allreduce(void *s, void *r, int n, void *d, int op)
{
    return g_world.collops->Allreduce(s, r, n, (struct MPIR_DATATYPE *)d, op, &g_world);
}
int h_reduce(void *s, void *r, int n, void *d, int op, int root)
{
    return g_world.collops->Reduce(s, r, n, (struct MPIR_DATATYPE *)d, op, root, &g_world);
}
int h_reduce_scatter(void *s, void *r, int *cnts, void *d, int op)
{
    return g_world.collops->Reduce_scatter(s, r, cnts, (struct MPIR_DATATYPE *)d, op, &g_world);
}
int h_scan(void *s, void *r, int n, void *d, int op)
{
    return g_world.collops->Scan(s, r, n, (struct MPIR_DATATYPE *)d, op, &g_world);
}
