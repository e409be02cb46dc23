/* harness.c -- TEST HELPER: a one-process stand-in for the MPICH runtime
 * calls integration/intra_mvx.c makes (MPIR_ToPointer, attributes,
 * MPIR_intra_collops, MPIR_COMM_WORLD), so tests/test_cpu_integration.py and
 * tests/test_gpu_integration.py can drive the shim's collops table through
 * ctypes.  Compile-check headers: integration/check/README.md.
 *
 * Datatype nodes are built the way the reference's constructors store them
 * (field values supplied by the test from the oracle's restated bounds);
 * MPIR_intra_collops, standing for MVAPICH's own (host) path, counts its
 * calls and, for a one-rank communicator, copies sendbuf to recvbuf. */
#include <stdlib.h>
#include <string.h>

#include "mpiimpl.h"
#include "mpiops.h"
#include "mpicoll.h"

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
static int g_host_calls;
static struct MPIR_COMMUNICATOR g_world;
struct MPIR_COMMUNICATOR *MPIR_COMM_WORLD = &g_world;

static void host_copy(void *s, void *r, long n, struct MPIR_DATATYPE *d)
{
    if (s != r && n > 0) memcpy(r, s, (size_t)(n * d->extent));
}
static int host_bcast(void *b, int n, struct MPIR_DATATYPE *d, int root, struct MPIR_COMMUNICATOR *c)
{
    (void)b; (void)n; (void)d; (void)root;
    return c->np == 1 ? MPI_SUCCESS : MPI_ERR_OTHER;
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
    (void)op; (void)c;
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

#ifdef HARNESS_SMP
int enable_shmem_collectives = 1;     /* src/env/initutil.c:146 */
#endif
MPI_Fint MPIR_F_TRUE = 1, MPIR_F_FALSE = 0;   /* initfutil.c:100, gfortran's literals */

/* one-rank world, the shim's table installed */
int h_init(void)
{
    g_world.np = 1;
    g_world.local_rank = 0;
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
