/*
 * mvx_opreg.c -- the MPI_Op registry (struct MPIR_OP, include/mpiops.h:1-11;
 * MPI_Op_create / MPI_Op_free, src/coll/opcreate.c:62-76, opfree.c:51-82),
 * the datatype constructors over libmvx_hip.so's type engine
 * (src/pt2pt/type_*.c), and the handles user functions are given.
 */
#include <string.h>

#include "mvx_internal.h"

#define MAX_USER_OPS 64
#define USER_OP_BASE 200
#define OP_COOKIE 0xca01beafu
static mvx_op_t g_user_ops[MAX_USER_OPS];

int mvxi_predefined(MPI_Op op) { return op >= MPI_MAX && op <= MPI_MAXLOC; }

mvx_op_t *mvxi_user_op(MPI_Op op)
{
    int i = op - USER_OP_BASE;
    if (i < 0 || i >= MAX_USER_OPS || g_user_ops[i].cookie != OP_COOKIE) return NULL;
    return &g_user_ops[i];
}

static int op_register(MPI_User_function *fn, MVX_Device_function *dfn, int commute, MPI_Op *op)
{
    int i;
    if (!op) return MPI_ERR_ARG;
    for (i = 0; i < MAX_USER_OPS; i++) {
        if (g_user_ops[i].cookie != OP_COOKIE) {
            g_user_ops[i].op = fn;
            g_user_ops[i].dop = dfn;
            g_user_ops[i].cookie = OP_COOKIE;
            g_user_ops[i].commute = commute;
            g_user_ops[i].permanent = 0;
            *op = USER_OP_BASE + i;
            return MPI_SUCCESS;
        }
    }
    return MPI_ERR_INTERN;
}

int MPI_Op_create(MPI_User_function *function, int commute, MPI_Op *op)
{
    return op_register(function, NULL, commute, op);
}

int mvx_op_create(MPI_User_function *function, int commute, MPI_Op *op)
{
    return op_register(function, NULL, commute, op);
}

int mvx_op_create_device(MVX_Device_function *function, int commute, MPI_Op *op)
{
    if (!function) return MPI_ERR_ARG;
    return op_register(NULL, function, commute, op);
}

int MPI_Op_free(MPI_Op *op)  /* opfree.c:51-82 */
{
    mvx_op_t *o;
    if (!op) return MPI_ERR_ARG;
    if (*op == MPI_OP_NULL) return MVX_ERR_OP_NULL;
    if (mvxi_predefined(*op)) return MVX_ERR_PERM_OP;
    o = mvxi_user_op(*op);
    if (!o) return MPI_ERR_OP;
    memset(o, 0, sizeof *o);
    *op = MPI_OP_NULL;
    return MPI_SUCCESS;
}

int mvx_op_free(MPI_Op *op) { return MPI_Op_free(op); }

/* the plan kind of an op handle (an invalid handle plans as predefined and
 * is rejected by mvxi_op_verdict) */
int mvxi_op_kind(MPI_Op op)
{
    const mvx_op_t *o = mvxi_predefined(op) ? NULL : mvxi_user_op(op);
    if (!o) return MVX_OPKIND_PREDEFINED;
    return o->commute ? MVX_OPKIND_USER_COMMUTE : MVX_OPKIND_USER_NONCOMMUTE;
}

/* The op's verdict on (op, type) before any data moves: 0, 329 (undefined
 * pair, reported only by ranks that call the op), MPI_ERR_OP (bad handle).
 * A user function accepts every datatype (the reference never checks). */
int mvxi_op_verdict(MPI_Op op, MPI_Datatype dt)
{
    if (mvxi_predefined(op)) return mvx_op_apply(op, dt, NULL, NULL, 0, NULL);
    return mvxi_user_op(op) ? MPI_SUCCESS : MPI_ERR_OP;
}

int mvxi_is_device_ptr(const void *p)
{
    hipPointerAttribute_t a;
    if (!p) return 0;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    return a.type == hipMemoryTypeDevice || a.isManaged;
}

int mvx_buffer_is_device(const void *p) { return mvxi_is_device_ptr(p); }

/* ---- derived datatypes (the table is libmvx_hip.so's) ------------------ */

/* the type engine's codes: a negative value is MVX_SETMSG(class, kind), a
 * code the reference makes with MPIR_Err_setmsg (error ring position added) */
static int type_rc(int rc)
{
    if (rc >= 0) return rc;
    rc = -rc;
    return mvxi_setmsg_code(rc & ((1 << MVX_ERR_CLASS_BITS) - 1), rc >> MVX_ERR_CLASS_BITS);
}

int MPI_Type_contiguous(int count, MPI_Datatype old, MPI_Datatype *newtype)
{
    return type_rc(mvx_type_contiguous(count, old, newtype));
}

int MPI_Type_vector(int count, int blocklen, int stride, MPI_Datatype old, MPI_Datatype *newtype)
{
    return type_rc(mvx_type_vector(count, blocklen, stride, old, newtype));
}

int MPI_Type_hvector(int count, int blocklen, MPI_Aint stride, MPI_Datatype old, MPI_Datatype *newtype)
{
    return type_rc(mvx_type_hvector(count, blocklen, stride, old, newtype));
}

int MPI_Type_indexed(int count, int *blocklens, int *indices, MPI_Datatype old, MPI_Datatype *newtype)
{
    return type_rc(mvx_type_indexed(count, blocklens, indices, old, newtype));
}

int MPI_Type_hindexed(int count, int *blocklens, MPI_Aint *indices, MPI_Datatype old, MPI_Datatype *newtype)
{
    return type_rc(mvx_type_hindexed(count, blocklens, indices, old, newtype));
}

int MPI_Type_struct(int count, int *blocklens, MPI_Aint *indices, MPI_Datatype *types, MPI_Datatype *newtype)
{
    return type_rc(mvx_type_struct(count, blocklens, indices, types, newtype));
}

int MPI_Type_commit(MPI_Datatype *datatype)   /* type_commit.c:41-143 */
{
    if (!datatype) return MVX_ERR_TYPE_NULL;
    return type_rc(mvx_type_commit(*datatype));
}

int MPI_Type_free(MPI_Datatype *datatype) { return type_rc(mvx_type_free(datatype)); }

int MPI_Type_extent(MPI_Datatype datatype, MPI_Aint *extent)
{
    long e;
    if (mvx_type_describe(datatype, NULL, NULL, &e, NULL)) return MVX_ERR_TYPE_NULL;
    if (!extent) return MPI_ERR_ARG;
    *extent = e;
    return MPI_SUCCESS;
}

int MPI_Type_size(MPI_Datatype datatype, int *size)
{
    long s;
    if (mvx_type_describe(datatype, NULL, NULL, NULL, &s)) return MVX_ERR_TYPE_NULL;
    if (!size) return MPI_ERR_ARG;
    *size = (int)s;
    return MPI_SUCCESS;
}

int MPI_Type_lb(MPI_Datatype datatype, MPI_Aint *displacement)   /* type_lb.c */
{
    long lb;
    if (mvx_type_layout(datatype, NULL, NULL, &lb, NULL, NULL, NULL)) return MVX_ERR_TYPE_NULL;
    if (!displacement) return MPI_ERR_ARG;
    *displacement = lb;
    return MPI_SUCCESS;
}

int MPI_Type_ub(MPI_Datatype datatype, MPI_Aint *displacement)   /* type_ub.c */
{
    long ub;
    if (mvx_type_layout(datatype, NULL, NULL, NULL, &ub, NULL, NULL)) return MVX_ERR_TYPE_NULL;
    if (!displacement) return MPI_ERR_ARG;
    *displacement = ub;
    return MPI_SUCCESS;
}

/* ---- the handle a user function is given for a libmvx type (mvx_embed.h) */
#define MAX_TYPE_ALIASES 256
static struct { int type, handle; } g_alias[MAX_TYPE_ALIASES];
static int g_nalias;

int mvx_type_set_handle(int type, int handle)
{
    int i;
    for (i = 0; i < g_nalias; i++)
        if (g_alias[i].type == type) break;
    if (handle == type) {
        if (i < g_nalias) g_alias[i] = g_alias[--g_nalias];
        return MPI_SUCCESS;
    }
    if (i == g_nalias) {
        if (g_nalias == MAX_TYPE_ALIASES) return MPI_ERR_OTHER;
        g_nalias++;
    }
    g_alias[i].type = type;
    g_alias[i].handle = handle;
    return MPI_SUCCESS;
}

MPI_Datatype mvxi_user_handle(MPI_Datatype dt)
{
    int i;
    for (i = 0; i < g_nalias; i++)
        if (g_alias[i].type == dt) return g_alias[i].handle;
    return dt;
}
