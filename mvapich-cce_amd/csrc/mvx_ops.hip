// mvx_ops.hip -- the device side of the MPI local reduction path, written for
// gfx950 (CDNA4, wave64): the (op, datatype) dispatch, the launch policy and
// the C-ABI of include/mvx_hip.h.  The kernels and their per-op tables are in
// mvx_ops_kern.h and mvx_ops_{cmp,arith,logic,loc}.hip (design notes at the
// top of mvx_ops_kern.h).
#include "mvx_ops_kern.h"

namespace mvx {

// a handle's dte_type, where the Fortran types share one with a C type
// (initfutil.c:238-245, 261, 279: INTEGER is MPIR_INT, REAL MPIR_FLOAT,
// DOUBLE PRECISION MPIR_DOUBLE); the old types of derived types switch on it
static int dte_of(int h)
{
    switch (h) {
    case MPI_INTEGER: return MPI_INT;
    case MPI_REAL: return MPI_FLOAT;
    case MPI_DOUBLE_PRECISION: return MPI_DOUBLE;
    default: return h;
    }
}

// the op kind of a derived handle (mvx_dtype.hip): MAXLOC / MINLOC are the
// only ops with derived cases -- a count-2 contiguous type over one base
// (stride-2 {value, loc} scalars, global_ops.c:1387-1503 / 1625-1740), and an
// MPIR_STRUCT type by the dte_type of its old_types[0], read as that base's C
// pair struct (1280-1384 / 1520-1620); every other case is 329
static int derived_kind(const dt::Info &d)
{
    if (d.kind == dt::K_STRUCT) {
        switch (dte_of(d.old)) {
        case MPI_INT: return EK_PII;             // MPIR_2int_loctype
        case MPI_FLOAT: return EK_PFI;
        case MPI_LONG: case MPI_LONG_LONG_INT: return EK_PLI;
        case MPI_SHORT: return EK_PSI;
        case MPI_DOUBLE: return EK_PDI;
        case MPI_LONG_DOUBLE: return EK_LDBL_INT;
        default: return EK_DERIVED;
        }
    }
    if (d.kind != dt::K_CONTIG || d.count != 2) return EK_DERIVED;
    switch (dte_of(d.old)) {      // the base's dte_type, global_ops.c:1395-1497
    case MPI_INT: return EK_PII;
    case MPI_LONG: case MPI_LONG_LONG_INT: return EK_PP64;
    case MPI_SHORT: return EK_PP16;
    case MPI_CHAR: return EK_PP8;
    case MPI_FLOAT: return EK_PPF;
    case MPI_DOUBLE: return EK_PPD;
    case MPI_LONG_DOUBLE: return EK_PPX;
    default: return EK_DERIVED;
    }
}

static int ekind(int dtype)
{
    if (dtype >= MVX_TYPE_DERIVED_BASE) {
        dt::Info d;
        return dt::info(dtype, &d) ? derived_kind(d) : EK_NONE;
    }
    switch (dtype) {
    case MPI_CHAR: return EK_I8;
    case MPI_UNSIGNED_CHAR: return EK_U8;
    case MPI_BYTE: return EK_BYTE;
    case MPI_SHORT: return EK_I16;
    case MPI_UNSIGNED_SHORT: return EK_U16;
    case MPI_INT: return EK_I32;
    case MPI_UNSIGNED: return EK_U32;
    case MPI_LONG: case MPI_LONG_LONG_INT: return EK_I64;
    case MPI_UNSIGNED_LONG: return EK_U64;
    case MPI_FLOAT: return EK_F32;
    case MPI_DOUBLE: return EK_F64;
    case MPI_COMPLEX: return EK_C32;
    case MPI_DOUBLE_COMPLEX: return EK_C64;
    case MPI_FLOAT_INT: return EK_PFI;
    case MPI_DOUBLE_INT: return EK_PDI;
    case MPI_LONG_INT: return EK_PLI;
    case MPI_SHORT_INT: return EK_PSI;
    case MPI_2INT: return EK_PII;
    case MPI_LONG_DOUBLE: return EK_LDBL;
    case MPI_LONG_DOUBLE_INT: return EK_LDBL_INT;
    case MPI_INTEGER: return EK_I32;
    case MPI_REAL: return EK_F32;
    case MPI_DOUBLE_PRECISION: return EK_F64;
    case MPI_LOGICAL: return EK_LOGICAL;
    // the Fortran pairs: contiguous(2, x), the MAXLOC / MINLOC stride-2 case
    // of x's dte_type (global_ops.c:1387-1503); no case for COMPLEX (1498)
    case MPI_2INTEGER: return EK_PII;
    case MPI_2REAL: return EK_PPF;
    case MPI_2DOUBLE_PRECISION: return EK_PPD;
    case MPI_2COMPLEX: case MPI_2DOUBLE_COMPLEX: return EK_DERIVED;
    default: return EK_NONE;
    }
}

// Returns the kernel set, or NULL with *rc set to the reference's answer for
// that (op, type): 329 where the op's switch has no case for it
// (global_ops.c:158-161 and every sibling default), and MPI_ERR_OP for a
// handle outside MPI_MAX..MPI_MAXLOC.
static const KSet *lookup(int op, int dtype, int *rc)
{
    int ek = ekind(dtype);
    *rc = MVX_ERR_OP_NOT_DEFINED;
    if (ek == EK_LOGICAL && (op == MPI_BAND || op == MPI_BOR || op == MPI_BXOR))
        ek = EK_U32;                 // bitwise on the MPI_Fint word

    switch (op) {
    case MPI_MAX: case MPI_MIN:
        return lookup_cmp(op, ek);
    case MPI_SUM: case MPI_PROD:
        return lookup_arith(op, ek);
    case MPI_LAND: case MPI_LOR: case MPI_LXOR: case MPI_BAND: case MPI_BOR: case MPI_BXOR:
        if (ek == EK_LOGICAL && flog_sync()) { *rc = MPI_ERR_OTHER; return nullptr; }
        return lookup_logic(op, ek);
    case MPI_MAXLOC: case MPI_MINLOC:
        return lookup_loc(op, ek);
    default:
        *rc = MPI_ERR_OP;
        return nullptr;
    }
}

// Grid: one pass over the data (a block per 256*U chunks) up to this cap,
// grid-stride beyond it; a full pass measured best on the config-2 kernel.
static int g_block_cap = 1 << 20;
// Non-temporal above this many bytes touched by one launch (all operands +
// the result); below it the result is likely re-read from L2 / MALL.
static long g_nt_min_bytes = 64L << 20;
static int g_prog4 = 1;          // programs over 3-4 leaves on the KMAX = 4 kernels
static int g_prog_u = 1;
static int g_generic_only = 0;   // MVX_PROG_GENERIC=1: no fixed-tree kernels (A/B runs)
static int g_chain_rt = 1;       // MVX_CHAIN_RT=0: chains of 5-7 leaves on the masked program (A/B)
// resident blocks per CU for the non-temporal launches of each family (0 =
// as many as registers allow); MVX_CAP_{APPLY,PROG,TREE} override for A/B runs
static int g_cap[FAM_N] = {0, 0, 2};
static int g_no_body = 0;        // MVX_NO_BODY=1: fixed trees through k_combine (A/B runs)
static size_t g_cap_lds[FAM_N];
static const char *g_last = "";
static char g_last_buf[96];
static const char *g_last_sym = "";
static unsigned g_last_blocks;
static size_t g_last_lds;
static const void *g_last_fn;

// LDS per CU of the device the kernels run on, from its architecture name
// (the runtime's per-multiprocessor attribute reports the 64 KiB per-block
// limit instead): gfx950 has 160 KiB; earlier CDNA parts 64 KiB.  A
// reservation sized for 160 KiB on a 64 KiB part would cap the kernel at one
// resident block per CU, so the reservation follows the part.
static size_t lds_per_cu()
{
    static size_t v = 0;
    if (v) return v;
    int dev = 0;
    hipDeviceProp_t pr;
    v = 64 * 1024;
    if (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&pr, dev) == hipSuccess) {
        if (!strncmp(pr.gcnArchName, "gfx950", 6)) v = 160 * 1024;
    } else {
        (void)hipGetLastError();
    }
    return v;
}

// dynamic LDS per block that leaves room for `cap` blocks per CU and not one
// more (the kernels do not touch it): the middle of the range,
// 2 * LDS / (2 * cap + 1), clear of the allocator's rounding at the edges; at
// most 64 KiB (no function attribute needed).
static size_t cap_lds(int cap)
{
    const size_t lds = lds_per_cu();
    if (cap < 2) return 0;
    const size_t b = (lds * 2 / (size_t)(2 * cap + 1)) & ~(size_t)1023;
    return b > 64 * 1024 ? 64 * 1024 : b;
}

static void init_env()
{
    static int done = 0;
    if (done) return;
    done = 1;
    const char *e = getenv("MVX_NT_MIN_BYTES");
    if (e) g_nt_min_bytes = atol(e);
    e = getenv("MVX_BLOCK_CAP");
    if (e && atoi(e) > 0) g_block_cap = atoi(e);
    e = getenv("MVX_PROG_U");
    if (e && atoi(e) == 2) g_prog_u = 2;
    e = getenv("MVX_PROG_GENERIC");
    if (e && atoi(e) == 1) g_generic_only = 1;
    e = getenv("MVX_PROG4");
    if (e && atoi(e) == 0) g_prog4 = 0;
    e = getenv("MVX_CHAIN_RT");
    if (e && atoi(e) == 0) g_chain_rt = 0;
    e = getenv("MVX_NO_BODY");
    if (e && atoi(e) == 1) g_no_body = 1;
    const char *caps[FAM_N] = {"MVX_CAP_APPLY", "MVX_CAP_PROG", "MVX_CAP_TREE"};
    for (int f = 0; f < FAM_N; ++f) {
        e = getenv(caps[f]);
        if (e) g_cap[f] = atoi(e);
        g_cap_lds[f] = cap_lds(g_cap[f]);
    }
}

static int launch(const KSet *ks, const KFam &F, Params &P, hipStream_t stream)
{
    init_env();
    int nleaves = 0;
    for (int q = 0; q < P.k; ++q) nleaves += 1 + (P.fold[q] != nullptr);
    const int nt = (long)(nleaves + 1) * P.n * ks->esize >= g_nt_min_bytes;
    const void *fn = F.fn[nt];
    const int unroll = F.unroll[nt];
    const size_t lds = nt ? g_cap_lds[F.fam] : 0;
    const int es = ks->esize;
    const uintptr_t m = (uintptr_t)P.dst & 15;
    bool same = true;
    for (int q = 0; q < P.k; ++q) {
        if (((uintptr_t)P.src[q] & 15) != m) same = false;
        if (P.fold[q] && ((uintptr_t)P.fold[q] & 15) != m) same = false;
    }
    const long pre = (long)((16 - m) & 15);
    if (same && pre % es == 0) {
        long head = pre / es;
        if (head > P.n) head = P.n;
        P.head = head;
        P.nvec = (P.n - head) * es / ks->chunk;
        P.vec_ok = 1;
    } else {
        P.head = 0;
        P.nvec = 0;
        P.vec_ok = 0;
    }
    bool folded = false;
    for (int q = 0; q < P.k; ++q) folded |= P.fold[q] != nullptr;
    const bool body_k = P.k == F.body_k || (F.body_kmin && P.k >= F.body_kmin && P.k <= F.body_k);
    if (nt && F.body && !g_no_body && body_k && P.vec_ok && P.head == 0 && P.nvec > 0 &&
        P.nvec * ks->chunk == P.n * es && !folded) {
        BodyParams B;
        memset(&B, 0, sizeof B);
        for (int q = 0; q < P.k; ++q) B.src[q] = reinterpret_cast<const u32x4 *>(P.src[q]);
        B.dst = reinterpret_cast<u32x4 *>(P.dst);
        B.nvec = P.nvec;
        B.k = P.k;
        long work = (P.nvec * F.body_units + F.body_unroll * 256 - 1) / (F.body_unroll * 256);
        const unsigned blocks = (unsigned)(work < g_block_cap ? work : g_block_cap);
        void *bargs[] = {&B};
        const size_t blds = cap_lds(F.body_cap);
        hipError_t e = hipLaunchKernel(F.body, dim3(blocks), dim3(256), bargs, blds, stream);
        g_last_blocks = blocks;
        g_last_lds = blds;
        g_last_fn = F.body;
        snprintf(g_last_buf, sizeof g_last_buf, "%s_k%d_nt", ks->name, P.k);
        g_last = g_last_buf;
        g_last_sym = F.body_sym();
        return e == hipSuccess ? MPI_SUCCESS : MPI_ERR_OTHER;
    }
    long work = P.vec_ok ? (P.nvec + unroll * 256 - 1) / (unroll * 256)
                         : (P.n + 255) / 256;
    if (work < 1) work = 1;
    const unsigned blocks = (unsigned)(work < g_block_cap ? work : g_block_cap);
    void *args[] = {&P};
    hipError_t e = hipLaunchKernel(fn, dim3(blocks), dim3(256), args, lds, stream);
    g_last_blocks = blocks;
    g_last_lds = lds;
    g_last_fn = fn;
    snprintf(g_last_buf, sizeof g_last_buf, "%s_k%d%s", ks->name, P.k, nt ? "_nt" : "");
    g_last = g_last_buf;
    g_last_sym = F.sym[nt]();
    return e == hipSuccess ? MPI_SUCCESS : MPI_ERR_OTHER;
}

}  // namespace mvx

using namespace mvx;


extern "C" int mvx_op_supported(int op, int dtype)
{
    int rc;
    return lookup(op, dtype, &rc) != nullptr;
}

extern "C" int mvx_op_element_size(int op, int dtype)
{
    int rc;
    const KSet *ks = lookup(op, dtype, &rc);
    return ks ? ks->esize : 0;
}

extern "C" int mvx_op_apply(int op, int dtype, const void *in, void *inout,
                            size_t n, void *stream)
{
    int rc;
    const KSet *ks = lookup(op, dtype, &rc);
    if (!ks) return rc;
    if (n == 0) return MPI_SUCCESS;
    Params P;
    memset(&P, 0, sizeof P);
    P.src[0] = (const char *)inout;   // a: the inout operand
    P.src[1] = (const char *)in;      // b
    P.dst = (char *)inout;
    P.n = (long)n;
    P.k = 2;
    return launch(ks, ks->apply, P, (hipStream_t)stream);
}

extern "C" int mvx_op_program(int op, int dtype, const void *const *srcs,
                              const void *const *fold, int k, unsigned tree_mask,
                              unsigned chain_mask, void *dst, size_t n, void *stream)
{
    int rc;
    const KSet *ks = lookup(op, dtype, &rc);
    if (!ks) return rc;
    if (k < 1 || k > MVX_COMBINE_KMAX || !srcs) return MPI_ERR_ARG;
    /* every step must stay inside the k leaves */
    for (int l = 0; l < 3; ++l)
        for (int q = 0; q < 8; ++q)
            if ((tree_mask >> (l * 8 + q) & 1u) && q + (1 << l) >= k) return MPI_ERR_ARG;
    if ((tree_mask >> 24) || (chain_mask & 1u) || (chain_mask >> k)) return MPI_ERR_ARG;
    if (n == 0) return MPI_SUCCESS;
    Params P;
    memset(&P, 0, sizeof P);
    for (int q = 0; q < k; ++q) {
        P.src[q] = (const char *)srcs[q];
        P.fold[q] = fold ? (const char *)fold[q] : nullptr;
    }
    P.dst = (char *)dst;
    P.n = (long)n;
    P.k = k;
    P.tree_mask = tree_mask;
    P.chain_mask = chain_mask;
    if (k <= 2) {
        /* the only programs over <= 2 leaves: nothing, or y0 op y1 */
        if (k == 2 && !(tree_mask & 1u) && !(chain_mask & 2u)) return MPI_ERR_ARG;
        return launch(ks, ks->apply, P, (hipStream_t)stream);
    }
    init_env();
    bool folded = false;
    for (int q = 0; q < k; ++q) folded |= P.fold[q] != nullptr;
    if (!g_generic_only && !folded && chain_mask == 0 && (k == 8 || k == 4) && tree_mask == mvx_tree_mask(k))
        return launch(ks, k == 8 ? ks->tree8 : ks->tree4, P, (hipStream_t)stream);
    /* chains of 5-7 leaves (pairwise Reduce_scatter at p = 5..7): the 8-leaf
     * chain body with a run-time leaf count, else its masked program */
    if (!g_generic_only && !folded && tree_mask == 0 && k >= 4 && chain_mask == mvx_chain_mask(k) &&
        (k == 4 || g_chain_rt || k == 8))
        return launch(ks, k == 4 ? ks->chain4 : ks->chain8, P, (hipStream_t)stream);
    if (g_prog_u == 2 && ks->prog2.fn[0])
        return launch(ks, ks->prog2, P, (hipStream_t)stream);
    if (k <= 4 && g_prog4)
        return launch(ks, ks->prog4, P, (hipStream_t)stream);
    return launch(ks, ks->prog, P, (hipStream_t)stream);
}

extern "C" unsigned mvx_tree_mask(int k)
{
    unsigned m = 0;
    for (int l = 0; (1 << l) < k && l < 3; ++l)
        for (int q = 0; q + (1 << l) < k; q += 2 << l) m |= 1u << (l * 8 + q);
    return m;
}

extern "C" unsigned mvx_chain_mask(int k)
{
    return k >= 2 && k <= 32 ? (unsigned)(((1ull << k) - 1) & ~1ull) : 0u;
}

extern "C" int mvx_op_combine(int op, int dtype, const void *const *srcs,
                              const void *const *fold, int k, int shape,
                              void *dst, size_t n, void *stream)
{
    if (shape != MVX_SHAPE_TREE && shape != MVX_SHAPE_CHAIN) {
        int rc;
        return lookup(op, dtype, &rc) ? MPI_ERR_ARG : rc;
    }
    return mvx_op_program(op, dtype, srcs, fold, k,
                          shape == MVX_SHAPE_TREE ? mvx_tree_mask(k) : 0u,
                          shape == MVX_SHAPE_CHAIN ? mvx_chain_mask(k) : 0u, dst, n, stream);
}

extern "C" void mvx_hip_set_launch(int block_cap, int nt_min_bytes_log2)
{
    init_env();
    if (block_cap > 0) g_block_cap = block_cap;
    if (nt_min_bytes_log2 > 0) g_nt_min_bytes = 1L << nt_min_bytes_log2;
    if (nt_min_bytes_log2 < 0) g_nt_min_bytes = 1L << 62;   // never non-temporal
}

extern "C" const char *mvx_hip_last_kernel(void) { return g_last; }

extern "C" const char *mvx_hip_last_kernel_symbol(void) { return g_last_sym; }

extern "C" void mvx_hip_last_launch(unsigned *blocks, size_t *dynamic_lds, int *blocks_per_cu)
{
    if (blocks) *blocks = g_last_blocks;
    if (dynamic_lds) *dynamic_lds = g_last_lds;
    if (blocks_per_cu) {
        int occ = 0;
        if (!g_last_fn ||
            hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, g_last_fn, 256, g_last_lds) != hipSuccess) {
            (void)hipGetLastError();
            occ = 0;
        }
        *blocks_per_cu = occ;
    }
}
