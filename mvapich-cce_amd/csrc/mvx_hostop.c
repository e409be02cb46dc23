/*
 * mvx_hostop.c -- the predefined ops as MPI_User_functions (MPIR_MAXF ...
 * MPIR_MINLOC, global_ops.c; include/mpiimpl.h:201-212) on operands in any
 * memory.  Device operands run the op kernel in place; host operands are
 * streamed through HBM (host_apply).  The op functions have no communicator,
 * so their staging (g_hop) is the process's, one call at a time.
 */
#include <pthread.h>
#include <stdlib.h>

#include "mvx_internal.h"

static int g_op_errno = 0;   /* MPIR_Op_errno, global_ops.c:41 */

int mvx_op_errno(void)
{
    int e = g_op_errno;
    g_op_errno = 0;
    return e;
}

/* Host-resident operands (the reference's MPI user buffers): a chunked
 * pipeline over HOP_NB slots.  Chunk c: a pageable operand is copied into a
 * pinned bounce slot by the copy pool (mvx_host.c) and DMA'd from there; a
 * page-locked operand is DMA'd directly.  The kernel runs on stream 0, the
 * D2H of the result on stream 1 (into the bounce, or straight into a
 * page-locked inout), and the host drains chunk c-L out of the bounce after
 * issuing chunk c, so host copies, both PCIe directions and the kernel
 * overlap (L: mvxi_host_drain_lag, mvx_host.c).  Below HOP_BOUNCE_MIN bytes per operand the bounce's per-chunk
 * overheads (pool wake-ups, one more copy) cost more than they hide, and
 * pageable operands are handed to HIP's own pageable copy path instead
 * (tools/bench_host.py: 2 MiB 165 vs 299 us, 256 MiB 14.7 vs 12.8 ms;
 * profiles/r02/bench_host.jsonl).  Device operands are used in place; both
 * operands get an HBM mirror (HBM is plentiful, and no device slot is reused
 * while a copy may still read it). */
#define HOP_NB 4            /* slots: >= the drain lag + 2 (mvxi_host_drain_lag) */
#define HOP_BOUNCE_MIN (64L << 20)
#define HOP_CHUNK_MIN (1L << 20)
#define HOP_CHUNK_MAX (16L << 20)
#define HOP_PIN_CHUNK_MIN (4L << 20)
#define HOP_PIN_CHUNK_MAX (64L << 20)   /* tools/host_chunk_sweep.sh, profiles/r02/host_chunk_sweep.txt */
static struct {
    hipStream_t s[2];
    hipEvent_t ein[HOP_NB], ek[HOP_NB], eout[HOP_NB];
    char *bin, *bout, *dev;       /* HOP_NB bounce slots: bin 2 chunks, bout 1; dev: both operands */
    size_t bin_bytes, bout_bytes, dev_bytes;
} g_hop;

static int hop_init(size_t slot, size_t dev)
{
    int b;
    if (!g_hop.s[0]) {
        if (mvxi_queue_stream(&g_hop.s[0], "MVX_STAGE_STREAM", "plain") != hipSuccess ||
            mvxi_queue_stream(&g_hop.s[1], "MVX_STAGE_STREAM", "plain") != hipSuccess)
            return MPI_ERR_OTHER;
        for (b = 0; b < HOP_NB; b++)
            if (hipEventCreateWithFlags(&g_hop.ein[b], hipEventDisableTiming) != hipSuccess ||
                hipEventCreateWithFlags(&g_hop.ek[b], hipEventDisableTiming) != hipSuccess ||
                hipEventCreateWithFlags(&g_hop.eout[b], hipEventDisableTiming) != hipSuccess)
                return MPI_ERR_OTHER;
    }
    if ((slot && (mvxi_grow_host(&g_hop.bin, &g_hop.bin_bytes, HOP_NB * 2 * slot) ||
                  mvxi_grow_host(&g_hop.bout, &g_hop.bout_bytes, HOP_NB * slot))) ||
        mvxi_grow(&g_hop.dev, &g_hop.dev_bytes, dev))
        return MPI_ERR_OTHER;
    return MPI_SUCCESS;
}

/* Page-locked host operands need no staging: the op kernel reads and writes
 * them in place over PCIe through their device address (the same address
 * for hipHostMalloc'd and hipHostRegister'ed memory, interior pointers
 * included: tools/zc_attr.hip).  256 MiB SUM float32 9.94-10.07 ms against
 * 10.9 ms for 2 H2D + kernel + 1 D2H through HBM (tools/zc_probe.hip: a
 * kernel's PCIe reads reach 55 GB/s, the DMA engines' 57.5).
 * MVX_HOST_ZEROCOPY=0 keeps the DMA pipeline for them.  Pageable operands
 * keep the DMA pipeline: a kernel reading the pinned bounce slots in place
 * (just filled by the copy pool) ran the 256 MiB op in 13.8-14.4 ms against
 * 11.4-11.5 through HBM (tools/zc_ab.sh, profiles/r05/zero_copy_bounce_ab.jsonl). */
static int zerocopy_on(void)
{
    static int on = -1;
    if (on < 0) {
        const char *v = getenv("MVX_HOST_ZEROCOPY");
        on = v ? atoi(v) != 0 : 1;
    }
    return on;
}

/* the device address of page-locked host memory, or NULL */
static void *host_dev_alias(const void *p)
{
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return NULL;
    }
    return a.type == hipMemoryTypeHost ? a.devicePointer : NULL;
}

static int host_apply_locked(MPI_Op op, MPI_Datatype t, const char *in, char *inout, long len,
                             int in_dev, int io_dev, int kin, int kio)
{
    const int in_pin = kin == MVX_BUF_PINNED, io_pin = kio == MVX_BUF_PINNED;
    int e, ts, rc, bounce_in, bounce_io;
    long chunk, c, nch, lag;
    size_t bytes, cb, slot;
    hipStream_t sd;
    mvx_dtype_info(t, &e, &ts);
    bytes = (size_t)len * e;
    if ((in_dev || in_pin) && (io_dev || io_pin) && zerocopy_on()) {
        const void *din = in_dev ? (const void *)in : host_dev_alias(in);
        void *dio = io_dev ? (void *)inout : host_dev_alias(inout);
        if (din && dio) {
            if ((rc = hop_init(0, 0)) || (rc = mvx_op_apply(op, t, din, dio, (size_t)len, g_hop.s[0])))
                return rc;
            return hipStreamSynchronize(g_hop.s[0]) == hipSuccess ? MPI_SUCCESS : MPI_ERR_OTHER;
        }
    }
    /* pageable memory partly under another call's registration is never
     * handed to HIP (MVX_BUF_BOUNCE): bounced at any size */
    bounce_in = !in_dev && !in_pin && (bytes >= (size_t)HOP_BOUNCE_MIN || kin == MVX_BUF_BOUNCE);
    bounce_io = !io_dev && !io_pin && (bytes >= (size_t)HOP_BOUNCE_MIN || kio == MVX_BUF_BOUNCE);
    /* chunk: whole 256-element groups (the device operands keep the kernel's
     * 16-byte vector path) */
    if (bounce_in || bounce_io) {       /* pool copies pace the pipeline: ~8 chunks */
        cb = bytes / 8;
        if (cb < (size_t)HOP_CHUNK_MIN) cb = HOP_CHUNK_MIN;
        if (cb > (size_t)HOP_CHUNK_MAX) cb = HOP_CHUNK_MAX;
    } else if ((!in_dev && !in_pin) || (!io_dev && !io_pin)) {
        cb = 32L << 20;                 /* HIP stages pageable copies itself: whole 32 MiB pieces */
    } else {                            /* DMA only: fewer, larger copies */
        cb = bytes / 4;
        if (cb < (size_t)HOP_PIN_CHUNK_MIN) cb = HOP_PIN_CHUNK_MIN;
        if (cb > (size_t)HOP_PIN_CHUNK_MAX) cb = HOP_PIN_CHUNK_MAX;
    }
    {
        static long fixed = -1;       /* MVX_HOST_CHUNK_MIB: a fixed chunk (tuning) */
        if (fixed < 0) {
            const char *v = getenv("MVX_HOST_CHUNK_MIB");
            fixed = v ? atol(v) : 0;
        }
        if (fixed > 0) cb = (size_t)fixed << 20;
    }
    chunk = (long)(cb / ((size_t)e * 256)) * 256;
    if (chunk < 256) chunk = 256;
    if (chunk > len) chunk = len;
    slot = (bounce_in || bounce_io) ? al256((size_t)chunk * e) : 0;
    if ((rc = hop_init(slot, 2 * al256(bytes)))) return rc;
    nch = (len + chunk - 1) / chunk;
    sd = nch > 1 ? g_hop.s[1] : g_hop.s[0];    /* one chunk: everything in order on one stream */
    lag = mvxi_host_drain_lag();
    for (c = 0; c < nch + lag; c++) {
        if (c < nch) {
            const int b = (int)(c % HOP_NB);
            const long n = len - c * chunk < chunk ? len - c * chunk : chunk;
            const size_t o = (size_t)(c * chunk) * e, sz = (size_t)n * e;
            char *bi = slot ? g_hop.bin + (size_t)b * 2 * slot : NULL;
            char *din = in_dev ? (char *)in + o : g_hop.dev + o;
            char *dio = io_dev ? inout + o : g_hop.dev + al256(bytes) + o;
            /* bounce slot b was last read by the H2D of chunk c - HOP_NB */
            if (slot && c >= HOP_NB && hipEventSynchronize(g_hop.ein[b]) != hipSuccess) return MPI_ERR_OTHER;
            if (bounce_in) mvx_pcopy(bi, in + o, sz);
            if (bounce_io) mvx_pcopy(bi + slot, inout + o, sz);
            if (!in_dev && hipMemcpyAsync(din, bounce_in ? bi : in + o, sz, hipMemcpyHostToDevice,
                                          g_hop.s[0]) != hipSuccess)
                return MPI_ERR_OTHER;
            if (!io_dev && hipMemcpyAsync(dio, bounce_io ? bi + slot : inout + o, sz, hipMemcpyHostToDevice,
                                          g_hop.s[0]) != hipSuccess)
                return MPI_ERR_OTHER;
            if (slot && hipEventRecord(g_hop.ein[b], g_hop.s[0]) != hipSuccess) return MPI_ERR_OTHER;
            if ((rc = mvx_op_apply(op, t, din, dio, (size_t)n, g_hop.s[0]))) return rc;
            if (!io_dev) {
                if (sd != g_hop.s[0] &&
                    (hipEventRecord(g_hop.ek[b], g_hop.s[0]) != hipSuccess ||
                     hipStreamWaitEvent(sd, g_hop.ek[b], 0) != hipSuccess))
                    return MPI_ERR_OTHER;
                if (hipMemcpyAsync(bounce_io ? g_hop.bout + (size_t)b * slot : inout + o, dio, sz,
                                   hipMemcpyDeviceToHost, sd) != hipSuccess ||
                    (bounce_io && hipEventRecord(g_hop.eout[b], sd) != hipSuccess))
                    return MPI_ERR_OTHER;
            }
        }
        if (c >= lag && bounce_io) {   /* drain chunk c - lag */
            const long p = c - lag;
            const int b = (int)(p % HOP_NB);
            const long n = len - p * chunk < chunk ? len - p * chunk : chunk;
            if (hipEventSynchronize(g_hop.eout[b]) != hipSuccess) return MPI_ERR_OTHER;
            mvx_pcopy(inout + (size_t)(p * chunk) * e, g_hop.bout + (size_t)b * slot, (size_t)n * e);
        }
    }
    if (hipStreamSynchronize(g_hop.s[0]) != hipSuccess || hipStreamSynchronize(sd) != hipSuccess)
        return MPI_ERR_OTHER;
    return MPI_SUCCESS;
}

static pthread_mutex_t g_hop_mu = PTHREAD_MUTEX_INITIALIZER;

/* g_hop's streams and slots serve one call at a time.  A host operand the
 * registration cache hands out as page-locked is held until the call's last
 * DMA on it is done (a failed call drains its streams first). */
static int host_apply(MPI_Op op, MPI_Datatype t, const char *in, char *inout, long len, int in_dev, int io_dev)
{
    int rc, e, ts;
    unsigned long hin = 0, hio = 0;
    size_t bytes;
    mvx_dtype_info(t, &e, &ts);
    bytes = (size_t)len * e;
    pthread_mutex_lock(&g_hop_mu);
    {
        unsigned long *mine[1] = {&hin};
        int kin = in_dev ? MVX_BUF_DEVICE : mvxi_buf_kind_hold(in, bytes, &hin, NULL, 0);
        const int kio = io_dev ? MVX_BUF_DEVICE : mvxi_buf_kind_hold(inout, bytes, &hio, mine, hin ? 1 : 0);
        /* in's registration merged into inout's union and lost with it */
        if (kin == MVX_BUF_PINNED && !hin && !mvx_host_pinned(in)) {
            unsigned long *other[1] = {&hio};
            kin = mvxi_buf_kind_hold(in, bytes, &hin, other, hio ? 1 : 0);
        }
        rc = host_apply_locked(op, t, in, inout, len, in_dev, io_dev, kin, kio);
    }
    if (rc != MPI_SUCCESS && (hin || hio)) {
        if (g_hop.s[0]) (void)hipStreamSynchronize(g_hop.s[0]);
        if (g_hop.s[1]) (void)hipStreamSynchronize(g_hop.s[1]);
        (void)hipGetLastError();
    }
    pthread_mutex_unlock(&g_hop_mu);
    mvxi_buf_release(hin);
    mvxi_buf_release(hio);
    return rc;
}

static void uop_call(MPI_Op op, void *in, void *inout, int *len, MPI_Datatype *t)
{
    int rc;
    if (!len || !t) { g_op_errno = MPI_ERR_ARG; return; }
    rc = mvx_op_apply(op, *t, NULL, NULL, 0, NULL);   /* verdict first */
    if (rc == MPI_SUCCESS && *len > 0) {
        const int in_dev = mvxi_is_device_ptr(in), io_dev = mvxi_is_device_ptr(inout);
        if (in_dev && io_dev) {
            rc = mvx_op_apply(op, *t, in, inout, (size_t)*len, NULL);
            if (rc == MPI_SUCCESS && hipStreamSynchronize(NULL) != hipSuccess) rc = MPI_ERR_OTHER;
        } else if (!in || !inout) {
            rc = MPI_ERR_BUFFER;
        } else {
            rc = host_apply(op, *t, (const char *)in, (char *)inout, *len, in_dev, io_dev);
        }
    }
    if (rc) g_op_errno = rc;
}

#define UOP(NAME, OPH) \
    void NAME(void *in, void *io, int *len, MPI_Datatype *t) { uop_call(OPH, in, io, len, t); }
UOP(MPIR_MAXF, MPI_MAX)
UOP(MPIR_MINF, MPI_MIN)
UOP(MPIR_SUM, MPI_SUM)
UOP(MPIR_PROD, MPI_PROD)
UOP(MPIR_LAND, MPI_LAND)
UOP(MPIR_BAND, MPI_BAND)
UOP(MPIR_LOR, MPI_LOR)
UOP(MPIR_BOR, MPI_BOR)
UOP(MPIR_LXOR, MPI_LXOR)
UOP(MPIR_BXOR, MPI_BXOR)
UOP(MPIR_MAXLOC, MPI_MAXLOC)
UOP(MPIR_MINLOC, MPI_MINLOC)
