// mvx_ops_logic.hip -- kernel table of LAND, LOR, LXOR, BAND, BOR, BXOR
// (one translation unit of libmvx_hip.so,
// so the kernel instantiations compile in parallel; mvx_ops_kern.h)
#define MVX_OPS_LOGICAL_TU 1
#include "mvx_ops_kern.h"

namespace mvx {

const KSet *lookup_logic(int op, int ek)
{
    switch (op) {
    case MPI_LAND:
        switch (ek) { ARITH_INT(OLAND, "land") FLOATS(OLAND, "land")
        LDBL(OLAND, "land") LOGICAL(OLAND, "land") default: return nullptr; }
    case MPI_LOR:
        switch (ek) { ARITH_INT(OLOR, "lor") FLOATS(OLOR, "lor")
        LDBL(OLOR, "lor") LOGICAL(OLOR, "lor") default: return nullptr; }
    case MPI_LXOR:
        switch (ek) { ARITH_INT(OLXOR, "lxor") FLOATS(OLXOR, "lxor")
        LDBL(OLXOR, "lxor") LOGICAL(OLXOR, "lxor") default: return nullptr; }
    case MPI_BAND:
        switch (ek) { case EK_BYTE: ARITH_INT(OBAND, "band") default: return nullptr; }
    case MPI_BOR:
        switch (ek) { case EK_BYTE: ARITH_INT(OBOR, "bor") default: return nullptr; }
    case MPI_BXOR:
        switch (ek) { case EK_BYTE: ARITH_INT(OBXOR, "bxor") default: return nullptr; }
    default:
        return nullptr;
    }
}

}  // namespace mvx

using namespace mvx;

// MPI_LOGICAL's words are process-wide (MPIR_F_TRUE / MPIR_F_FALSE,
// initfutil.c:100-102), g_flog is per device: the words set last are copied
// to a device when they are set there, and before the first LAND / LOR /
// LXOR on MPI_LOGICAL that runs on any other device afterwards.
namespace {
int32_t g_flog_words[2] = {1, 0};
unsigned g_flog_gen = 0;                 // 0: the compiled-in default everywhere
constexpr int FLOG_DEVS = 64;
unsigned g_flog_on[FLOG_DEVS];           // generation each device holds

int flog_copy(int dev)
{
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_flog), g_flog_words, sizeof g_flog_words) != hipSuccess) {
        (void)hipGetLastError();
        return MPI_ERR_OTHER;
    }
    if (dev >= 0 && dev < FLOG_DEVS) g_flog_on[dev] = g_flog_gen;
    return MPI_SUCCESS;
}
}  // namespace

namespace mvx {
int flog_sync()
{
    int dev = -1;
    if (!g_flog_gen || hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= FLOG_DEVS) return MPI_SUCCESS;
    return g_flog_on[dev] == g_flog_gen ? MPI_SUCCESS : flog_copy(dev);
}
}  // namespace mvx

extern "C" int mvx_set_fortran_logical(int true_value, int false_value)
{
    int dev = -1;
    g_flog_words[0] = true_value;
    g_flog_words[1] = false_value;
    if (++g_flog_gen == 0) g_flog_gen = 1;
    if (hipGetDevice(&dev) != hipSuccess) dev = -1;
    return flog_copy(dev);
}
