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

extern "C" int mvx_set_fortran_logical(int true_value, int false_value)
{
    const int32_t v[2] = {true_value, false_value};
    return hipMemcpyToSymbol(HIP_SYMBOL(g_flog), v, sizeof v) == hipSuccess ? MPI_SUCCESS : MPI_ERR_OTHER;
}
