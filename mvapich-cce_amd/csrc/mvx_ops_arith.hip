// mvx_ops_arith.hip -- kernel table of SUM, PROD (one translation unit of libmvx_hip.so,
// so the kernel instantiations compile in parallel; mvx_ops_kern.h)
#include "mvx_ops_kern.h"

namespace mvx {

const KSet *lookup_arith(int op, int ek)
{
    switch (op) {
    case MPI_SUM:
        switch (ek) { ARITH_INT(OSUM, "sum") FLOATS(OSUM, "sum") CMPLX(OSUM, "sum")
        LDBL(OSUM, "sum") default: return nullptr; }
    case MPI_PROD:
        switch (ek) { ARITH_INT(OPROD, "prod") FLOATS(OPROD, "prod") CMPLX(OPROD, "prod")
        LDBL(OPROD, "prod") default: return nullptr; }
    default:
        return nullptr;
    }
}

}  // namespace mvx
