// mvx_ops_cmp.hip -- kernel table of MAX, MIN (one translation unit of libmvx_hip.so,
// so the kernel instantiations compile in parallel; mvx_ops_kern.h)
#include "mvx_ops_kern.h"

namespace mvx {

const KSet *lookup_cmp(int op, int ek)
{
    switch (op) {
    case MPI_MAX:
        switch (ek) { SIGNED_INT(OMAX, "max") FLOATS(OMAX, "max")
        LDBL(OMAX, "max") default: return nullptr; }
    case MPI_MIN:
        switch (ek) { SIGNED_INT(OMIN, "min") FLOATS(OMIN, "min")
        LDBL(OMIN, "min") default: return nullptr; }
    default:
        return nullptr;
    }
}

}  // namespace mvx
