// mvx_ops_loc.hip -- kernel table of MAXLOC, MINLOC (one translation unit of libmvx_hip.so,
// so the kernel instantiations compile in parallel; mvx_ops_kern.h)
#include "mvx_ops_kern.h"

namespace mvx {

const KSet *lookup_loc(int op, int ek)
{
    switch (op) {
    case MPI_MAXLOC:
        switch (ek) { PAIRS(OMAXLOC, "maxloc")
        LDBL_INT(OMAXLOC, "maxloc") CONTIG_PAIRS(OMAXLOC, "maxloc") default: return nullptr; }
    case MPI_MINLOC:
        switch (ek) { PAIRS(OMINLOC, "minloc")
        LDBL_INT(OMINLOC, "minloc") CONTIG_PAIRS(OMINLOC, "minloc") default: return nullptr; }
    default:
        return nullptr;
    }
}

}  // namespace mvx
