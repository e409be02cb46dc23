/* COMPILE-CHECK ONLY (integration/check/README.md): the compile-check
 * headers must lay out every member integration/intra_mvx.c reads exactly
 * as the reference's own headers do (ref_layout.h, measured from them by
 * ref_layout.py).  Built into both check libraries, plain and _SMP_: a
 * difference stops the build. */
#include <stddef.h>

#include "mpiimpl.h"
#include "mpiops.h"
#include "mpicoll.h"
#include "ref_layout.h"

typedef struct MPIR_COMMUNICATOR comm_t;
typedef struct MPIR_DATATYPE dtype_t;
typedef struct MPIR_OP op_t;
typedef struct _MPIR_COLLOPS collops_t;

#define CHECK_OFF(T, m, v) \
    _Static_assert(offsetof(T, m) == (v), #T "." #m " is not where the reference's header puts it");
#define CHECK_SIZE(T, v) \
    _Static_assert(sizeof(T) == (v), "sizeof " #T " differs from the reference's header");

REF_OFFSETS(CHECK_OFF)
REF_SIZES(CHECK_SIZE)

/* something to link */
int mvx_check_layout_pinned(void) { return 1; }
