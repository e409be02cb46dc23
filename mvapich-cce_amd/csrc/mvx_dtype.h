// mvx_dtype.h -- internal interface of the datatype engine (mvx_dtype.hip)
// to the op kernels (mvx_ops.hip), both in libmvx_hip.so.  The C-ABI is in
// include/mvx_hip.h.
#ifndef MVX_DTYPE_INTERNAL_H
#define MVX_DTYPE_INTERNAL_H

namespace mvx {
namespace dt {

// the reference's dte_type of a handle (mpid/ch2/datatype.h): vector and
// indexed constructors produce HVECTOR / HINDEXED (type_vec.c:101-107,
// type_ind.c:119-129)
enum Kind { K_BASIC = 0, K_CONTIG, K_HVECTOR, K_HINDEXED, K_STRUCT, K_UB, K_LB };

struct Info {
    int kind;
    int old;        // CONTIG: old type after flattening; HVECTOR / HINDEXED:
                    // the old type; STRUCT: old_types[0]; BASIC: itself
    int count;      // CONTIG: replication count
    int is_contig;  // the reference's is_contig
    int dense;      // 1: elements are `extent` bytes from the origin, moved
                    // whole (basic types, contiguous types of them); 0: the
                    // type map has holes -- moved packed (mvx_type_pack)
    long extent, size, lb, ub;
    long span_lo, span_hi;   // lowest / one past highest type-map byte of one element
};

// basic or derived handle; false for an unknown handle
bool info(int handle, Info *out);

}  // namespace dt
}  // namespace mvx

#endif
