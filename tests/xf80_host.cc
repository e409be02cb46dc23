// TEST INFRASTRUCTURE: the device's x87 emulation (mvapich-cce_amd/csrc/
// mvx_xf80.h) compiled for the host, so tests/test_cpu_xf80.py can compare
// it with the oracle's native x87 arithmetic on millions of bit patterns
// without a GPU.  Same calling convention as the oracle's orc_op.
#include <stddef.h>
#include "mvx_xf80.h"

using namespace xf;

extern "C" int xf_host_op(int op, int dtype, const void *in, void *inout, long n)
{
    if (dtype == 12) {
        const xf80 *b = (const xf80 *)in;
        xf80 *a = (xf80 *)inout;
        for (long i = 0; i < n; ++i) {
            switch (op) {
            case 100: a[i] = max(a[i], b[i]); break;
            case 101: a[i] = min(a[i], b[i]); break;
            case 102: a[i] = add(a[i], b[i]); break;
            case 103: a[i] = mul(a[i], b[i]); break;
            case 104: a[i] = land(a[i], b[i]); break;
            case 106: a[i] = lor(a[i], b[i]); break;
            case 108: a[i] = lxor(a[i], b[i]); break;
            default: return -1;
            }
        }
        return 0;
    }
    if (dtype == 22) {
        const pxi *b = (const pxi *)in;
        pxi *a = (pxi *)inout;
        for (long i = 0; i < n; ++i) {
            if (op == 111) a[i] = loc<false>(a[i], b[i]);
            else if (op == 110) a[i] = loc<true>(a[i], b[i]);
            else return -1;
        }
        return 0;
    }
    return -1;
}
