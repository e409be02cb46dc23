/*
 * TEST INFRASTRUCTURE: MPI_User_function bodies for the user-op tests.
 * Compiled by tests/uops.py into a shared library; the same function
 * pointers are registered with the oracle (orc_user_op_set) and with the
 * product (MPI_Op_create), so both call identical code.
 *
 *   uop_addem   int      inout += in        (examples/test/coll/coll9.c, coll11.c)
 *   uop_assoc   int      order check: inout = in when in < inout, else a
 *                        100000 marker (coll10.c, coll11.c, scantst.c)
 *   uop_add_f64 double   inout = in + inout (longuser.c)
 *   uop_fsum    float    inout = in + inout (rounding shows the association)
 *   uop_mix     unsigned neither commutative nor associative: any change of
 *                        operand role or grouping changes the bits
 *   uop_affine  unsigned long: (a, b) in the two 32-bit halves is the map
 *                        x -> a*x + b; the result is in composed after
 *                        inout, which is associative but not commutative
 *   uop_idsum   struct {int a; (4-byte hole); double b}, a derived struct
 *                        type: a and b summed field by field, the hole
 *                        never read or written
 */
#include <stdint.h>

#define BAD_ANSWER 100000

void uop_addem(void *in, void *inout, int *len, int *dt)
{
    const int *a = (const int *)in;
    int *b = (int *)inout;
    (void)dt;
    for (int i = 0; i < *len; i++) b[i] += a[i];
}

void uop_assoc(void *in, void *inout, int *len, int *dt)
{
    const int *a = (const int *)in;
    int *b = (int *)inout;
    (void)dt;
    for (int i = 0; i < *len; i++) b[i] = (b[i] <= a[i]) ? BAD_ANSWER : a[i];
}

void uop_add_f64(void *in, void *inout, int *len, int *dt)
{
    const double *a = (const double *)in;
    double *b = (double *)inout;
    (void)dt;
    for (int i = 0; i < *len; i++) b[i] = a[i] + b[i];
}

void uop_fsum(void *in, void *inout, int *len, int *dt)
{
    const float *a = (const float *)in;
    float *b = (float *)inout;
    (void)dt;
    for (int i = 0; i < *len; i++) b[i] = a[i] + b[i];
}

void uop_mix(void *in, void *inout, int *len, int *dt)
{
    const uint32_t *a = (const uint32_t *)in;
    uint32_t *b = (uint32_t *)inout;
    (void)dt;
    for (int i = 0; i < *len; i++) {
        const uint32_t x = a[i], y = b[i];
        b[i] = x * 31u + (y ^ (y >> 3)) * 7u + 1u;
    }
}

/* uop_mix over a derived type of 3 unsigned words (MPI_Type_contiguous(3,
 * MPI_UNSIGNED)): *len counts derived elements, so 3 * *len words -- the
 * element-wise contract a user function has with its datatype */
int uop_last_dt;   /* the datatype handle uop_mix3 was last given */

void uop_mix3(void *in, void *inout, int *len, int *dt)
{
    int n = 3 * *len;
    uop_last_dt = *dt;
    uop_mix(in, inout, &n, dt);
}

void uop_affine(void *in, void *inout, int *len, int *dt)
{
    const uint64_t *a = (const uint64_t *)in;
    uint64_t *b = (uint64_t *)inout;
    (void)dt;
    for (int i = 0; i < *len; i++) {
        const uint32_t a1 = (uint32_t)a[i], b1 = (uint32_t)(a[i] >> 32);
        const uint32_t a2 = (uint32_t)b[i], b2 = (uint32_t)(b[i] >> 32);
        /* x -> a2*(a1*x + b1) + b2 */
        b[i] = (uint64_t)(a1 * a2) | ((uint64_t)(a2 * b1 + b2) << 32);
    }
}

typedef struct { int a; int hole; double b; } idpair_t;

void uop_idsum(void *in, void *inout, int *len, int *dt)
{
    const idpair_t *x = (const idpair_t *)in;
    idpair_t *y = (idpair_t *)inout;
    (void)dt;
    for (int i = 0; i < *len; i++) {
        y[i].a = (int)((unsigned)x[i].a + (unsigned)y[i].a);
        y[i].b = x[i].b + y[i].b;
    }
}
