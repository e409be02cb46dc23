#pragma once
// mvx_ops_kern.h -- kernels and kernel sets of the device side of the MPI local
// reduction path (included by mvx_ops.hip and the per-op table units
// mvx_ops_{cmp,arith,logic,loc}.hip, compiled in parallel), written for
// gfx950 (CDNA4, wave64).  Built into libmvx_hip.so; C-ABI in
// include/mvx_hip.h.
//
// One kernel template covers every predefined op x type of the reference
// (src/coll/global_ops.c:56-1745) and every combine order of its collectives
// (src/coll/intra_fns_new.c): a launch reads k leaf operands (optionally each
// pre-folded with a partner, the non-power-of-two fold of intra_fns_new.c
// 5548-5577 / 4641-4671 / 6283-6312), reduces them in registers by a small
// combine program (tree steps by level, then a chain; include/mvx_hip.h)
// whose left operand always plays the reference's `inoutvec` role, and
// writes the result once.  A k-way combine is one HBM pass instead
// of the reference's log2(p) or p-1 passes over the block.
//
// Element-wise: no MFMA, no LDS.  Every lane moves 16 bytes per operand per
// chunk (global_load_dwordx4), chunks are lane-contiguous so a wave touches
// 1 KiB per load instruction, several chunks per lane are in flight before
// the first use, and the store is one dwordx4 per chunk.  Pair types
// (MAXLOC/MINLOC) are 8 or 16 bytes, so a 16-byte lane load always holds
// whole pairs: no LDS transposition is needed.
//
// Numerics follow the reference's x86-64 gcc -O2 build: IEEE round-to-nearest
// f32/f64 with denormals (no flush), no contraction (-ffp-contract=off keeps
// the complex product of global_ops.c:518-519 unfused), MAX/MIN as the
// select `(b > a) ? b : a` of coll.h:14-19 (not v_max: NaN and signed-zero
// roles matter), integer arithmetic in unsigned form (the reference's signed
// wrap, without UB).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "mvx_mpi.h"
#include "mvx_hip.h"
#include "mvx_xf80.h"
#include "mvx_dtype.h"

namespace mvx {

enum { OMAX = 0, OMIN, OSUM, OPROD, OLAND, OBAND, OLOR, OBOR, OLXOR, OBXOR,
       OMINLOC, OMAXLOC };

// Element layouts: the reference's C types on x86-64 LP64.
struct cf32 { float re, im; };                          // global_ops.c:43-46
struct cf64 { double re, im; };                         // global_ops.c:48-51
struct pfi { float v; int32_t l; };                     // initdte.c:74-78
// The padding is an explicit member so the inout operand's padding bytes are
// carried through the register copy and written back unchanged (an unnamed
// hole is `undef` to LLVM); the reference never writes them either
// (global_ops.c:1335-1346 assign value and loc only).
struct pdi { double v; int32_t l; int32_t pad; };       // 16 B
struct pli { int64_t v; int32_t l; int32_t pad; };      // 16 B
struct psi { int16_t v; int16_t pad; int32_t l; };      // 8 B
struct pii { int32_t v; int32_t l; };                   // MPI_2INT
static_assert(sizeof(pdi) == 16 && sizeof(pli) == 16 && sizeof(psi) == 8, "");
// contiguous count-2 types over one base type (MPI_2INT's family, e.g.
// MPI_Type_contiguous(2, MPI_FLOAT)): value and loc both of the base type,
// global_ops.c:1387-1503 / 1625-1740
template <typename B> struct pp { B v; B l; };
static_assert(sizeof(pp<int8_t>) == 2 && sizeof(pp<double>) == 16, "");

// x87 long double (16-byte slot) and MPI_LONG_DOUBLE_INT (32 bytes):
// integer emulation of the x87 unit, mvx_xf80.h
using xf::xf80;
using xf::pxi;
static_assert(sizeof(xf80) == 16 && sizeof(pxi) == 32, "");
template <typename B> struct pp;

// the x87 types: every op is dozens of integer instructions, so their
// combines are ALU-bound and keep full occupancy (no k_tree_body, no
// residency cap: the 8-leaf x87 SUM tree ran 109.7 us at 2 blocks per CU
// against 74.4 us uncapped, profiles/r02/bench_kernels_x87.jsonl).  The
// MPI_LONG_DOUBLE_INT MAXLOC / MINLOC trees have their own body kernel,
// k_pxi_loc_body (one element per lane pair).
template <typename T> struct alu_heavy { static constexpr bool v = false; };
template <> struct alu_heavy<xf80> { static constexpr bool v = true; };
template <> struct alu_heavy<pxi> { static constexpr bool v = true; };
template <> struct alu_heavy<pp<xf80>> { static constexpr bool v = true; };

// ---------------------------------------------------------------------------
// the ops: F<op, T>::f(a, b) returns the new inout value (a = inout, b = in)

template <int O, typename T> struct F;

template <typename T> struct F<OMAX, T> {     // coll.h:17-18
    static __device__ __forceinline__ T f(T a, T b) { return (b > a) ? b : a; }
};
template <typename T> struct F<OMIN, T> {     // coll.h:14-15
    static __device__ __forceinline__ T f(T a, T b) { return (a > b) ? b : a; }
};

template <typename T> __device__ __forceinline__ T add_(T a, T b) { return (T)(a + b); }
template <typename T> __device__ __forceinline__ T mul_(T a, T b) { return (T)(a * b); }
// promote narrow unsigned before multiplying so the product cannot overflow int
template <> __device__ __forceinline__ uint8_t mul_(uint8_t a, uint8_t b)
{ return (uint8_t)((uint32_t)a * (uint32_t)b); }
template <> __device__ __forceinline__ uint16_t mul_(uint16_t a, uint16_t b)
{ return (uint16_t)((uint32_t)a * (uint32_t)b); }

template <typename T> struct F<OSUM, T> {
    static __device__ __forceinline__ T f(T a, T b) { return add_(a, b); }
};
template <> struct F<OSUM, cf32> {
    static __device__ __forceinline__ cf32 f(cf32 a, cf32 b)
    { cf32 r; r.re = a.re + b.re; r.im = a.im + b.im; return r; }
};
template <> struct F<OSUM, cf64> {
    static __device__ __forceinline__ cf64 f(cf64 a, cf64 b)
    { cf64 r; r.re = a.re + b.re; r.im = a.im + b.im; return r; }
};
template <typename T> struct F<OPROD, T> {
    static __device__ __forceinline__ T f(T a, T b) { return mul_(a, b); }
};
template <> struct F<OPROD, cf32> {            // global_ops.c:513-521
    static __device__ __forceinline__ cf32 f(cf32 c, cf32 b)
    { cf32 r; r.re = c.re * b.re - c.im * b.im; r.im = c.im * b.re + c.re * b.im; return r; }
};
template <> struct F<OPROD, cf64> {            // global_ops.c:523-531
    static __device__ __forceinline__ cf64 f(cf64 c, cf64 b)
    { cf64 r; r.re = c.re * b.re - c.im * b.im; r.im = c.im * b.re + c.re * b.im; return r; }
};
template <typename T> struct F<OLAND, T> {
    static __device__ __forceinline__ T f(T a, T b) { return (a != T(0) && b != T(0)) ? T(1) : T(0); }
};
template <typename T> struct F<OLOR, T> {
    static __device__ __forceinline__ T f(T a, T b) { return (a != T(0) || b != T(0)) ? T(1) : T(0); }
};
template <typename T> struct F<OLXOR, T> {
    static __device__ __forceinline__ T f(T a, T b) { return ((a != T(0)) != (b != T(0))) ? T(1) : T(0); }
};
template <typename T> struct F<OBAND, T> {
    static __device__ __forceinline__ T f(T a, T b) { return (T)(a & b); }
};
template <typename T> struct F<OBOR, T> {
    static __device__ __forceinline__ T f(T a, T b) { return (T)(a | b); }
};
template <typename T> struct F<OBXOR, T> {
    static __device__ __forceinline__ T f(T a, T b) { return (T)(a ^ b); }
};
// MAXLOC / MINLOC: global_ops.c:1297-1309 and 1524-1536, as selects
// (no divergent branches): equal values keep a's value and the smaller loc;
// otherwise b wins only if strictly larger (smaller); a NaN on either side
// compares false both ways, so a is kept.  The padding member comes from a.
template <typename T, bool MIN>
__device__ __forceinline__ T loc_op(T a, T b)
{
    const bool eq = a.v == b.v;
    const bool take = MIN ? (a.v > b.v) : (a.v < b.v);
    const decltype(a.l) lmin = (a.l > b.l) ? b.l : a.l;   // MPIR_MIN, coll.h:14-15
    T r = a;
    r.v = take ? b.v : a.v;
    r.l = eq ? lmin : (take ? b.l : a.l);
    return r;
}
template <typename T> struct F<OMAXLOC, T> {
    static __device__ __forceinline__ T f(T a, T b) { return loc_op<T, false>(a, b); }
};
template <typename T> struct F<OMINLOC, T> {
    static __device__ __forceinline__ T f(T a, T b) { return loc_op<T, true>(a, b); }
};

// the x87 types (global_ops.c:149-155 and the HAVE_LONG_DOUBLE case of every
// op; 1365-1378 / 1605-1618 for LONG_DOUBLE_INT)
template <> struct F<OMAX, xf80> { static __device__ __forceinline__ xf80 f(xf80 a, xf80 b) { return xf::max(a, b); } };
template <> struct F<OMIN, xf80> { static __device__ __forceinline__ xf80 f(xf80 a, xf80 b) { return xf::min(a, b); } };
template <> struct F<OSUM, xf80> { static __device__ __forceinline__ xf80 f(xf80 a, xf80 b) { return xf::add(a, b); } };
template <> struct F<OPROD, xf80> { static __device__ __forceinline__ xf80 f(xf80 a, xf80 b) { return xf::mul(a, b); } };
template <> struct F<OLAND, xf80> { static __device__ __forceinline__ xf80 f(xf80 a, xf80 b) { return xf::land(a, b); } };
template <> struct F<OLOR, xf80> { static __device__ __forceinline__ xf80 f(xf80 a, xf80 b) { return xf::lor(a, b); } };
template <> struct F<OLXOR, xf80> { static __device__ __forceinline__ xf80 f(xf80 a, xf80 b) { return xf::lxor(a, b); } };
template <> struct F<OMAXLOC, pxi> { static __device__ __forceinline__ pxi f(pxi a, pxi b) { return xf::loc<false>(a, b); } };
template <> struct F<OMINLOC, pxi> { static __device__ __forceinline__ pxi f(pxi a, pxi b) { return xf::loc<true>(a, b); } };

// contiguous(2, MPI_LONG_DOUBLE) pairs (global_ops.c:1483-1496, 1720-1733):
// x87 compares of the values; equal -> loc = MPIR_MIN(a.l, b.l) (x87 select);
// b strictly larger (smaller) -> both of b's 10-byte values.  Each slot's
// padding stays the inout operand's.
template <bool MIN>
__device__ __forceinline__ pp<xf80> xloc2(pp<xf80> a, pp<xf80> b)
{
    const int c = xf::cmp(a.v, b.v);
    pp<xf80> r = a;
    if (c == 0) {
        r.l = xf::min(a.l, b.l);
    } else if (c == (MIN ? 1 : -1)) {
        r.v = xf::with_bits(a.v, b.v.m, b.v.se);
        r.l = xf::with_bits(a.l, b.l.m, b.l.se);
    }
    return r;
}
template <> struct F<OMAXLOC, pp<xf80>> { static __device__ __forceinline__ pp<xf80> f(pp<xf80> a, pp<xf80> b) { return xloc2<false>(a, b); } };
template <> struct F<OMINLOC, pp<xf80>> { static __device__ __forceinline__ pp<xf80> f(pp<xf80> a, pp<xf80> b) { return xloc2<true>(a, b); } };

#ifdef MVX_OPS_LOGICAL_TU   // one TU owns the .TRUE. / .FALSE. words (mvx_ops_logic.hip)
// MPI_LOGICAL (dte_type MPIR_LOGICAL, one MPI_Fint): LAND / LOR / LXOR
// compare each word with the Fortran .TRUE. and store .TRUE. or .FALSE.
// (global_ops.c:646-655, 875-884, 1104-1113 with mpi_fort.h:11-19:
// FROM_FLOG(x) = x == MPIR_F_TRUE, TO_FLOG(v) = v ? MPIR_F_TRUE :
// MPIR_F_FALSE).  BAND / BOR / BXOR are bitwise on the word (678-684 ...)
// and run the 32-bit integer kernels.
struct flog { int32_t v; };
__constant__ int32_t g_flog[2] = {1, 0};     // MPIR_F_TRUE, MPIR_F_FALSE (gfortran)
__device__ __forceinline__ flog to_flog(bool t) { flog r; r.v = t ? g_flog[0] : g_flog[1]; return r; }
template <> struct F<OLAND, flog> {
    static __device__ __forceinline__ flog f(flog a, flog b) { return to_flog(a.v == g_flog[0] && b.v == g_flog[0]); }
};
template <> struct F<OLOR, flog> {
    static __device__ __forceinline__ flog f(flog a, flog b) { return to_flog(a.v == g_flog[0] || b.v == g_flog[0]); }
};
template <> struct F<OLXOR, flog> {
    static __device__ __forceinline__ flog f(flog a, flog b) { return to_flog((a.v == g_flog[0]) != (b.v == g_flog[0])); }
};
#endif

// ---------------------------------------------------------------------------
// launch parameters (passed by value, ~170 bytes of kernarg)

struct Params {
    const char *src[MVX_COMBINE_KMAX];
    const char *fold[MVX_COMBINE_KMAX];
    char *dst;
    long n;      // elements
    long head;   // scalar elements before the 16-byte aligned body
    long nvec;   // chunks in the body (16 bytes, or one element if wider)
    int k;       // leaves
    int vec_ok;  // all pointers share their alignment mod 16
    unsigned tree_mask;   // bit l*8+q: y[q] = op(y[q], y[q + 2^l]), levels 0..2
    unsigned chain_mask;  // bit q (q >= 1): y[0] = op(y[0], y[q]) after the tree
};

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));  // one dwordx4

// A chunk is what one lane moves per operand per step: 16 bytes of
// elements, or one element of a wider type (MPI_LONG_DOUBLE_INT, 32 bytes:
// two dwordx4).  Moved to/from the registers by memcpy (a well-defined bit
// copy that keeps pair padding bytes; union punning lets clang drop the
// element writes).
template <typename T> struct CG {
    static constexpr int bytes = sizeof(T) > 16 ? (int)sizeof(T) : 16;
    static constexpr int w = bytes / 16;          // dwordx4 per chunk
    static constexpr int v = bytes / (int)sizeof(T);  // elements per chunk
};

template <typename T> struct Chunk {
    T e[CG<T>::v];
};
// 1-byte elements stay in their four 32-bit words (the SWAR chunk op, CF8):
// as 16 byte members the loads and stores were split into bytes and packed
// again around every op
template <> struct Chunk<uint8_t> { uint32_t w[4]; };
template <> struct Chunk<int8_t> { uint32_t w[4]; };

// The op over a whole chunk, a = op(a, b) element by element.  One-byte
// types run as SWAR on the chunk's four 32-bit words: element by element
// the compiler extracted, combined and re-packed every byte, and the 1-byte
// apply kernels ran at 0.65-0.73 of HBM peak against 0.78-0.81 for every
// wider type (tools/bench_kernels.py all, profiles/r05/bench_kernels_all.jsonl).
template <int O, typename T>
struct CF {
    static __device__ __forceinline__ void f(Chunk<T> &a, const Chunk<T> &b)
    {
#pragma unroll
        for (int j = 0; j < CG<T>::v; ++j) a.e[j] = F<O, T>::f(a.e[j], b.e[j]);
    }
};

typedef uint16_t u16x2 __attribute__((ext_vector_type(2)));   // one packed-16 register

// per byte of a word: 0x80 if the byte is nonzero, else 0
__device__ __forceinline__ uint32_t swar_nz(uint32_t x)
{
    return (((x & 0x7f7f7f7fu) + 0x7f7f7f7fu) | x) & 0x80808080u;
}

// bytes as two packed-16 lanes each (even bytes, odd bytes), op lane-wise,
// low 8 bits of each lane kept: unsigned MAX / MIN, wrapping PROD
template <int O>
__device__ __forceinline__ uint32_t swar_p16(uint32_t a, uint32_t b)
{
    const uint32_t ae = a & 0x00ff00ffu, ao = (a >> 8) & 0x00ff00ffu;
    const uint32_t be = b & 0x00ff00ffu, bo = (b >> 8) & 0x00ff00ffu;
    u16x2 xe, xo, ye, yo, re, ro;
    __builtin_memcpy(&xe, &ae, 4); __builtin_memcpy(&xo, &ao, 4);
    __builtin_memcpy(&ye, &be, 4); __builtin_memcpy(&yo, &bo, 4);
    if constexpr (O == OMAX) { re = __builtin_elementwise_max(xe, ye); ro = __builtin_elementwise_max(xo, yo); }
    else if constexpr (O == OMIN) { re = __builtin_elementwise_min(xe, ye); ro = __builtin_elementwise_min(xo, yo); }
    else { re = xe * ye; ro = xo * yo; }
    uint32_t e, o;
    __builtin_memcpy(&e, &re, 4); __builtin_memcpy(&o, &ro, 4);
    return (e & 0x00ff00ffu) | ((o & 0x00ff00ffu) << 8);
}

// one word of four 1-byte elements, op O; SIGNED: int8_t MAX / MIN
template <int O, bool SIGNED>
__device__ __forceinline__ uint32_t swar8(uint32_t a, uint32_t b)
{
    if constexpr (O == OBAND) return a & b;
    else if constexpr (O == OBOR) return a | b;
    else if constexpr (O == OBXOR) return a ^ b;
    else if constexpr (O == OSUM) return ((a & 0x7f7f7f7fu) + (b & 0x7f7f7f7fu)) ^ ((a ^ b) & 0x80808080u);
    else if constexpr (O == OLAND) return (swar_nz(a) & swar_nz(b)) >> 7;
    else if constexpr (O == OLOR) return (swar_nz(a) | swar_nz(b)) >> 7;
    else if constexpr (O == OLXOR) return (swar_nz(a) ^ swar_nz(b)) >> 7;
    else if constexpr (SIGNED) return swar_p16<O>(a ^ 0x80808080u, b ^ 0x80808080u) ^ 0x80808080u;   // biased order
    else return swar_p16<O>(a, b);
}

template <int O, bool SIGNED>
struct CF8 {
    template <typename T>
    static __device__ __forceinline__ void f(Chunk<T> &a, const Chunk<T> &b)
    {
#pragma unroll
        for (int w = 0; w < 4; ++w) a.w[w] = swar8<O, SIGNED>(a.w[w], b.w[w]);
    }
};
template <int O> struct CF<O, uint8_t> {
    static __device__ __forceinline__ void f(Chunk<uint8_t> &a, const Chunk<uint8_t> &b) { CF8<O, false>::f(a, b); }
};
template <int O> struct CF<O, int8_t> {
    static __device__ __forceinline__ void f(Chunk<int8_t> &a, const Chunk<int8_t> &b) { CF8<O, true>::f(a, b); }
};

// whole-element store: the pair padding is an explicit member carried from
// leaf 0, so the element path writes the same bytes as the 16-byte path
template <typename T>
__device__ __forceinline__ void store_elt(T *d, const T &r) { *d = r; }

// The combine program.  KMAX = 2 is the plain op (y0 = y0 op y1); for
// KMAX = 8 every step is fixed at compile time and switched on by a
// wave-uniform mask bit, so the leaves stay in registers.
template <int O, typename T, int KMAX>
__device__ __forceinline__ void reduce_leaves(T (&y)[KMAX], int k, unsigned tree_mask,
                                              unsigned chain_mask)
{
    if constexpr (KMAX == 2) {
        if (k == 2) y[0] = F<O, T>::f(y[0], y[1]);
    } else {
#pragma unroll
        for (int l = 0; (1 << l) < KMAX; ++l) {
#pragma unroll
            for (int q = 0; q + (1 << l) < KMAX; ++q)
                if (tree_mask & (1u << (l * 8 + q))) y[q] = F<O, T>::f(y[q], y[q + (1 << l)]);
        }
#pragma unroll
        for (int q = 1; q < KMAX; ++q)
            if (chain_mask & (1u << q)) y[0] = F<O, T>::f(y[0], y[q]);
    }
}

template <int O, typename T, int KMAX>
__device__ __forceinline__ void scalar_elem(const Params &P, long i)
{
    T y[KMAX];
#pragma unroll
    for (int q = 0; q < KMAX; ++q) {
        if (q < P.k) {
            y[q] = reinterpret_cast<const T *>(P.src[q])[i];
            if (P.fold[q]) y[q] = F<O, T>::f(y[q], reinterpret_cast<const T *>(P.fold[q])[i]);
        }
    }
    reduce_leaves<O, T, KMAX>(y, P.k, P.tree_mask, P.chain_mask);
    store_elt(reinterpret_cast<T *>(P.dst) + i, y[0]);
}

// U = 16-byte chunks per lane per iteration (loads in flight per operand).
// NT = non-temporal loads and stores (global_load/store_dwordx4 ... nt): for
// a launch that streams far more than the 256 MiB Infinity Cache, keeping the
// once-touched lines out of the caches measured 6.59 vs 5.68 TB/s on the
// config-2 kernel (tools/tune_sum.hip, cold caches).
template <int NT>
__device__ __forceinline__ u32x4 ld(const u32x4 *p)
{
    if constexpr (NT) return __builtin_nontemporal_load(p);
    else return *p;
}

// OPAQUE: an empty asm makes the stored dwordx4 opaque first.  Where the
// value was assembled from narrower fields (the x87 types' 16-bit sign and
// exponent) the optimiser otherwise re-typed the store and dropped its
// non-temporal hint (the x87 MAXLOC / MINLOC trees stored cached); for the
// other types the store already keeps it and their code stays as measured.
template <int NT, bool OPAQUE = false>
__device__ __forceinline__ void st(u32x4 *p, u32x4 v)
{
    if constexpr (NT) {
        if constexpr (OPAQUE) __asm__("" : "+v"(v));
        __builtin_nontemporal_store(v, p);
    } else {
        *p = v;
    }
}

template <typename T, int NT>
__device__ __forceinline__ Chunk<T> ld_chunk(const u32x4 *base, long c)
{
    u32x4 r[CG<T>::w];
#pragma unroll
    for (int w = 0; w < CG<T>::w; ++w) r[w] = ld<NT>(base + c * CG<T>::w + w);
    Chunk<T> x;
    __builtin_memcpy(&x, r, sizeof x);
    return x;
}

template <typename T, int NT>
__device__ __forceinline__ void st_chunk(u32x4 *base, long c, const Chunk<T> &x)
{
    u32x4 r[CG<T>::w];
    __builtin_memcpy(r, &x, sizeof x);
#pragma unroll
    for (int w = 0; w < CG<T>::w; ++w) st<NT, alu_heavy<T>::v>(base + c * CG<T>::w + w, r[w]);
}

// PROG = 0: the program comes from the masks (any chain of trees over
// k <= KMAX leaves); PROG = 1: the full balanced tree over exactly KMAX
// leaves, steps fixed at compile time -- the Allreduce / Reduce order at
// p = 4 and 8 (Rabenseifner), where the generic form evaluated and
// discarded 24 masked steps for the 7 the tree needs.
template <int O, typename T, int KMAX, int U, int NT, int PROG = 0>
__global__ void __launch_bounds__(256)
k_combine(const Params P)
{
    // the launch may reserve dynamic LDS to cap resident blocks per CU
    // (launch(), g_cap); the kernel never uses it -- the reference here
    // (never taken) marks the kernel as one that takes dynamic LDS
    extern __shared__ char lds_cap[];
    if (P.n < 0) lds_cap[threadIdx.x] = 0;
    constexpr int V = CG<T>::v;
    const long tid = (long)blockIdx.x * 256 + threadIdx.x;
    const long nthr = (long)gridDim.x * 256;

    if (!P.vec_ok) {  // operands misaligned against each other: element loads
        for (long i = tid; i < P.n; i += nthr) scalar_elem<O, T, KMAX>(P, i);
        return;
    }
    {   // head and tail elements outside the aligned body
        const long tail0 = P.head + P.nvec * V;
        const long nscal = P.head + (P.n - tail0);
        for (long s = tid; s < nscal; s += nthr) {
            const long i = s < P.head ? s : tail0 + (s - P.head);
            scalar_elem<O, T, KMAX>(P, i);
        }
    }
    const u32x4 *src[KMAX];
    const u32x4 *fold[KMAX];
#pragma unroll
    for (int q = 0; q < KMAX; ++q) {
        src[q] = reinterpret_cast<const u32x4 *>(P.src[q] + P.head * (long)sizeof(T));
        fold[q] = P.fold[q] ? reinterpret_cast<const u32x4 *>(P.fold[q] + P.head * (long)sizeof(T)) : nullptr;
    }
    u32x4 *dst = reinterpret_cast<u32x4 *>(P.dst + P.head * (long)sizeof(T));
    const int k = P.k;
    const unsigned tmask = P.tree_mask, cmask = P.chain_mask;

    for (long c0 = (long)blockIdx.x * (256 * U) + threadIdx.x; c0 < P.nvec; c0 += nthr * U) {
        Chunk<T> x[U][KMAX];
        // issue every load of the iteration before the first use
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long c = c0 + (long)u * 256;
            if (c < P.nvec) {
#pragma unroll
                for (int q = 0; q < KMAX; ++q)
                    if (PROG == 1 || q < k) x[u][q] = ld_chunk<T, NT>(src[q], c);
            }
        }
#pragma unroll
        for (int q = 0; q < KMAX; ++q) {
            // fixed trees are launched without folded leaves (mvx_op_program):
            // no branch between the loads and the tree keeps every load of
            // the iteration in flight before the first add
            if (PROG == 0 && q < k && fold[q]) {
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const long c = c0 + (long)u * 256;
                    if (c < P.nvec) {
                        const Chunk<T> f = ld_chunk<T, NT>(fold[q], c);
                        CF<O, T>::f(x[u][q], f);
                    }
                }
            }
        }
        // the combine program: each wave-uniform step is tested once and
        // applied to all U*V elements of the batch (chunks past the end
        // compute on unloaded registers and are never stored)
        if constexpr (KMAX == 2) {
            if (k == 2) {
#pragma unroll
                for (int u = 0; u < U; ++u)
                    CF<O, T>::f(x[u][0], x[u][1]);
            }
        } else if constexpr (PROG == 1) {
#pragma unroll
            for (int h = 1; h < KMAX; h <<= 1)
#pragma unroll
                for (int q = 0; q + h < KMAX; q += 2 * h)
#pragma unroll
                    for (int u = 0; u < U; ++u)
                        CF<O, T>::f(x[u][q], x[u][q + h]);
        } else {
#pragma unroll
            for (int l = 0; (1 << l) < KMAX; ++l) {
#pragma unroll
                for (int q = 0; q + (1 << l) < KMAX; ++q) {
                    if (tmask & (1u << (l * 8 + q))) {
#pragma unroll
                        for (int u = 0; u < U; ++u)
                            CF<O, T>::f(x[u][q], x[u][q + (1 << l)]);
                    }
                }
            }
#pragma unroll
            for (int q = 1; q < KMAX; ++q) {
                if (cmask & (1u << q)) {
#pragma unroll
                    for (int u = 0; u < U; ++u)
                        CF<O, T>::f(x[u][0], x[u][q]);
                }
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long c = c0 + (long)u * 256;
            if (c < P.nvec) st_chunk<T, NT>(dst, c, x[u][0]);
        }
    }
}

// The fixed full tree over the aligned body only: what a large C3 / C5
// combine is once the plan's blocks are 16-byte aligned and whole (no head,
// no tail, no folded leaves).  Its prologue is a handful of scalar loads
// (k_combine's head / tail / misalignment paths are gone), which matters at
// the few resident blocks per CU the residency cap leaves
// (tools/tune_occ.hip: the same loop behind k_combine's prologue ran 2 us
// slower per 50 us launch).
struct BodyParams {
    const u32x4 *src[8];
    u32x4 *dst;
    long nvec;   // chunks
    int k;       // leaves (k_chain_body<..., 8, ...>: 5 to 8)
};

// 56 KiB of static LDS per block: 2 resident blocks (8 waves) per CU.
// tools/tune_occ.hip, profiles/r02/tune_occ_lds.jsonl: the 8-leaf f32 tree
// at U = 2 runs 47.8 / 94.5 us (8 x 32 / 64 MiB leaves, 79 / 80 % of HBM
// peak) at 2 blocks per CU against 50.0 / 100.3 us at 3, 4 or 5 -- fewer,
// fuller waves keep each HBM channel on fewer rows.  (LDS reservations of
// 41-52 KiB, which the runtime's occupancy query calls 3 blocks per CU, run
// like 3; 53 KiB and up like 2.)
#define BODY_LDS_CAP (56 * 1024)
#ifndef BODY_ST_NT
#define BODY_ST_NT 1   // non-temporal result stores (cached: C4 204.8 -> 215.0 us, C5 96.1 -> 97.1, C3 unchanged)
#endif

template <int O, typename T, int KMAX, int U>
__global__ void __launch_bounds__(256)
k_tree_body(const BodyParams P)
{
    __shared__ char lds_cap[BODY_LDS_CAP];
    if (P.nvec < 0) lds_cap[threadIdx.x] = 0;
    const long nthr = (long)gridDim.x * 256;
    for (long c0 = (long)blockIdx.x * (256 * U) + threadIdx.x; c0 < P.nvec; c0 += nthr * U) {
        Chunk<T> x[U][KMAX];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long c = c0 + (long)u * 256;
            if (c < P.nvec)
#pragma unroll
                for (int q = 0; q < KMAX; ++q) x[u][q] = ld_chunk<T, 1>(P.src[q], c);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long c = c0 + (long)u * 256;
            if (c < P.nvec) {
#pragma unroll
                for (int h = 1; h < KMAX; h <<= 1)
#pragma unroll
                    for (int q = 0; q + h < KMAX; q += 2 * h)
                        CF<O, T>::f(x[u][q], x[u][q + h]);
                st_chunk<T, BODY_ST_NT>(P.dst, c, x[u][0]);
            }
        }
    }
}

// The same over a full CHAIN ((y0 op y1) op y2) ..., the pairwise
// Reduce_scatter's order (C4: k = 4, p = 4).  The 8-leaf instantiation
// takes chains of 5 to 8 leaves (P.k, a wave-uniform test per leaf): the
// pairwise chains at p = 5, 6, 7, which otherwise run the masked program at
// one chunk per lane.
template <int O, typename T, int KMAX, int U>
__global__ void __launch_bounds__(256)
k_chain_body(const BodyParams P)
{
    __shared__ char lds_cap[BODY_LDS_CAP];
    if (P.nvec < 0) lds_cap[threadIdx.x] = 0;
    const int k = KMAX == 8 ? P.k : KMAX;
    const long nthr = (long)gridDim.x * 256;
    for (long c0 = (long)blockIdx.x * (256 * U) + threadIdx.x; c0 < P.nvec; c0 += nthr * U) {
        Chunk<T> x[U][KMAX];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long c = c0 + (long)u * 256;
            if (c < P.nvec)
#pragma unroll
                for (int q = 0; q < KMAX; ++q)
                    if (q < k) x[u][q] = ld_chunk<T, 1>(P.src[q], c);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long c = c0 + (long)u * 256;
            if (c < P.nvec) {
#pragma unroll
                for (int q = 1; q < KMAX; ++q)
                    if (q < k) CF<O, T>::f(x[u][0], x[u][q]);
                st_chunk<T, BODY_ST_NT>(P.dst, c, x[u][0]);
            }
        }
    }
}

// MPI_LONG_DOUBLE_INT MAXLOC / MINLOC (global_ops.c:1365-1378 / 1605-1618)
// as lane PAIRS.  An element is 32 bytes: the x87 value in the first 16
// (significand, sign / exponent, slot padding), the int loc and padding in
// the second.  One element per lane made every load instruction touch 2 KiB
// with half of each 128-byte line (the tree ran at 65 % of HBM peak whatever
// its occupancy, profiles/r03/bench_kernels_x87_cap_sweep.jsonl); here lane
// 2j holds the value half of element j and lane 2j+1 its loc half, so each
// load and store is 1 KiB contiguous per wave.  The even lane compares, one
// DPP quad permutation hands the result to its odd partner, and each lane
// selects its own half: value and sign / exponent from the winner with a's
// slot padding (even), loc as the reference sets it (odd).
template <bool MIN>
__device__ __forceinline__ u32x4 loc_half(u32x4 a, u32x4 b, bool odd)
{
    xf80 va, vb;
    __builtin_memcpy(&va, &a, sizeof va);
    __builtin_memcpy(&vb, &b, sizeof vb);
    // meaningful in even lanes: 1 = b wins, 2 = equal values, 0 = keep a
    const xf::xord o = xf::order(va, vb);
    const bool win = !o.un & (MIN ? o.gt : !(o.gt | o.eq));
    int code = win ? 1 : ((!o.un & o.eq) ? 2 : 0);
    code = __builtin_amdgcn_update_dpp(0, code, 0xA0, 0xF, 0xF, false);   // quad_perm [0, 0, 2, 2]
    const bool take = code == 1;
    const int32_t la = (int32_t)a.x, lb = (int32_t)b.x;
    const uint32_t lsel = code == 2 ? (uint32_t)(la < lb ? la : lb) : (take ? b.x : a.x);
    u32x4 r = a;
    r.x = odd ? lsel : (take ? b.x : a.x);
    r.y = odd ? a.y : (take ? b.y : a.y);
    r.z = odd ? a.z : (take ? ((b.z & 0xffffu) | (a.z & 0xffff0000u)) : a.z);
    return r;
}

// the full tree over KMAX leaves; BodyParams.nvec counts elements (32 B)
template <int O, int KMAX, int U>
__global__ void __launch_bounds__(256)
k_pxi_loc_body(const BodyParams P)
{
    // the launch may reserve dynamic LDS to cap resident blocks per CU
    extern __shared__ char lds_cap[];
    if (P.nvec < 0) lds_cap[threadIdx.x] = 0;
    constexpr bool MIN = O == OMINLOC;
    const long n = 2 * P.nvec;                 // 16-byte halves; even, so pairs stay whole
    const bool odd = threadIdx.x & 1;
    const long nthr = (long)gridDim.x * 256;
    for (long c0 = (long)blockIdx.x * (256 * U) + threadIdx.x; c0 < n; c0 += nthr * U) {
        u32x4 x[U][KMAX];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long c = c0 + (long)u * 256;
            if (c < n)
#pragma unroll
                for (int q = 0; q < KMAX; ++q) x[u][q] = ld<1>(P.src[q] + c);
        }
        // every lane runs the tree (lanes past the end on unloaded
        // registers, never stored), so the DPP partner is always active
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int h = 1; h < KMAX; h <<= 1)
#pragma unroll
                for (int q = 0; q + h < KMAX; q += 2 * h) x[u][q] = loc_half<MIN>(x[u][q], x[u][q + h], odd);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long c = c0 + (long)u * 256;
            if (c < n) st<BODY_ST_NT, true>(P.dst + c, x[u][0]);
        }
    }
}

}  // namespace mvx

// ---------------------------------------------------------------------------
// dispatch: (op, datatype handle) -> kernel set

namespace mvx {

typedef void (*KFn)(const Params);

// The launched template as rocprofv3 names it ("k_combine<2, float, 2, 4,
// 1>"), from the compiler's own spelling of the template arguments, so
// profiles and PMC summaries can be matched to what actually ran.
template <int O, typename T, int KMAX, int U, int NT, int PROG = 0>
static const char *ksym()
{
    static char buf[160];
    if (!buf[0]) {
        const char *pf = __PRETTY_FUNCTION__;
        const char *t = strstr(pf, "T = ");
        const char *e = t ? strstr(t, ", KMAX") : nullptr;
        const int tl = (t && e) ? (int)(e - t - 4) : 1;
        const char *tn = (t && e) ? t + 4 : "?";
        // every template argument, as rocprofv3 names the kernel
        snprintf(buf, sizeof buf, "k_combine<%d, %.*s, %d, %d, %d, %d>", O, tl, tn, KMAX, U, NT, PROG);
    }
    return buf;
}

typedef const char *(*SymFn)();

template <int O, typename T, int KMAX, int U>
static const char *ksym_chain_body()
{
    static char buf[160];
    if (!buf[0]) {
        const char *pf = __PRETTY_FUNCTION__;
        const char *t = strstr(pf, "T = ");
        const char *e = t ? strstr(t, ", KMAX") : nullptr;
        const int tl = (t && e) ? (int)(e - t - 4) : 1;
        const char *tn = (t && e) ? t + 4 : "?";
        snprintf(buf, sizeof buf, "k_chain_body<%d, %.*s, %d, %d>", O, tl, tn, KMAX, U);
    }
    return buf;
}

template <int O, typename T, int KMAX, int U>
static const char *ksym_body()
{
    static char buf[160];
    if (!buf[0]) {
        const char *pf = __PRETTY_FUNCTION__;
        const char *t = strstr(pf, "T = ");
        const char *e = t ? strstr(t, ", KMAX") : nullptr;
        const int tl = (t && e) ? (int)(e - t - 4) : 1;
        const char *tn = (t && e) ? t + 4 : "?";
        snprintf(buf, sizeof buf, "k_tree_body<%d, %.*s, %d, %d>", O, tl, tn, KMAX, U);
    }
    return buf;
}

// A kernel family: [0] the cached build, [1] the non-temporal one (NT), each
// with its chunks in flight per lane (U) and its residency class (FAM_*)
enum { FAM_APPLY = 0, FAM_PROG, FAM_TREE, FAM_N };
struct KFam {
    const void *fn[2];
    SymFn sym[2];
    int unroll[2];
    int fam;
    const void *body;      // k_tree_body / k_chain_body for large aligned launches, or null
    SymFn body_sym;
    int body_unroll;
    int body_k;            // the body kernel's leaf count (launches with other k never use it)
    int body_kmin;         // or, when set, the fewest leaves it takes (k_chain_body<..., 8, ...>: 5)
    int body_units;        // 16-byte units one body thread moves per element (k_pxi_loc_body: 2)
    int body_cap;          // resident blocks per CU by a dynamic LDS reservation (0: none)
};

struct KSet {
    KFam apply;            // KMAX 2 (k <= 2)
    KFam prog;             // KMAX 8 combine program (masks)
    KFam prog2;            // 4-byte types: the U = 2 program (MVX_PROG_U=2); fn[0] null otherwise
    KFam prog4;            // programs over 3 or 4 leaves: KMAX 4 at U = 2 (MVX_PROG4=0: prog)
    KFam tree8, tree4;     // PROG = 1: full trees over 8 / 4 leaves
    KFam chain8, chain4;   // full chains over 8 / 4 leaves: k_chain_body, else the masked program
    int esize;
    int chunk;             // bytes per chunk (16, or the element if wider)
    const char *name;
};

template <int O, int KMAX, int U>
static const char *ksym_pxi_body()
{
    static char buf[96];
    if (!buf[0]) snprintf(buf, sizeof buf, "k_pxi_loc_body<%d, %d, %d>", O, KMAX, U);
    return buf;
}

static inline int env_int(const char *name, int dflt)
{
    const char *e = getenv(name);
    return e ? atoi(e) : dflt;
}

template <int O, typename T, int KMAX, int U0, int U1, int PROG>
static KFam kfam(int fam)
{
    KFam f;
    f.fn[0] = (const void *)&k_combine<O, T, KMAX, U0, 0, PROG>;
    f.fn[1] = (const void *)&k_combine<O, T, KMAX, U1, 1, PROG>;
    f.sym[0] = &ksym<O, T, KMAX, U0, 0, PROG>;
    f.sym[1] = &ksym<O, T, KMAX, U1, 1, PROG>;
    f.unroll[0] = U0;
    f.unroll[1] = U1;
    f.fam = (fam == FAM_TREE && alu_heavy<T>::v) ? FAM_PROG : fam;
    f.body_units = 1;
    f.body_cap = 0;
    f.body_kmin = 0;
    if constexpr (PROG == 1 && !alu_heavy<T>::v) {
        f.body = (const void *)&k_tree_body<O, T, KMAX, U1>;
        f.body_sym = &ksym_body<O, T, KMAX, U1>;
        f.body_unroll = U1;
        f.body_k = KMAX;
    } else if constexpr (PROG == 1 && std::is_same<T, pxi>::value && (O == OMAXLOC || O == OMINLOC)) {
        // one element per lane pair at 4 resident blocks per CU: 8 x 64 MiB
        // MAXLOC tree 96.4 us (78 % of HBM peak) against 115-117 us one
        // element per lane; U = 2 at 3 blocks 96.2-96.9, uncapped 99-101
        // (profiles/r03/bench_kernels_x87_pair_sweep.jsonl); MVX_PXI_U /
        // MVX_PXI_CAP for A/B runs
        const int u = env_int("MVX_PXI_U", 1);
        f.body = u == 2 ? (const void *)&k_pxi_loc_body<O, KMAX, 2> : (const void *)&k_pxi_loc_body<O, KMAX, 1>;
        f.body_sym = u == 2 ? &ksym_pxi_body<O, KMAX, 2> : &ksym_pxi_body<O, KMAX, 1>;
        f.body_unroll = u == 2 ? 2 : 1;
        f.body_k = KMAX;
        f.body_units = 2;
        f.body_cap = env_int("MVX_PXI_CAP", 4);
    } else {
        f.body = nullptr;
        f.body_sym = nullptr;
        f.body_unroll = 0;
        f.body_k = 0;
    }
    return f;
}

// a full chain: the masked program, with k_chain_body for large aligned launches
template <int O, typename T, int KMAX>
static KFam kchain()
{
    KFam f = kfam<O, T, MVX_COMBINE_KMAX, 1, 1, 0>(FAM_PROG);
    if constexpr (!alu_heavy<T>::v) {
        f.body = (const void *)&k_chain_body<O, T, KMAX, 2>;
        f.body_sym = &ksym_chain_body<O, T, KMAX, 2>;
        f.body_unroll = 2;
        f.body_k = KMAX;
        f.body_kmin = KMAX == 8 ? 5 : 0;
    }
    return f;
}

// Chunks in flight per lane, and (launch()) resident blocks per CU, for the
// non-temporal (large) launches -- round 2, tools/tune_occ.hip,
// profiles/r02/tune_occ.jsonl: at full occupancy a streaming launch keeps ~10x
// the bytes in flight Little's law needs and every HBM channel juggles rows
// from all the streams; fewer resident blocks with more loads each measured
// k = 8, 8 x 32 MiB: U1 uncapped 76.5 %, U2 at 2 blocks / CU 79.0 %;
// k = 8, 8 x 64 MiB: 77.0 % -> 79.9 % (BODY_LDS_CAP).  The plain op (k = 2)
// and the masked program gain nothing from a cap and keep U = 4 / 1 at full
// occupancy, as do the cached (small-launch) builds.
template <int O, typename T>
static KSet kset(const char *name)
{
    KSet s;
    s.apply = kfam<O, T, 2, 4, 4, 0>(FAM_APPLY);
    if constexpr (std::is_same<T, pxi>::value && (O == OMAXLOC || O == OMINLOC)) {
        // the plain op on MPI_LONG_DOUBLE_INT as lane pairs too (the trees'
        // k_pxi_loc_body with KMAX = 2): one 32-byte element per lane ran it
        // at 0.56 of HBM peak (profiles/r05/bench_kernels_all.jsonl)
        s.apply.body = (const void *)&k_pxi_loc_body<O, 2, 1>;
        s.apply.body_sym = &ksym_pxi_body<O, 2, 1>;
        s.apply.body_unroll = 1;
        s.apply.body_k = 2;
        s.apply.body_units = 2;
        s.apply.body_cap = env_int("MVX_PXI_APPLY_CAP", 4);
    }
    // (a 2-leaf body at U = 3 and 2 blocks per CU ran 123.8 vs 126.4 us in
    // the standalone sweep, profiles/r02/tune_occ_k2.jsonl, but 124.8 vs
    // 123.5-124.8 us in the product: not adopted)
    s.prog = kfam<O, T, MVX_COMBINE_KMAX, 1, 1, 0>(FAM_PROG);
    if constexpr (alu_heavy<T>::v) {
        // x87 (integer-emulated, ALU-bound) trees: U = 1 keeps 53-57 VGPRs
        // and 7-8 waves per SIMD (U = 2: 98, 4 waves); SUM tree k = 8 57.6 ->
        // 53.3 us (profiles/r02/bench_kernels_x87.jsonl)
        s.tree8 = kfam<O, T, 8, 1, 1, 1>(FAM_TREE);
        s.tree4 = kfam<O, T, 4, 1, 1, 1>(FAM_TREE);
    } else {
        s.tree8 = kfam<O, T, 8, 1, 2, 1>(FAM_TREE);
        s.tree4 = kfam<O, T, 4, 1, 2, 1>(FAM_TREE);
    }
    s.chain8 = kchain<O, T, 8>();
    s.chain4 = kchain<O, T, 4>();
    if constexpr (alu_heavy<T>::v) {
        s.prog4 = kfam<O, T, 4, 1, 1, 0>(FAM_PROG);
    } else {
        s.prog4 = kfam<O, T, 4, 2, 2, 0>(FAM_PROG);
    }
    if constexpr (sizeof(T) == 4) {
        s.prog2 = kfam<O, T, MVX_COMBINE_KMAX, 2, 2, 0>(FAM_PROG);
    } else {
        memset(&s.prog2, 0, sizeof s.prog2);
    }
    s.esize = (int)sizeof(T);
    s.chunk = CG<T>::bytes;
    s.name = name;
    return s;
}

// element kinds of the datatype handles (mvx_mpi.h / reference mpi.h:64-115)
enum { EK_NONE = 0, EK_I8, EK_U8, EK_BYTE, EK_I16, EK_U16, EK_I32, EK_U32,
       EK_I64, EK_U64, EK_F32, EK_F64, EK_C32, EK_C64, EK_PFI, EK_PDI, EK_PLI,
       EK_PSI, EK_PII, EK_LDBL, EK_LDBL_INT,
       // derived contiguous types: count-2 pairs of one base, and the rest
       EK_PP8, EK_PP16, EK_PP64, EK_PPF, EK_PPD, EK_PPX, EK_DERIVED,
       EK_LOGICAL };

// Integer SUM/PROD/logical/bitwise results do not depend on signedness in
// two's complement, so those share the unsigned kernel of the same width;
// MAX/MIN compare and keep the signed kernels.
#define ARITH_INT(O, NAME)                                                   \
    case EK_I8: case EK_U8:   { static KSet s = kset<O, uint8_t>(NAME "_u8"); return &s; } \
    case EK_I16: case EK_U16: { static KSet s = kset<O, uint16_t>(NAME "_u16"); return &s; } \
    case EK_I32: case EK_U32: { static KSet s = kset<O, uint32_t>(NAME "_u32"); return &s; } \
    case EK_I64: case EK_U64: { static KSet s = kset<O, uint64_t>(NAME "_u64"); return &s; }
#define FLOATS(O, NAME)                                                      \
    case EK_F32: { static KSet s = kset<O, float>(NAME "_f32"); return &s; } \
    case EK_F64: { static KSet s = kset<O, double>(NAME "_f64"); return &s; }
#define CMPLX(O, NAME)                                                       \
    case EK_C32: { static KSet s = kset<O, cf32>(NAME "_c32"); return &s; }  \
    case EK_C64: { static KSet s = kset<O, cf64>(NAME "_c64"); return &s; }
#define SIGNED_INT(O, NAME)                                                  \
    case EK_I8:  { static KSet s = kset<O, int8_t>(NAME "_i8"); return &s; } \
    case EK_U8:  { static KSet s = kset<O, uint8_t>(NAME "_u8"); return &s; } \
    case EK_I16: { static KSet s = kset<O, int16_t>(NAME "_i16"); return &s; } \
    case EK_U16: { static KSet s = kset<O, uint16_t>(NAME "_u16"); return &s; } \
    case EK_I32: { static KSet s = kset<O, int32_t>(NAME "_i32"); return &s; } \
    case EK_U32: { static KSet s = kset<O, uint32_t>(NAME "_u32"); return &s; } \
    case EK_I64: { static KSet s = kset<O, int64_t>(NAME "_i64"); return &s; } \
    case EK_U64: { static KSet s = kset<O, uint64_t>(NAME "_u64"); return &s; }
#define PAIRS(O, NAME)                                                       \
    case EK_PFI: { static KSet s = kset<O, pfi>(NAME "_float_int"); return &s; } \
    case EK_PDI: { static KSet s = kset<O, pdi>(NAME "_double_int"); return &s; } \
    case EK_PLI: { static KSet s = kset<O, pli>(NAME "_long_int"); return &s; } \
    case EK_PSI: { static KSet s = kset<O, psi>(NAME "_short_int"); return &s; } \
    case EK_PII: { static KSet s = kset<O, pii>(NAME "_2int"); return &s; }

#define LDBL(O, NAME)                                                        \
    case EK_LDBL: { static KSet s = kset<O, xf80>(NAME "_f80"); return &s; }
#define LDBL_INT(O, NAME)                                                    \
    case EK_LDBL_INT: { static KSet s = kset<O, pxi>(NAME "_long_double_int"); return &s; }
#define LOGICAL(O, NAME)                                                     \
    case EK_LOGICAL: { static KSet s = kset<O, flog>(NAME "_logical"); return &s; }
#define CONTIG_PAIRS(O, NAME)                                                \
    case EK_PP8:  { static KSet s = kset<O, pp<int8_t>>(NAME "_2char"); return &s; } \
    case EK_PP16: { static KSet s = kset<O, pp<int16_t>>(NAME "_2short"); return &s; } \
    case EK_PP64: { static KSet s = kset<O, pp<int64_t>>(NAME "_2long"); return &s; } \
    case EK_PPF:  { static KSet s = kset<O, pp<float>>(NAME "_2float"); return &s; } \
    case EK_PPD:  { static KSet s = kset<O, pp<double>>(NAME "_2double"); return &s; } \
    case EK_PPX:  { static KSet s = kset<O, pp<xf80>>(NAME "_2long_double"); return &s; }

// the per-op kernel tables, one translation unit each (nullptr: no case for
// that element kind in the op's switch -> the reference's 329)
const KSet *lookup_cmp(int op, int ek);     // MAX, MIN           mvx_ops_cmp.hip
const KSet *lookup_arith(int op, int ek);   // SUM, PROD          mvx_ops_arith.hip
const KSet *lookup_logic(int op, int ek);   // L* and B* ops      mvx_ops_logic.hip
int flog_sync();                            // MPI_LOGICAL's words on this device (mvx_ops_logic.hip)
const KSet *lookup_loc(int op, int ek);     // MAXLOC, MINLOC     mvx_ops_loc.hip

}  // namespace mvx

