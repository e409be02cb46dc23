// mvx_xf80.h -- x87 80-bit extended precision (`long double` on x86-64) in
// integer arithmetic, for MPI_LONG_DOUBLE / MPI_LONG_DOUBLE_INT on the
// device.
//
// The reference evaluates these types with the host's x87 unit
// (global_ops.c:149-155, 259-265, 376-382, 504-510, 637-643, 866-872,
// 1095-1101, 1365-1378, 1605-1618), under the x86-64 Linux default control
// word: 64-bit precision, round to nearest even, every exception masked.  The
// functions here reproduce that bit for bit, including what the masked
// exceptions leave behind:
//   * unsupported encodings (unnormals, pseudo-infinities, pseudo-NaNs) are
//     invalid operands: arithmetic returns the real indefinite QNaN
//     (sign 1, exponent 0x7fff, significand 0xC000000000000000) and every
//     comparison is unordered;
//   * pseudo-denormals (exponent 0, integer bit 1) are read as the
//     denormal exponent;
//   * inf - inf and 0 * inf give the real indefinite;
//   * a NaN operand propagates quieted.  Between two NaNs a QNaN beats an
//     SNaN, and between NaNs of one kind the larger significand wins (Intel
//     SDM vol. 1 table 4-7, x87 column);
//   * a tiny result is denormalised with one rounding at the denormal
//     position (masked underflow), and overflow gives infinity.
// tests/test_cpu_xf80.py checks all of this against this container's x87.
//
// Both host and device code compile this header: the host build is the
// fuzz harness that checks it against the oracle's x87.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define XF_FN __host__ __device__ __forceinline__
#else
#define XF_FN static inline
#endif

namespace xf {

// one MPI_LONG_DOUBLE element: the 10 bytes x87 stores plus the 6 bytes of
// its 16-byte slot, which an x87 store never writes (carried from the inout
// operand)
struct xf80 {
    uint64_t m;      // significand, explicit integer bit 63
    uint16_t se;     // sign 15, biased exponent 14..0
    uint16_t pad0;
    uint32_t pad1;
};

typedef unsigned __int128 u128;

enum { K_ZERO = 0, K_FIN, K_INF, K_QNAN, K_SNAN, K_BAD };

// written as selects: on the device every lane classifies its own operand,
// and nested ifs became exec-mask branches around each class
XF_FN int klass(uint64_t m, uint32_t e)
{
    const bool j = (m >> 63) != 0;
    const int top = !j ? K_BAD                      // pseudo-infinity / pseudo-NaN
                  : (m << 1) == 0 ? K_INF : ((m >> 62) & 1 ? K_QNAN : K_SNAN);
    const int bottom = m == 0 ? K_ZERO : K_FIN;     // denormal or pseudo-denormal
    const int mid = j ? K_FIN : K_BAD;              // unnormal
    return e == 0x7fff ? top : (e == 0 ? bottom : mid);
}

XF_FN xf80 with_bits(xf80 pads, uint64_t m, uint32_t se)
{
    xf80 r = pads;
    r.m = m;
    r.se = (uint16_t)se;
    return r;
}

XF_FN xf80 indefinite(xf80 pads) { return with_bits(pads, 0xC000000000000000ull, 0xffff); }

// result of an arithmetic op with a NaN operand (and no invalid encoding)
XF_FN xf80 nan_result(xf80 a, int ka, xf80 b, int kb)
{
    const bool na = ka == K_QNAN || ka == K_SNAN, nb = kb == K_QNAN || kb == K_SNAN;
    uint64_t m;
    uint32_t se;
    if (na && nb) {
        if (ka != kb) {                              // the QNaN wins
            m = ka == K_QNAN ? a.m : b.m;
            se = ka == K_QNAN ? a.se : b.se;
        } else if (a.m != b.m) {                     // larger significand
            m = a.m > b.m ? a.m : b.m;
            se = a.m > b.m ? a.se : b.se;
        } else {                                     // equal: ties go to b... see tests
            m = a.m;
            se = (a.se & b.se & 0x8000) | 0x7fff;
        }
    } else if (na) {
        m = a.m;
        se = a.se;
    } else {
        m = b.m;
        se = b.se;
    }
    return with_bits(a, m | (1ull << 62), se);
}

XF_FN int clz128(u128 x)
{
    const uint64_t hi = (uint64_t)(x >> 64), lo = (uint64_t)x;
    return hi ? __builtin_clzll(hi) : (lo ? 64 + __builtin_clzll(lo) : 128);
}

// round S (binary point after bit 64: significand = S >> 64) to 64 bits,
// nearest even, at effective exponent e >= 1; encode with sign s
XF_FN xf80 round_pack(xf80 pads, uint32_t s, int e, u128 S)
{
    uint64_t r = (uint64_t)(S >> 64);
    const uint64_t low = (uint64_t)S;
    if ((low >> 63) && ((low << 1) || (r & 1))) {
        if (++r == 0) {
            r = 1ull << 63;
            ++e;
        }
    }
    if (e >= 0x7fff) return with_bits(pads, 1ull << 63, (s << 15) | 0x7fff);   // overflow
    const uint32_t enc = (r >> 63) ? (uint32_t)e : 0u;                          // denormal
    return with_bits(pads, r, (s << 15) | enc);
}

// a + b for two normal operands (integer bit set, exponent 1..0x7ffe) whose
// exponents differ by at most 64, in 64-bit halves: the same value, rounding
// and encoding as add()'s general path (whose 128-bit shifts dominate the
// emulated add on the device), which handles everything else.  Returns false
// when the operands are outside that case.
//
// Written as selects: the same-sign sum and the opposite-sign difference
// (with its normalisation) are both computed and one is kept, and the
// rounding carry and the overflow are selects too.  Lanes of a wave disagree
// on the sign case about half the time on mixed-sign data, so a branch ran
// both sides anyway, plus the exec-mask bookkeeping around each.
XF_FN bool add_normal(xf80 a, xf80 b, xf80 *out)
{
    const uint32_t ea = a.se & 0x7fff, eb = b.se & 0x7fff;
    const bool normal = ea - 1u < 0x7ffeu && eb - 1u < 0x7ffeu && (a.m >> 63) && (b.m >> 63);
    // |a| >= |b| from here
    const bool swap = eb > ea || (eb == ea && b.m > a.m);
    const int xa = (int)(swap ? eb : ea), xb = (int)(swap ? ea : eb);
    const uint64_t ma = swap ? b.m : a.m, mb = swap ? a.m : b.m;
    const uint32_t sa = (swap ? b.se : a.se) >> 15, sb = (swap ? a.se : b.se) >> 15;
    const int d = xa - xb;
    if (!normal || d > 64) return false;
    // B = mb * 2^(64 - d) as hi:lo below A = ma:0 (no bit is lost for d <= 64)
    const uint64_t hi = d >= 64 ? 0 : mb >> (d & 63);
    const uint64_t lo = d == 0 ? 0 : (d >= 64 ? mb : mb << ((64 - d) & 63));
    // same signs: the sum, shifted right with a sticky bit on a carry out
    const uint64_t sh = ma + hi;
    const bool carry = sh < ma;
    const uint64_t add_h = carry ? ((sh >> 1) | (1ull << 63)) : sh;
    const uint64_t add_l = carry ? ((sh << 63) | (lo >> 1) | (lo & 1)) : lo;
    const int add_e = xa + (carry ? 1 : 0);
    // opposite signs: the difference, normalised (a tiny result stays denormal)
    const uint64_t dl = 0 - lo;
    const uint64_t dh = ma - hi - (lo != 0 ? 1 : 0);
    const bool cancel = dh == 0 && dl == 0;                  // exact cancellation: +0
    int lz = dh ? __builtin_clzll(dh) : 64 + __builtin_clzll(dl | 1);
    if (lz > xa - 1) lz = xa - 1;
    const uint64_t sub_h = lz >= 64 ? dl << ((lz - 64) & 63)
                         : (lz > 0 ? (dh << (lz & 63)) | (dl >> ((64 - lz) & 63)) : dh);
    const uint64_t sub_l = lz >= 64 ? 0 : (lz > 0 ? dl << (lz & 63) : dl);
    const int sub_e = xa - lz;
    const bool same = sa == sb;
    const uint64_t rh = same ? add_h : sub_h, rl = same ? add_l : sub_l;
    const int e = same ? add_e : sub_e;
    // round to nearest even; a carry out of the significand bumps the exponent
    const bool up = (rl >> 63) && ((rl << 1) || (rh & 1));
    const uint64_t r1 = rh + (up ? 1 : 0);
    const bool wrap = up && r1 == 0;
    const uint64_t r = wrap ? (1ull << 63) : r1;
    const int e2 = e + (wrap ? 1 : 0);
    const bool over = e2 >= 0x7fff;                          // overflow: infinity
    const uint64_t m = over ? (1ull << 63) : r;
    const uint32_t enc = over ? 0x7fffu : ((r >> 63) ? (uint32_t)e2 : 0u);
    *out = (!same && cancel) ? with_bits(a, 0, 0) : with_bits(a, m, (sa << 15) | enc);
    return true;
}

// a + b (the reference's `a[i] = a[i] + b[i]`); pads from a
XF_FN xf80 add(xf80 a, xf80 b)
{
    xf80 r;
    if (add_normal(a, b, &r)) return r;
    const uint32_t ea = a.se & 0x7fff, eb = b.se & 0x7fff;
    uint32_t sa = a.se >> 15, sb = b.se >> 15;
    const int ka = klass(a.m, ea), kb = klass(b.m, eb);
    if (ka == K_BAD || kb == K_BAD) return indefinite(a);
    if (ka >= K_QNAN || kb >= K_QNAN) return nan_result(a, ka, b, kb);
    if (ka == K_INF || kb == K_INF) {
        if (ka == K_INF && kb == K_INF && sa != sb) return indefinite(a);
        return ka == K_INF ? with_bits(a, a.m, a.se) : with_bits(a, b.m, b.se);
    }
    if (ka == K_ZERO && kb == K_ZERO) return with_bits(a, 0, (sa & sb) << 15);
    int xa = ea ? (int)ea : 1, xb = eb ? (int)eb : 1;
    uint64_t ma = a.m, mb = b.m;
    if (xb > xa || (xb == xa && mb > ma)) {          // |a| >= |b| from here
        const int t = xa; xa = xb; xb = t;
        const uint64_t tm = ma; ma = mb; mb = tm;
        const uint32_t ts = sa; sa = sb; sb = ts;
    }
    u128 A = (u128)ma << 64, B = (u128)mb << 64;
    const int d = xa - xb;
    if (d >= 128) {
        B = B != 0;
    } else if (d > 0) {
        const bool sticky = (B << (128 - d)) != 0;
        B = (B >> d) | (u128)sticky;
    }
    int e = xa;
    u128 S;
    if (sa == sb) {
        S = A + B;
        if (S < A) {                                  // carry out of bit 127
            S = (S >> 1) | (S & 1) | ((u128)1 << 127);
            ++e;
        }
    } else {
        S = A - B;
        if (S == 0) return with_bits(a, 0, 0);        // exact cancellation: +0
        int lz = clz128(S);
        if (lz > e - 1) lz = e - 1;
        S <<= lz;
        e -= lz;
    }
    return round_pack(a, sa, e, S);
}

// a * b (the reference's `a[i] = a[i] * b[i]`); pads from a
XF_FN xf80 mul(xf80 a, xf80 b)
{
    const uint32_t ea = a.se & 0x7fff, eb = b.se & 0x7fff;
    const uint32_t s = (a.se ^ b.se) >> 15;
    const int ka = klass(a.m, ea), kb = klass(b.m, eb);
    if (ka == K_BAD || kb == K_BAD) return indefinite(a);
    if (ka >= K_QNAN || kb >= K_QNAN) return nan_result(a, ka, b, kb);
    if (ka == K_INF || kb == K_INF) {
        if (ka == K_ZERO || kb == K_ZERO) return indefinite(a);
        return with_bits(a, 1ull << 63, (s << 15) | 0x7fff);
    }
    if (ka == K_ZERO || kb == K_ZERO) return with_bits(a, 0, s << 15);
    int xa = ea ? (int)ea : 1, xb = eb ? (int)eb : 1;
    uint64_t ma = a.m, mb = b.m;
    int la = __builtin_clzll(ma), lb = __builtin_clzll(mb);
    ma <<= la;
    mb <<= lb;
    xa -= la;
    xb -= lb;
    u128 P = (u128)ma * mb;                           // in [2^126, 2^128)
    int e = xa + xb - 16383 + 1;
    if (!(P >> 127)) {
        P <<= 1;
        --e;
    }
    if (e < 1) {                                      // denormalise, then one rounding
        const int sh = 1 - e;
        if (sh >= 128) {
            P = P != 0;
        } else {
            const bool sticky = (P << (128 - sh)) != 0;
            P = (P >> sh) | (u128)sticky;
        }
        e = 1;
    }
    return round_pack(a, s, e, P);
}

// An ordered operand as an unsigned 81-bit key (hi: 17 bits, lo: 64) that
// sorts as the x87 orders the values: the magnitude is (exponent, with
// denormals and pseudo-denormals at 1 and zero at 0; significand); a
// negative nonzero value takes the complement of its magnitude, every other
// value has bit 16 of hi set -- so -0 and +0 share one key, and equal keys
// are exactly the x87's equal values.  `u`: unordered (a NaN, or an invalid
// encoding: exponent 0x7fff except an infinity, or an unnormal).
struct xkey {
    uint32_t hi;
    uint64_t lo;
    bool u;
};

// The class tests are bools combined with & and | (never && / || / ?: on
// them): on the device each stays a lane mask and combines in scalar
// mask instructions, with no branch -- the short-circuit forms became
// exec-mask branches around every step of the MPI_MAX / MIN / MAXLOC /
// MINLOC trees, and integer 0 / 1 forms cost vector instructions
// (--save-temps of mvx_ops_{cmp,loc}.hip).
XF_FN xkey key(const xf80 &a)
{
    const uint32_t e = a.se & 0x7fff;
    const bool j = (a.m >> 63) != 0;
    const bool ez = e == 0, mz = a.m == 0;
    const uint32_t x = (ez & !mz) ? 1u : e;                     // 0 only for a zero
    const bool neg = ((a.se & 0x8000) != 0) & !(ez & mz);
    xkey k;
    k.hi = neg ? (~x & 0xffffu) : (x | 0x10000u);
    k.lo = neg ? ~a.m : a.m;
    k.u = (!j & !ez) | ((e == 0x7fff) & ((a.m << 1) != 0));
    return k;
}

// a against b: greater, equal, unordered (gt / eq meaningless when un)
struct xord {
    bool gt, eq, un;
};

XF_FN xord order(const xf80 &a, const xf80 &b)
{
    const xkey ka = key(a), kb = key(b);
    const bool heq = ka.hi == kb.hi;
    xord o;
    o.gt = (ka.hi > kb.hi) | (heq & (ka.lo > kb.lo));
    o.eq = heq & (ka.lo == kb.lo);
    o.un = ka.u | kb.u;
    return o;
}

// x87 compare: -1, 0, 1, or 2 = unordered (NaN or invalid encoding), as
// selects on the classes: unordered is every class from K_QNAN up (exponent
// 0x7fff except an infinity, or an unnormal); magnitudes order by (exponent,
// with denormals and pseudo-denormals at 1; significand), zero below all;
// one sign flip.  MPI_MAX / MIN use this form: its class tests run largely
// as scalar mask instructions, and the 8-leaf MAX tree measured 49.6-50.1 us
// with it against 51.5-51.7 us through order() (profiles/r03/
// bench_kernels_x87_ab.jsonl, bench_kernels_x87_pair_*.jsonl); the loc ops
// use order(), whose compare result the lane-pair kernel hands across lanes.
XF_FN int cmp(const xf80 &a, const xf80 &b)
{
    const uint32_t ea = a.se & 0x7fff, eb = b.se & 0x7fff;
    const bool ja = (a.m >> 63) != 0, jb = (b.m >> 63) != 0;
    const bool ua = ea == 0x7fff ? !(ja && (a.m << 1) == 0) : (ea != 0 && !ja);
    const bool ub = eb == 0x7fff ? !(jb && (b.m << 1) == 0) : (eb != 0 && !jb);
    const bool za = ea == 0 && a.m == 0, zb = eb == 0 && b.m == 0;
    const uint32_t xa = za ? 0u : (ea ? ea : 1u), xb = zb ? 0u : (eb ? eb : 1u);
    const bool gt = xa > xb || (xa == xb && a.m > b.m);
    const bool eq = xa == xb && a.m == b.m;
    const uint32_t sa = a.se >> 15, sb = b.se >> 15;
    const int c = eq ? 0 : (gt != (sa != 0) ? 1 : -1);      // magnitude order, sign applied
    const int r = (za && zb) ? 0 : (sa != sb ? (sa ? -1 : 1) : c);
    return (ua || ub) ? 2 : r;
}

XF_FN bool truth(const xf80 &a)                       // `a != 0`, unordered is true
{
    const int k = klass(a.m, a.se & 0x7fff);
    return k != K_ZERO;
}

XF_FN xf80 from_bool(xf80 pads, bool t)               // (long double)(int)t
{
    return t ? with_bits(pads, 1ull << 63, 0x3fff) : with_bits(pads, 0, 0);
}

// the reference's MPI_MAX / MPI_MIN select (coll.h:14-19): the chosen
// operand's 10 value bytes, the slot padding of a
XF_FN xf80 max(xf80 a, xf80 b) { return cmp(b, a) == 1 ? with_bits(a, b.m, b.se) : a; }
XF_FN xf80 min(xf80 a, xf80 b) { return cmp(a, b) == 1 ? with_bits(a, b.m, b.se) : a; }

XF_FN xf80 land(xf80 a, xf80 b) { return from_bool(a, truth(a) && truth(b)); }
XF_FN xf80 lor(xf80 a, xf80 b) { return from_bool(a, truth(a) || truth(b)); }
XF_FN xf80 lxor(xf80 a, xf80 b) { return from_bool(a, truth(a) != truth(b)); }

// MPI_LONG_DOUBLE_INT: struct { long double value; int loc; } (global_ops.c
// 1263-1268), 32 bytes; the padding after loc is an explicit member
struct pxi {
    xf80 v;
    int32_t l;
    int32_t pad[3];
};

// global_ops.c:1365-1378 (MAXLOC) and 1605-1618 (MINLOC): equal values keep
// the smaller loc; otherwise b replaces a only when strictly larger
// (smaller), value bytes and loc; unordered keeps a
template <bool MIN>
XF_FN pxi loc(pxi a, pxi b)
{
    const xord o = order(a.v, b.v);
    const bool take = !o.un & (MIN ? o.gt : !(o.gt | o.eq));
    const bool same = !o.un & o.eq;
    const int32_t lmin = a.l < b.l ? a.l : b.l;
    pxi r = a;
    r.v.m = take ? b.v.m : a.v.m;
    r.v.se = take ? b.v.se : a.v.se;
    r.l = same ? lmin : (take ? b.l : a.l);
    return r;
}

}  // namespace xf
