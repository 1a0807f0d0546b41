// sp_libm.h -- bit-exact emulation of the glibc float libm the reference calls.
//
// The reference computes std::sin/cos/exp/log/pow/erf/acos on floats, i.e. glibc's sinf, cosf,
// expf, logf, powf, erff and acosf.  None of them is correctly rounded (against a double
// evaluation: sinf/cosf differ on ~1.3% of inputs, logf 0.7%, erff 4.4%, acosf 7.7%), so the GPU
// must run glibc's own algorithms to reproduce the reference bit for bit:
//
//   expf, logf, powf, sinf, cosf : glibc 2.35 x86-64 FMA ifunc variants (ARM optimized-routines
//       algorithms built with -mfma: double-precision evaluation, FMAs exactly where GCC fused)
//   erff, acosf (__ieee754_acosf) : fdlibm single-precision code (no FMA; erff calls expf)
//
// Each function below follows the instruction sequence of the system libm.so.6 (see
// tools/extract_glibc_libm.py for the data and addresses) and is verified exhaustively against
// the host libm over all 2^32 inputs (powf: structured + random pairs) by
// tests/test_libm_exact.py.  The same source is compiled for the host and for gfx950 with
// explicit fma() and no contraction, so the host verification carries over to the device.
//
// Attribution: the algorithms, polynomial coefficients and tables restated here are those of
// the GNU C Library 2.35 (glibc, LGPL-2.1-or-later), whose expf/logf/powf/sinf/cosf come from
// Arm's optimized-routines (Copyright (c) 2017-2018 Arm Ltd., MIT / LGPL as distributed with
// glibc) and whose erff/acosf/atanf/atan2f are Sun Microsystems' fdlibm (Copyright (C) 1993 Sun
// Microsystems, Inc.: "Permission to use, copy, modify, and distribute this software is freely
// granted, provided that this notice is preserved").  The table values in sp_glibc_data.h are
// read from the system libm.so.6 by tools/extract_glibc_libm.py.
#pragma once
#include "sp_math.h"
#include "sp_glibc_data.h"

namespace spm {

SP_HD double dfma(double a, double b, double c) { return __builtin_fma(a, b, c); }
SP_HD double gd(const uint64_t* t, int i) { return u2d(t[i]); }

// The f64 constant with bits B, put in a VGPR pair next to its use.  A polynomial step
// dfma(r, K1, K2) needs one of its two constants in VGPRs (gfx9 VOP3: one SGPR pair, no f64
// literal), and left alone the compiler hoists that pair out of every loop: in the DirectLighting
// megakernel powf's two accumulator constants were held for the whole kernel and, at 128 VGPRs,
// reloaded from scratch in every sample of the 16-sample rho loop.  The moves take the
// polynomial's variable as a (never read) operand, so they cannot be hoisted above it; they are
// ordinary instructions otherwise (not volatile: free to schedule).  The value is the constant.
template <uint64_t B>
SP_HD double vk(double dep)
{
#if defined(__HIP_DEVICE_COMPILE__)
    uint32_t lo, hi;
    asm("v_mov_b32 %0, %1 ; %2" : "=v"(lo) : "i"((uint32_t)(B & 0xffffffffull)), "v"(dep));
    asm("v_mov_b32 %0, %1 ; %2" : "=v"(hi) : "i"((uint32_t)(B >> 32)), "v"(dep));
    return u2d(((uint64_t)hi << 32) | (uint64_t)lo);
#else
    (void)dep;
    return u2d(B);
#endif
}

// Tables read with a per-lane index.  In device code they are served from LDS copies (a
// 64-lane gather from a global table touches several cache lines per instruction and keeps the
// vector L1 busy); every kernel that can reach this libm calls libm_lds_init() first.
#if defined(__HIP_DEVICE_COMPILE__)
static __shared__ uint64_t lds_exp2f_t[32];
static __shared__ uint64_t lds_logf_t[32];
static __shared__ uint64_t lds_powf_t[32];
__device__ __forceinline__ void libm_lds_init(int tid, int nthreads)
{
    for (int i = tid; i < 32; i += nthreads) {
        lds_exp2f_t[i] = glibc::EXP2F_T[i];
        lds_logf_t[i]  = glibc::LOGF_T[i];
        lds_powf_t[i]  = glibc::POWF_T[i];
    }
}
#define SPM_EXP2F_T lds_exp2f_t
#define SPM_LOGF_T lds_logf_t
#define SPM_POWF_T lds_powf_t
#else
SP_HD void libm_lds_init(int, int) {} // host pass / host build: tables are read in place
#define SPM_EXP2F_T glibc::EXP2F_T
#define SPM_LOGF_T glibc::LOGF_T
#define SPM_POWF_T glibc::POWF_T
#endif
SP_HD float gf(const uint32_t* t, int i) { return u2f(t[i]); }

// x86 default NaN produced by invalid operations such as 0/0 (sign bit set).
SP_HD float x86_default_nan() { return u2f(0xffc00000u); }
// x86 NaN propagation for a unary op on a NaN input: the input, quieted.
SP_HD float x86_quiet(float x) { return u2f(f2u(x) | 0x00400000u); }
SP_HD bool  is_nan_bits(float x) { return (f2u(x) & 0x7fffffffu) > 0x7f800000u; }
// SSE addss/mulss with a NaN operand return the first NaN operand, quieted.
SP_HD float x86_add(float a, float b)
{
    if (is_nan_bits(a)) return x86_quiet(a);
    if (is_nan_bits(b)) return x86_quiet(b);
    return a + b;
}

// ------------------------------------------------------------------------------------ expf
SP_HD float lm_expf(float x)
{
#if defined(SP_XP_FASTLIBM) && defined(__HIP_DEVICE_COMPILE__) // timing-only bound (sp_path.hpp SP_XP_*)
    return __expf(x);
#endif
    using namespace glibc;
    const uint32_t ix     = f2u(x);
    const uint32_t abstop = (ix >> 20) & 0x7ffu;
    const double   xd     = (double)x;
    if (abstop > 0x42au) {
        if (ix == 0xff800000u) return 0.0f;
        if (abstop > 0x7f7u) return x86_add(x, x); // inf or nan
        if (x > gf(EXPF_LIM, 0)) return __builtin_inff(); // __math_oflowf(0)
        if (gf(EXPF_LIM, 1) > x) return 0.0f;             // __math_uflowf(0)
        if (!(gf(EXPF_LIM, 2) <= x)) return u2f(0x00000001u); // __math_may_uflowf(0): 0x1.4p-75f^2
    }
    const double invln2n = gd(EXPF_K, 1), shift = gd(EXPF_K, 0);
    double       kd      = dfma(invln2n, xd, shift);
    const uint64_t ki    = d2u(kd);
    kd -= shift;
    const double r = dfma(invln2n, xd, -kd);
    uint64_t     t = SPM_EXP2F_T[ki & 31u] + (ki << 47);
    const double s  = u2d(t);
    const double z  = dfma(r, gd(EXPF_K, 2), vk<EXPF_K[3]>(r));
    const double r2 = r * r;
    double       y  = dfma(r, gd(EXPF_K, 4), gd(ONE_D, 0));
    y               = dfma(z, r2, y);
    y               = y * s;
    return (float)y;
}

// ------------------------------------------------------------------------------------ logf
SP_HD float lm_logf(float x)
{
#if defined(SP_XP_FASTLIBM) && defined(__HIP_DEVICE_COMPILE__) // timing-only bound (sp_path.hpp SP_XP_*)
    return __logf(x);
#endif
    using namespace glibc;
    uint32_t ix = f2u(x);
    if (ix == 0x3f800000u) return 0.0f;
    if (ix - 0x00800000u > 0x7effffffu) {
        if (ix * 2u == 0u) return -__builtin_inff();                 // __math_divzerof(1)
        if (ix == 0x7f800000u) return x;
        if (ix * 2u > 0xfeffffffu) return x86_quiet(x);              // NaN: (x-x)/(x-x)
        if (ix & 0x80000000u) return x86_default_nan();              // x < 0
        ix = f2u(x * gf(TWO23_F, 0)) - (23u << 23);                  // subnormal
    }
    const uint32_t tmp  = ix - 0x3f330000u;
    const uint32_t i    = (tmp >> 19) & 15u;
    const int32_t  k    = (int32_t)tmp >> 23;
    const uint32_t iz   = ix - (tmp & 0xff800000u);
    const double   invc = gd(SPM_LOGF_T, 2 * i), logc = gd(SPM_LOGF_T, 2 * i + 1);
    const double   z    = (double)u2f(iz);
    const double   r    = dfma(z, invc, gd(MINUS_ONE_D, 0));
    const double   y0   = dfma((double)k, gd(LOGF_K, 0), logc);
    const double   r2   = r * r;
    double         y    = dfma(r, gd(LOGF_K, 2), vk<LOGF_K[3]>(r));
    y                   = dfma(r2, gd(LOGF_K, 1), y);
    y                   = dfma(r2, y, r + y0);
    return (float)y;
}

// ------------------------------------------------------------------------------------ powf
SP_HD int powf_checkint(uint32_t iy)
{
    const int e = (int)((iy >> 23) & 0xffu);
    if (e < 0x7f) return 0;
    if (e > 0x7f + 23) return 2;
    if (iy & ((1u << (0x7f + 23 - e)) - 1u)) return 0;
    if (iy & (1u << (0x7f + 23 - e))) return 1;
    return 2;
}
SP_HD bool powf_zeroinfnan(uint32_t ix) { return 2u * ix - 1u >= 2u * 0x7f800000u - 1u; }
SP_HD bool issignalingf(uint32_t ix) { return ((ix & 0x7fffffffu) > 0x7f800000u) && !(ix & 0x00400000u); }

SP_HD float lm_powf(float x, float y)
{
#if defined(SP_XP_FASTLIBM) && defined(__HIP_DEVICE_COMPILE__) // timing-only bound (sp_path.hpp SP_XP_*)
    return __powf(x, y);
#endif
    using namespace glibc;
    uint32_t       sign_bias = 0;
    uint32_t       ix = f2u(x);
    const uint32_t iy = f2u(y);
    if (ix - 0x00800000u >= 0x7f000000u || powf_zeroinfnan(iy)) {
        if (powf_zeroinfnan(iy)) {
            if (2u * iy == 0u) return issignalingf(ix) ? x86_add(x, y) : 1.0f;
            if (ix == 0x3f800000u) return issignalingf(iy) ? x86_add(x, y) : 1.0f;
            if (2u * ix > 2u * 0x7f800000u || 2u * iy > 2u * 0x7f800000u) return x86_add(x, y);
            if (2u * ix == 2u * 0x3f800000u) return 1.0f;
            if ((2u * ix < 2u * 0x3f800000u) == !(iy & 0x80000000u)) return 0.0f;
            return y * y;
        }
        if (powf_zeroinfnan(ix)) {
            float x2 = x * x;
            if ((ix & 0x80000000u) && powf_checkint(iy) == 1) x2 = -x2;
            return (iy & 0x80000000u) ? 1.0f / x2 : x2;
        }
        if (ix & 0x80000000u) {
            const int yint = powf_checkint(iy);
            if (yint == 0) return x86_default_nan(); // __math_invalidf(x): (x-x)/(x-x)
            if (yint == 1) sign_bias = 1u << 16;
            ix &= 0x7fffffffu;
        }
        if (ix < 0x00800000u) {
            ix = f2u(x * gf(TWO23_F, 0)) & 0x7fffffffu;
            ix -= 23u << 23;
        }
    }
    // log2_inline
    const uint32_t tmp  = ix - 0x3f330000u;
    const uint32_t i    = (tmp >> 19) & 15u;
    const uint32_t top  = tmp & 0xff800000u;
    const uint32_t iz   = ix - top;
    const int32_t  k    = (int32_t)top >> 23;
    const double   invc = gd(SPM_POWF_T, 2 * i), logc = gd(SPM_POWF_T, 2 * i + 1);
    const double   z    = (double)u2f(iz);
    const double   r    = dfma(z, invc, gd(MINUS_ONE_D, 0));
    const double   y0   = (double)k + logc;
    const double   r2   = r * r;
    double         yy   = dfma(r, gd(POWF_A, 0), vk<POWF_A[1]>(r));
    const double   p    = dfma(r, gd(POWF_A, 2), vk<POWF_A[3]>(r));
    const double   r4   = r2 * r2;
    double         q    = dfma(r, gd(POWF_A, 4), y0);
    q                   = dfma(r2, p, q);
    yy                  = dfma(yy, r4, q);
    const double ylogx  = (double)y * yy;
    if (((d2u(ylogx) >> 47) & 0xffffu) > 0x80beu) {
        if (ylogx > gd(POWF_LIM, 0)) return sign_bias ? -__builtin_inff() : __builtin_inff(); // __math_oflowf
        if (ylogx > gd(POWF_LIM, 1)) {
            // may overflow: glibc checks the rounding direction; round-to-nearest keeps the value
            const float one = gf(POWF_FLIM, 1) < 0.0f ? 1.0f : 1.0f;
            (void)one;
        }
        if (!(gd(POWF_LIM, 2) < ylogx)) return sign_bias ? -0.0f : 0.0f;               // __math_uflowf
        if (!(gd(POWF_LIM, 3) <= ylogx)) return u2f(sign_bias ? 0x80000001u : 0x00000001u); // may_uflow
    }
    // exp2_inline(ylogx, sign_bias)
    const double   shift = gd(EXP2F_K, 0);
    double         kd    = ylogx + shift;
    const uint64_t ki    = d2u(kd);
    kd -= shift;
    const double   rr  = ylogx - kd;
    uint64_t       t   = SPM_EXP2F_T[ki & 31u];
    const uint64_t ski = ki + sign_bias;
    t += ski << 47;
    const double s   = u2d(t);
    const double zz  = dfma(rr, gd(EXP2F_K, 1), vk<EXP2F_K[2]>(rr));
    const double rr2 = rr * rr;
    double       res = dfma(rr, gd(EXP2F_K, 3), gd(ONE_D, 0));
    res              = dfma(zz, rr2, res);
    res              = res * s;
    return (float)res;
}

// ------------------------------------------------------------------------------------ sinf / cosf
// __sincosf_table[2] layout (14 doubles each): sign[4], hpi_inv, hpi, c0, c1, s1, c2, s2, c3, s3, c4.
// Table 1 is table 0 with the cosine coefficients c0..c4 negated (sign, hpi and s1..s3 equal), so
// no table is read at run time: table-0 constants fold into the code, a table-1 cosine polynomial
// is the exact negation of the table-0 one (every intermediate flips sign), and sign[n & 3] is
// {1, -1, -1, 1}.  Indexing a table by the lane's quadrant made the compiler hoist the constant-
// index entries into 20 VGPRs for the whole kernel.
SP_HD double sc(int k) { return gd(glibc::SINCOSF_T, k); }
enum { SC_HPI_INV = 4, SC_HPI = 5, SC_C0 = 6, SC_C1 = 7, SC_S1 = 8, SC_C2 = 9, SC_S2 = 10, SC_C3 = 11, SC_S3 = 12, SC_C4 = 13 };
SP_HD double sincos_sign(int q) { return (q == 1 || q == 2) ? -1.0 : 1.0; } // sign[q], q = n & 3

SP_HD float sincosf_poly(double x, double x2, int tab, int n)
{
    if ((n & 1) == 0) {
        const double s1 = dfma(x2, sc(SC_S3), vk<glibc::SINCOSF_T[SC_S2]>(x2));
        const double x3 = x2 * x;
        const double x7 = x2 * x3;
        const double s  = dfma(x3, sc(SC_S1), x);
        return (float)dfma(s1, x7, s);
    }
    const double x4 = x2 * x2;
    const double c1 = dfma(x2, sc(SC_C1), vk<glibc::SINCOSF_T[SC_C0]>(x2));
    const double c2 = dfma(x2, sc(SC_C4), vk<glibc::SINCOSF_T[SC_C3]>(x2));
    const double x6 = x2 * x4;
    const double c  = dfma(x4, sc(SC_C2), c1);
    const float  r  = (float)dfma(c2, x6, c);
    return tab ? -r : r;
}

SP_HD double sincosf_reduce_large(uint32_t xi, int* np)
{
    const uint32_t* arr   = glibc::INV_PIO4 + ((xi >> 26) & 15u);
    const int       shift = (int)((xi >> 23) & 7u);
    xi                    = (xi & 0xffffffu) | 0x800000u;
    xi <<= shift;
    uint64_t res0 = (uint64_t)(uint32_t)(xi * arr[0]);
    uint64_t res1 = (uint64_t)xi * arr[4];
    uint64_t res2 = (uint64_t)xi * arr[8];
    res0          = (res2 >> 32) | (res0 << 32);
    res0 += res1;
    const uint64_t n = (res0 + (1ull << 61)) >> 62;
    res0 -= n << 62;
    const double x = (double)(int64_t)res0;
    *np            = (int)n;
    return x * u2d(glibc::PI63[0]);
}

// BOUNDED: the caller guarantees a finite |y| < 120 (abstop <= 0x42e), e.g. 2*pi*u for a canonical
// u in [0, 1).  Such inputs take one of the first two paths of the full function, so leaving the
// large-argument reduction (and its registers) out of the code changes no result.
template <bool BOUNDED = false>
SP_HD float lm_sinf(float y)
{
#if defined(SP_XP_FASTLIBM) && defined(__HIP_DEVICE_COMPILE__) // timing-only bound (sp_path.hpp SP_XP_*)
    return __sinf(y);
#endif
    const uint32_t iy     = f2u(y);
    const uint32_t abstop = (iy >> 20) & 0x7ffu;
    double         x      = (double)y;
    if (abstop <= 0x3f3u) {
        const double s = x * x;
        if (abstop <= 0x397u) return y;
        return sincosf_poly(x, s, 0, 0);
    }
    if (BOUNDED || abstop <= 0x42eu) {
        const double r  = x * sc(SC_HPI_INV);
        int          n  = (((int32_t)r) + 0x800000) >> 24;
        x               = dfma(-(double)n, sc(SC_HPI), x);
        const double sg = sincos_sign(n & 3);
        const int    tb = (n & 2) ? 1 : 0;
        return sincosf_poly(x * sg, x * x, tb, n);
    }
    if (abstop <= 0x7f7u) {
        const int sign = (int)(iy >> 31);
        int       n;
        x               = sincosf_reduce_large(iy, &n);
        const double sg = sincos_sign((n + sign) & 3);
        const int    tb = ((n + sign) & 2) ? 1 : 0;
        return sincosf_poly(x * sg, x * x, tb, n);
    }
    // __math_invalidf(y): (y - y) / (y - y)
    return ((iy & 0x7fffffffu) > 0x7f800000u) ? x86_quiet(y) : x86_default_nan();
}

template <bool BOUNDED = false> // as lm_sinf
SP_HD float lm_cosf(float y)
{
#if defined(SP_XP_FASTLIBM) && defined(__HIP_DEVICE_COMPILE__) // timing-only bound (sp_path.hpp SP_XP_*)
    return __cosf(y);
#endif
    const uint32_t iy     = f2u(y);
    const uint32_t abstop = (iy >> 20) & 0x7ffu;
    double         x      = (double)y;
    if (abstop <= 0x3f3u) {
        const double s = x * x;
        if (abstop <= 0x397u) return 1.0f;
        return sincosf_poly(x, s, 0, 1);
    }
    if (BOUNDED || abstop <= 0x42eu) {
        const double r  = x * sc(SC_HPI_INV);
        int          n  = (((int32_t)r) + 0x800000) >> 24;
        x               = dfma(-(double)n, sc(SC_HPI), x);
        const double sg = sincos_sign(n & 3);
        const int    tb = (n & 2) ? 1 : 0;
        return sincosf_poly(x * sg, x * x, tb, n ^ 1);
    }
    if (abstop <= 0x7f7u) {
        const int sign = (int)(iy >> 31);
        int       n;
        x               = sincosf_reduce_large(iy, &n);
        const double sg = sincos_sign((n + sign) & 3);
        const int    tb = ((n + sign) & 2) ? 1 : 0;
        return sincosf_poly(x * sg, x * x, tb, n ^ 1);
    }
    return ((iy & 0x7fffffffu) > 0x7f800000u) ? x86_quiet(y) : x86_default_nan();
}

// sinf(y) and cosf(y) of one BOUNDED argument (|y| < 120, finite), each bit-identical to the calls
// above: both take the same reduction and the same two polynomials, so one reduction and one of
// each polynomial serve both -- where the separate calls each evaluate both polynomials whenever
// the wave's lanes hold both quadrant parities.
SP_HD void lm_sincosf_bounded(float y, float* s_out, float* c_out)
{
#if defined(SP_XP_FASTLIBM) && defined(__HIP_DEVICE_COMPILE__) // timing-only bound (sp_path.hpp SP_XP_*)
    *s_out = __sinf(y); *c_out = __cosf(y); return;
#endif
    const uint32_t iy     = f2u(y);
    const uint32_t abstop = (iy >> 20) & 0x7ffu;
    double         x      = (double)y;
    int            n      = 0;
    int            tb     = 0;
    if (abstop > 0x3f3u) {
        const double r  = x * sc(SC_HPI_INV);
        n               = (((int32_t)r) + 0x800000) >> 24;
        x               = dfma(-(double)n, sc(SC_HPI), x);
        x               = x * sincos_sign(n & 3); // x2 below is the square of the signed x: exact
        tb              = (n & 2) ? 1 : 0;
    }
    const double x2 = x * x;
    const double s1 = dfma(x2, sc(SC_S3), vk<glibc::SINCOSF_T[SC_S2]>(x2));
    const double x3 = x2 * x;
    const double x7 = x2 * x3;
    const float  ps = (float)dfma(s1, x7, dfma(x3, sc(SC_S1), x));
    const double x4 = x2 * x2;
    const double c1 = dfma(x2, sc(SC_C1), vk<glibc::SINCOSF_T[SC_C0]>(x2));
    const double c2 = dfma(x2, sc(SC_C4), vk<glibc::SINCOSF_T[SC_C3]>(x2));
    const double x6 = x2 * x4;
    const float  pr = (float)dfma(c2, x6, dfma(x4, sc(SC_C2), c1));
    const float  pc = tb ? -pr : pr;
    const bool   odd = (n & 1) != 0;
    *s_out = odd ? pc : ps;
    *c_out = odd ? ps : pc;
    if (abstop <= 0x397u) { *s_out = y; *c_out = 1.0f; }
}

// sinf(y) and cosf(y) of any argument: the fused form where it applies, the two calls elsewhere
SP_HD void lm_sincosf(float y, float* s_out, float* c_out)
{
    if (((f2u(y) >> 20) & 0x7ffu) <= 0x42eu) { lm_sincosf_bounded(y, s_out, c_out); return; }
    *s_out = lm_sinf(y);
    *c_out = lm_cosf(y);
}

// ------------------------------------------------------------------------------------ erff
SP_HD float lm_erff(float x)
{
    using namespace glibc;
    const uint32_t hx = f2u(x);
    const uint32_t ix = hx & 0x7fffffffu;
    const float    one = gf(ERFF_MISC, 8);
    if (ix > 0x7f7fffffu) {
        if (is_nan_bits(x)) return x86_quiet(x);
        const int i = (int)((hx >> 31) << 1);
        return (float)(1 - i) + one / x;
    }
    if (ix <= 0x3f57ffffu) {       // |x| < 0.84375
        if (ix <= 0x317fffffu) {   // |x| < 2^-28
            if ((hx & 0x7c000000u) == 0u) {
                const float a = x * gf(ERFF_SMALL, 0);
                const float b = x * gf(ERFF_MISC, 0);
                return (b + a) * gf(ERFF_MISC, 2);
            }
            return x * gf(ERFF_SMALL, 1) + x;
        }
        const float z = x * x;
        float       q = gf(ERFF_SMALL, 6);
        float       p = gf(ERFF_SMALL, 2);
        q             = q * z + gf(ERFF_SMALL, 7);
        p             = p * z - gf(ERFF_SMALL, 3);
        q             = q * z + gf(ERFF_SMALL, 8);
        p             = p * z - gf(ERFF_SMALL, 4);
        q             = q * z + gf(ERFF_SMALL, 9);
        p             = p * z - gf(ERFF_SMALL, 5);
        q             = q * z + gf(ERFF_ERX, 0);
        p             = p * z + gf(ERFF_SMALL, 1);
        q             = q * z + one;
        const float y = p / q;
        return y * x + x;
    }
    if (ix <= 0x3f9fffffu) {       // 0.84375 <= |x| < 1.25
        const float s = __builtin_fabsf(x) - one;
        float       q = gf(ERFF_ERX, 8);
        float       p = gf(ERFF_ERX, 1);
        q             = q * s + gf(ERFF_ERX, 9);
        p             = p * s + gf(ERFF_ERX, 2);
        q             = q * s + gf(ERFF_ERX, 10);
        p             = p * s - gf(ERFF_ERX, 3);
        q             = q * s + gf(ERFF_ERX, 11);
        p             = p * s + gf(ERFF_ERX, 4);
        q             = q * s + gf(ERFF_ERX, 12);
        p             = p * s - gf(ERFF_ERX, 5);
        q             = q * s + gf(ERFF_ERX, 13);
        p             = p * s + gf(ERFF_ERX, 6);
        q             = q * s;
        p             = p * s - gf(ERFF_ERX, 7);
        q             = q + one;
        const float pq = p / q;
        if ((int32_t)hx < 0) return gf(ERFF_MISC, 5) - pq;
        return pq + gf(ERFF_MISC, 4);
    }
    if (ix > 0x40bfffffu) {        // |x| >= 6
        if ((int32_t)hx < 0) return gf(ERFF_MISC, 7) - one;
        return one - gf(ERFF_MISC, 7);
    }
    const float ax = __builtin_fabsf(x);
    const float s  = one / (x * x);
    float       R, S;
    if (ix <= 0x4036db6du) {       // |x| < 1/0.35
        float a = s * gf(ERFF_MID, 0) - gf(ERFF_MID, 1);
        float b = gf(ERFF_MID, 8);
        b       = b * s + gf(ERFF_MID, 9);
        a       = a * s - gf(ERFF_MID, 2);
        b       = b * s + gf(ERFF_MID, 10);
        a       = a * s - gf(ERFF_MID, 3);
        b       = b * s + gf(ERFF_MID, 11);
        a       = a * s - gf(ERFF_MID, 4);
        b       = b * s + gf(ERFF_MID, 12);
        a       = a * s - gf(ERFF_MID, 5);
        b       = b * s + gf(ERFF_MID, 13);
        a       = a * s - gf(ERFF_MID, 6);
        b       = b * s + gf(ERFF_MID, 14);
        a       = a * s - gf(ERFF_MID, 7);
        b       = b * s + gf(ERFF_MID, 15);
        b       = b * s + one;
        R       = a;
        S       = b;
    } else {
        float a = s * gf(ERFF_BIG, 0) - gf(ERFF_BIG, 1);
        float b = gf(ERFF_BIG, 7);
        b       = b * s + gf(ERFF_BIG, 8);
        a       = a * s - gf(ERFF_BIG, 2);
        b       = b * s + gf(ERFF_BIG, 9);
        a       = a * s - gf(ERFF_BIG, 3);
        b       = b * s + gf(ERFF_BIG, 10);
        a       = a * s - gf(ERFF_BIG, 4);
        b       = b * s + gf(ERFF_BIG, 11);
        a       = a * s - gf(ERFF_BIG, 5);
        b       = b * s + gf(ERFF_BIG, 12);
        a       = a * s - gf(ERFF_BIG, 6);
        b       = b * s + gf(ERFF_BIG, 13);
        b       = b * s + one;
        R       = a;
        S       = b;
    }
    const float z  = u2f(f2u(ax) & 0xfffff000u);
    const float e1 = lm_expf(-z * z - gf(ERFF_MISC, 6));
    const float rs = R / S;
    const float e2 = lm_expf((z - ax) * (z + ax) + rs);
    const float r  = e2 * e1;
    if ((int32_t)hx < 0) return r / ax - one;
    return one - r / ax;
}

// ------------------------------------------------------------------------------------ acosf
SP_HD float lm_acosf(float x)
{
    using namespace glibc;
    const uint32_t hx  = f2u(x);
    const uint32_t ix  = hx & 0x7fffffffu;
    const float    one = 1.0f;
    if (ix == 0x3f800000u) {
        if ((int32_t)hx > 0) return 0.0f;
        return gf(ACOSF_K, 1) + gf(ACOSF_K, 0);
    }
    if (ix > 0x3f800000u) {
        if (ix > 0x7f800000u) return x86_quiet(x); // NaN input
        return u2f(0x7fc00000u);                     // acosf wrapper: __kernel_standard_f -> NAN
    }
    if (ix <= 0x3effffffu) {       // |x| < 0.5
        if (ix <= 0x32800000u) return gf(ACOSF_K, 3) + gf(ACOSF_K, 2);
        const float z = x * x;
        float       p = gf(ACOSF_K, 4) * z + gf(ACOSF_K, 5);
        float       q = gf(ACOSF_K, 10) * z - gf(ACOSF_K, 11);
        p             = p * z - gf(ACOSF_K, 6);
        q             = q * z + gf(ACOSF_K, 12);
        p             = p * z + gf(ACOSF_K, 7);
        q             = q * z - gf(ACOSF_K, 13);
        p             = p * z - gf(ACOSF_K, 8);
        q             = q * z + one;
        p             = p * z + gf(ACOSF_K, 9);
        p             = p * z;
        const float r  = p / q;
        const float xr = r * x;
        const float t  = gf(ACOSF_K, 3) - xr;
        const float u  = x - t;
        return gf(ACOSF_K, 2) - u;
    }
    if ((int32_t)hx < 0) {         // x < -0.5
        const float z = (x + one) * 0.5f;
        float       p = gf(ACOSF_K, 4) * z;
        float       q = gf(ACOSF_K, 10) * z;
        const float s = __builtin_sqrtf(z);
        p             = p + gf(ACOSF_K, 5);
        q             = q - gf(ACOSF_K, 11);
        p             = p * z - gf(ACOSF_K, 6);
        q             = q * z + gf(ACOSF_K, 12);
        p             = p * z + gf(ACOSF_K, 7);
        q             = q * z - gf(ACOSF_K, 13);
        p             = p * z - gf(ACOSF_K, 8);
        q             = q * z;
        p             = p * z + gf(ACOSF_K, 9);
        q             = q + one;
        p             = p * z;
        const float r = p / q;
        float       w = r * s - gf(ACOSF_K, 3);
        w             = w + s;
        return gf(ACOSF_K, 0) - (w + w);
    }
    // x > 0.5
    const float z  = (one - x) * 0.5f;
    float       p  = gf(ACOSF_K, 4) * z;
    float       q  = gf(ACOSF_K, 10) * z;
    const float s  = __builtin_sqrtf(z);
    p              = p + gf(ACOSF_K, 5);
    q              = q - gf(ACOSF_K, 11);
    p              = p * z - gf(ACOSF_K, 6);
    q              = q * z + gf(ACOSF_K, 12);
    p              = p * z + gf(ACOSF_K, 7);
    q              = q * z - gf(ACOSF_K, 13);
    p              = p * z - gf(ACOSF_K, 8);
    q              = q * z;
    p              = p * z + gf(ACOSF_K, 9);
    q              = q + one;
    p              = p * z;
    const float r  = p / q;
    const float df = u2f(f2u(s) & 0xfffff000u);
    const float c  = (z - df * df) / (s + df);
    float       w  = r * s + c;
    w              = w + df;
    return w + w;
}

// ------------------------------------------------------------------------------------ atanf
// fdlibm s_atanf.c as built into glibc 2.35 x86-64 libm.so.6 (atanf @0x3e080, no FMA): the
// branch limits and the order of every float operation follow that disassembly.  Constants are
// the words it loads (atanhi/atanlo @0x9ebd0.., aT @0x9ec0c..).
SP_HD float lm_atanf(float x)
{
    const uint32_t hx = f2u(x);
    const uint32_t ix = hx & 0x7fffffffu;
    const float    one = 1.0f;
    if (ix > 0x4bffffffu) {                              // |x| >= 2^25, inf, NaN
        if (ix > 0x7f800000u) return x86_quiet(x);       // x + x
        if ((int32_t)hx > 0) return u2f(0x3fc90fdau) + u2f(0x33a22168u);
        return u2f(0xbfc90fdau) - u2f(0x33a22168u);
    }
    int   id;
    float hi = 0.0f, lo = 0.0f;
    if (ix <= 0x3edfffffu) {                             // |x| < 0.4375
        if (ix <= 0x30ffffffu) return x;                 // |x| < 2^-29 (huge + x > one)
        id = -1;
    } else {
        const float ax = abs_f(x);
        if (ix > 0x3f97ffffu) {
            if (ix > 0x401bffffu) {                      // 2.4375 <= |x| < 2^25
                id = 3; hi = u2f(0x3fc90fdau); lo = u2f(0x33a22168u);
                x  = -1.0f / ax;
            } else {                                     // 1.1875 <= |x| < 2.4375
                id = 2; hi = u2f(0x3f7b985eu); lo = u2f(0x33140fb4u);
                x  = (ax - 1.5f) / (ax * 1.5f + one);
            }
        } else if (ix > 0x3f2fffffu) {                   // 11/16 <= |x| < 19/16
            id = 1; hi = u2f(0x3f490fdau); lo = u2f(0x33222168u);
            x  = (ax - one) / (ax + one);
        } else {                                         // 7/16 <= |x| < 11/16
            id = 0; hi = u2f(0x3eed6338u); lo = u2f(0x31ac3769u);
            x  = ((ax + ax) - one) / (ax + 2.0f);
        }
    }
    const float z  = x * x;
    const float w  = z * z;
    float       s1 = u2f(0x3c8569d7u) * w + u2f(0x3d4bda59u);
    s1             = s1 * w + u2f(0x3d886b35u);
    s1             = s1 * w + u2f(0x3dba2e6eu);
    s1             = s1 * w + u2f(0x3e124925u);
    s1             = s1 * w + u2f(0x3eaaaaabu);
    s1             = s1 * z;
    float s2       = u2f(0xbd15a221u) * w - u2f(0x3d6ef16bu);
    s2             = s2 * w - u2f(0x3d9d8795u);
    s2             = s2 * w - u2f(0x3de38e38u);
    s2             = s2 * w - u2f(0x3e4ccccdu);
    s2             = s2 * w;
    const float sx = (s1 + s2) * x;
    if (id < 0) return x - sx;
    const float r = hi - ((sx - lo) - x);
    return ((int32_t)hx < 0) ? -r : r;
}

// ------------------------------------------------------------------------------------ atan2f
// fdlibm e_atan2f.c (__atan2f_finite @0x38be0 in the same libm; the atan2f wrapper only sets
// errno).  y first, x second, like std::atan2.
SP_HD float lm_atan2f(float y, float x)
{
    const uint32_t hx = f2u(x), hy = f2u(y);
    const uint32_t ix = hx & 0x7fffffffu, iy = hy & 0x7fffffffu;
    const float    tiny   = u2f(0x0da24260u);
    const float    pi     = u2f(0x40490fdbu);
    const float    pi_o_2 = u2f(0x3fc90fdbu);
    const float    pi_o_4 = u2f(0x3f490fdbu);
    if (ix > 0x7f800000u || iy > 0x7f800000u) return is_nan_bits(x) ? x86_quiet(x) : x86_quiet(y); // x + y
    if (hx == 0x3f800000u) return lm_atanf(y);
    const int m = (int)(((int32_t)hx >> 30) & 2) | (int)(hy >> 31);
    if (iy == 0) {
        if (m == 2) return tiny + pi;
        if (m == 3) return u2f(0xc0490fdbu) - tiny;
        return y;
    }
    if (ix == 0) return ((int32_t)hy < 0) ? u2f(0xbfc90fdbu) - tiny : tiny + pi_o_2;
    if (ix == 0x7f800000u) {
        if (iy == 0x7f800000u) {
            if (m == 2) return 3.0f * pi_o_4 + tiny;
            if (m == 3) return -3.0f * pi_o_4 - tiny;
            if (m == 1) return u2f(0xbf490fdbu) - tiny;
            return tiny + pi_o_4;
        }
        if (m == 2) return tiny + pi;
        if (m == 3) return u2f(0xc0490fdbu) - tiny;
        return (m == 1) ? -0.0f : 0.0f;
    }
    if (iy == 0x7f800000u) return ((int32_t)hy < 0) ? u2f(0xbfc90fdbu) - tiny : tiny + pi_o_2;
    const int32_t d = (int32_t)iy - (int32_t)ix;
    float         z;
    if (d > 0x1e7fffff) z = pi_o_2 - u2f(0x333bbd2eu);                  // |y/x| > 2^60
    else if ((int32_t)hx < 0 && (d >> 23) < -60) z = 0.0f;               // |y|/x < -2^60
    else z = lm_atanf(abs_f(y / x));
    if (m == 0) return z;
    if (m == 1) return u2f(f2u(z) ^ 0x80000000u);
    if (m == 2) return pi - (u2f(0x33bbbd2eu) + z);
    return (z + u2f(0x33bbbd2eu)) - pi;
}

// std::fmod(f, 1.0f) (glibc fmodf: exact).  For |f| < 2^23 the fraction f - trunc(f) is exact;
// the result carries the sign of f; inf/NaN give NaN.
SP_HD float fmod1(float f)
{
    const float a = abs_f(f);
    if (a < 8388608.0f) return copysign_f(f - __builtin_truncf(f), f);
    if (is_nan_bits(f)) return x86_quiet(f);
    if (!(a <= 3.40282347e38f)) return x86_default_nan();
    return copysign_f(0.0f, f);
}
// std::round(float): half away from zero (glibc roundf).
SP_HD float round_f(float f) { return __builtin_roundf(f); }

} // namespace spm
