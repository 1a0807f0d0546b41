// sp_math.h -- float arithmetic with the exact rounding behaviour of the reference.
//
// The reference (kjeffery/SimplePath) computes with SSE/AVX2 intrinsics.  To reproduce its
// per-pixel results bit for bit on gfx950 every operation here is spelled out in the same order,
// with an explicit fused multiply-add exactly where the reference issues one
// (math/Math.h:138 madd -> std::fma; math/Vector3.h:402-426 _mm_fmadd_ps/_mm_fmsub_ps/...),
// and plain IEEE binary32 add/mul/div/sqrt everywhere else.  Kernels are built with
// -ffp-contract=off so the compiler adds no FMAs of its own.
//
//   dot        math/Vector3.h:743  _mm_dp_ps(a, b, 0x7F) == (x*x' + y*y') + (z*z' + 0)
//   cross      math/Vector3.h:769  difference_of_products on shuffled lanes (FMA based)
//   normalize  math/Vector3.h:797  a * rsqrt(dot(a, a)), rsqrt = RSQRTSS + one Newton step
//              (math/Math.h:205-226).  RSQRTSS is an x86 table approximation; on the device it
//              is emulated from a table captured from the host CPU's RSQRTSS (sp_rsqrt.cpp).
//   std::max / std::min / std::clamp keep libstdc++'s argument order (NaN behaviour matters).
#pragma once

#include <stdint.h>
#include <math.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define SP_HD __host__ __device__ __forceinline__
#define SP_DEV __device__ __forceinline__
#else
#define SP_HD static inline
#define SP_DEV static inline
#endif

#if !defined(__HIP_DEVICE_COMPILE__)
#include <immintrin.h>
#endif

namespace spm {

// ---------------------------------------------------------------- bit casts
SP_HD uint32_t f2u(float f) { return __builtin_bit_cast(uint32_t, f); }
SP_HD float u2f(uint32_t u) { return __builtin_bit_cast(float, u); }
SP_HD uint64_t d2u(double d) { return __builtin_bit_cast(uint64_t, d); }
SP_HD double u2d(uint64_t u) { return __builtin_bit_cast(double, u); }

// ---------------------------------------------------------------- libstdc++ ordering helpers
SP_HD float std_max(float a, float b) { return (a < b) ? b : a; }            // std::max
SP_HD float std_min(float a, float b) { return (b < a) ? b : a; }            // std::min
SP_HD float std_clamp(float v, float lo, float hi) { return (v < lo) ? lo : ((hi < v) ? hi : v); }
SP_HD float sse_min(float a, float b) { return (a < b) ? a : b; }            // _mm_min_ps
SP_HD float sse_max(float a, float b) { return (a > b) ? a : b; }            // _mm_max_ps
SP_HD float fma_f(float a, float b, float c) { return __builtin_fmaf(a, b, c); }
SP_HD float abs_f(float a) { return __builtin_fabsf(a); }
SP_HD float sqrt_f(float a) { return __builtin_sqrtf(a); }
SP_HD float copysign_f(float a, float b) { return __builtin_copysignf(a, b); }

constexpr float k_pi          = 3.14159265358979323846f;   // std::numbers::pi_v<float>
constexpr float k_inv_pi      = 0.318309886183790671538f;  // std::numbers::inv_pi_v<float>
constexpr float k_ray_epsilon = 0.001f;                    // math/Ray.h:163
constexpr float k_infinite    = 3.40282346638528859812e+38f; // base/Constants.h:257 (FLT_MAX)

// ---------------------------------------------------------------- RSQRTSS emulation
// Table: for parity p (exponent - 127 mod 2) and the top `bits` mantissa bits, the RSQRTSS
// result bits for an input with biased exponent 127 + p.  Result exponent is shifted by
// -(exponent - 127 - p) / 2.  Built and verified against the host instruction in sp_rsqrt.cpp.
struct RsqrtTable {
    const uint32_t* entries; // 2 << bits
    int32_t         bits;
    uint32_t        zero_result;   // RSQRTSS(+0)
    uint32_t        denorm_result; // RSQRTSS(smallest positive denormal) -- class behaviour
    // Packed form (device copies): pack_shift > 0 means `entries` holds 16-bit values v and the
    // result bits are pack_hi | v << pack_shift (every captured table so far: one exponent, 12
    // significant mantissa bits -- half the LDS of 32-bit entries).
    int32_t  pack_shift = 0;
    uint32_t pack_hi    = 0;
};

SP_HD float rsqrtss_emulated(float x, const RsqrtTable& t)
{
    const uint32_t u = f2u(x);
    const uint32_t e = (u >> 23) & 0xffu;
    if ((u >> 31) != 0u) {
        if ((u & 0x7fffffffu) == 0u) return u2f(0xff800000u); // -0 -> -inf
        if (e == 0xffu && (u & 0x7fffffu) != 0u) return u2f(u | 0x400000u); // NaN -> quiet
        return u2f(0xffc00000u);                               // negative -> default NaN
    }
    if (e == 0xffu) {
        if ((u & 0x7fffffu) != 0u) return u2f(u | 0x400000u);
        return 0.0f;                                           // +inf -> +0
    }
    if (e == 0u) {
        if (u == 0u) return u2f(t.zero_result);
        return u2f(t.denorm_result);                           // RSQRTSS treats denormals as 0
    }
    const int32_t  ex   = (int32_t)e - 127;
    const int32_t  p    = ex & 1;
    const int32_t  q    = (ex - p) / 2;
    const uint32_t m    = (u & 0x7fffffu) >> (23 - t.bits);
    const uint32_t i    = ((uint32_t)p << t.bits) | m;
    const uint32_t r    = t.pack_shift ? (t.pack_hi | ((uint32_t)((const uint16_t*)t.entries)[i] << t.pack_shift)) : t.entries[i];
    const int32_t  re   = (int32_t)((r >> 23) & 0xffu) - q;
    return u2f((r & 0x807fffffu) | ((uint32_t)re << 23));
}

// math/Math.h:205 sp::rsqrt: r = RSQRTSS(a); c = 1.5*r + ((a*-0.5)*r)*(r*r)
SP_HD float rsqrt_newton(float a, float r)
{
    const float t1 = 1.5f * r;
    const float t2 = a * -0.5f;
    const float t3 = t2 * r;
    const float t4 = r * r;
    const float t5 = t3 * t4;
    return t1 + t5;
}

#if !defined(__HIP_DEVICE_COMPILE__)
static inline float rsqrtss_host(float x) { return _mm_cvtss_f32(_mm_rsqrt_ss(_mm_set_ss(x))); }
#else
static inline float rsqrtss_host(float) { return 0.0f; } // host-only helper; never emitted for gfx950
#endif

// ---------------------------------------------------------------- vectors
struct f3 {
    float x, y, z;
};

SP_HD f3 mk(float x, float y, float z) { f3 r; r.x = x; r.y = y; r.z = z; return r; }
SP_HD f3 add(f3 a, f3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
SP_HD f3 sub(f3 a, f3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
SP_HD f3 mul(f3 a, f3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
SP_HD f3 scale(f3 a, float s) { return mk(a.x * s, a.y * s, a.z * s); }   // Vector3 * float
SP_HD f3 scale(float s, f3 a) { return mk(s * a.x, s * a.y, s * a.z); }   // float * Vector3
SP_HD f3 divs(f3 a, float s) { return mk(a.x / s, a.y / s, a.z / s); }
SP_HD f3 neg(f3 a) { return mk(-a.x, -a.y, -a.z); }
SP_HD f3 madd(f3 a, f3 b, f3 c) { return mk(fma_f(a.x, b.x, c.x), fma_f(a.y, b.y, c.y), fma_f(a.z, b.z, c.z)); }
SP_HD f3 madd(float a, f3 b, f3 c) { return mk(fma_f(a, b.x, c.x), fma_f(a, b.y, c.y), fma_f(a, b.z, c.z)); }

// _mm_dp_ps(a, b, 0x7F): Temp2 = p0 + p1, Temp3 = p2 + (+0), result = Temp2 + Temp3
SP_HD float dot(f3 a, f3 b)
{
    const float p0 = a.x * b.x;
    const float p1 = a.y * b.y;
    const float p2 = a.z * b.z;
    return (p0 + p1) + (p2 + 0.0f);
}

// difference_of_products(a, b, c, d) per lane: cd = c*d; err = fnmadd(c,d,cd); dop = fmsub(a,b,cd)
SP_HD float dop1(float a, float b, float c, float d)
{
    const float cd  = c * d;
    const float err = fma_f(-c, d, cd);
    const float dop = fma_f(a, b, -cd);
    return dop + err;
}

// cross(a,b) = dop(shuffle<1,2,0>(a), shuffle<2,0,1>(b), shuffle<2,0,1>(a), shuffle<1,2,0>(b))
SP_HD f3 cross(f3 a, f3 b)
{
    return mk(dop1(a.y, b.z, a.z, b.y), dop1(a.z, b.x, a.x, b.z), dop1(a.x, b.y, a.y, b.x));
}

SP_HD float length(f3 a) { return sqrt_f(dot(a, a)); }

// ---------------------------------------------------------------- RGB (scalar struct, math/RGB.h)
struct rgb {
    float r, g, b;
};
SP_HD rgb mkc(float r, float g, float b) { rgb c; c.r = r; c.g = g; c.b = b; return c; }
SP_HD rgb cadd(rgb a, rgb b) { return mkc(a.r + b.r, a.g + b.g, a.b + b.b); }
SP_HD rgb csub(rgb a, rgb b) { return mkc(a.r - b.r, a.g - b.g, a.b - b.b); }
SP_HD rgb cmul(rgb a, rgb b) { return mkc(a.r * b.r, a.g * b.g, a.b * b.b); }
SP_HD rgb cscale(rgb a, float s) { return mkc(a.r * s, a.g * s, a.b * s); }   // RGB*float and float*RGB
SP_HD rgb cdivs(rgb a, float s) { return mkc(a.r / s, a.g / s, a.b / s); }
SP_HD bool cblack(rgb a) { return a.r == 0.0f && a.g == 0.0f && a.b == 0.0f; } // == RGB::black()
SP_HD float luminance(rgb c) { return 0.2126f * c.r + 0.7152f * c.g + 0.0722f * c.b; }

// ---------------------------------------------------------------- affine transforms
struct aff {
    f3 vx, vy, vz, p;
};
struct lin {
    f3 vx, vy, vz;
};

// AffineSpace::operator()(Point3), math/AffineSpace.h:79
SP_HD f3 xfm_point(const aff& m, f3 p)
{
    return madd(mk(p.x, p.x, p.x), m.vx, madd(mk(p.y, p.y, p.y), m.vy, madd(mk(p.z, p.z, p.z), m.vz, m.p)));
}
// LinearSpace3x3::operator()(Vector3), math/LinearSpace3x3.h:158
SP_HD f3 xfm_vector(const f3& vx, const f3& vy, const f3& vz, f3 a)
{
    return madd(mk(a.x, a.x, a.x), vx, madd(mk(a.y, a.y, a.y), vy, mul(mk(a.z, a.z, a.z), vz)));
}
SP_HD f3 xfm_vector(const aff& m, f3 a) { return xfm_vector(m.vx, m.vy, m.vz, a); }
SP_HD f3 xfm_vector(const lin& m, f3 a) { return xfm_vector(m.vx, m.vy, m.vz, a); }

} // namespace spm
