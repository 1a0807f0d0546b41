// sp_twist4.h -- the std::mt19937_64 twist on the 4-word lane-blocked state layout (sp_device.hpp
// MT_BLK = 4: word k of a lane at (k / 4) * 256 + lane * 4 + k % 4), four words per step.
//
// B = twist(A), generations A and B distinct.  With a lane's words 4g .. 4g + 3 contiguous (32
// bytes), a step loads group g + 1 of A and group g + 39 of A (first part) or g - 39 of B (second
// part) -- 156 = MT_N - MT_M = 39 groups, so both are whole, aligned groups -- and stores group g
// of B: two 16-byte accesses per 4 words each, where the word-by-word form issued 3 accesses per
// word.  The words and their order are those of mt_twist_inplace (sp_rng.h), which the host test
// (tests/test_numerics.py) checks against libstdc++'s generator.  UG groups per block: all their
// loads are issued before the block's stores.
#pragma once
#include "sp_rng.h"

namespace spm {

constexpr int TW4_GROUP_STRIDE = 256; // words between consecutive groups of one lane (4 words x 64 lanes)

// a group is 32-byte aligned (lane base lane * 32 B in a 256-B aligned buffer): two 16-byte accesses
SP_HD void tw4_load(const uint64_t* p, uint64_t w[4])
{
    const uint64_t* q = static_cast<const uint64_t*>(__builtin_assume_aligned(p, 32));
    w[0] = q[0]; w[1] = q[1]; w[2] = q[2]; w[3] = q[3];
}
SP_HD void tw4_store(uint64_t* p, const uint64_t w[4])
{
    uint64_t* q = static_cast<uint64_t*>(__builtin_assume_aligned(p, 32));
    q[0] = w[0]; q[1] = w[1]; q[2] = w[2]; q[3] = w[3];
}

template <int UG>
SP_HD void mt_twist_grouped4(const uint64_t* __restrict__ A, uint64_t* __restrict__ B)
{
    constexpr int NG = MT_N / 4;            // 78 groups
    constexpr int HG = (MT_N - MT_M) / 4;   // 39
    static_assert(MT_N % 4 == 0 && (MT_N - MT_M) % 4 == 0 && HG % UG == 0, "whole groups");
    uint64_t cur[4];
    tw4_load(A, cur);
    // words 0 .. 155: B[k] = A[k + 156] ^ mix(A[k], A[k + 1])
    for (int g0 = 0; g0 < HG; g0 += UG) {
        uint64_t nx[UG][4], mm[UG][4];
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
#endif
        for (int u = 0; u < UG; ++u) {
            tw4_load(A + (size_t)(g0 + u + 1) * TW4_GROUP_STRIDE, nx[u]);
            tw4_load(A + (size_t)(g0 + u + HG) * TW4_GROUP_STRIDE, mm[u]);
        }
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
#endif
        for (int u = 0; u < UG; ++u) {
            const uint64_t* a = (u == 0) ? cur : nx[u - 1];
            uint64_t        o[4];
            o[0] = mm[u][0] ^ mt_mix(a[0], a[1]);
            o[1] = mm[u][1] ^ mt_mix(a[1], a[2]);
            o[2] = mm[u][2] ^ mt_mix(a[2], a[3]);
            o[3] = mm[u][3] ^ mt_mix(a[3], nx[u][0]);
            tw4_store(B + (size_t)(g0 + u) * TW4_GROUP_STRIDE, o);
        }
        for (int i = 0; i < 4; ++i) cur[i] = nx[UG - 1][i];
    }
    // words 156 .. 311: B[k] = B[k - 156] ^ mix(A[k], A[k + 1]), and A[312] is B[0] (the last word)
    const uint64_t b0 = B[0];
    for (int g0 = HG; g0 < NG; g0 += UG) {
        uint64_t nx[UG][4], mm[UG][4];
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
#endif
        for (int u = 0; u < UG; ++u) {
            if (g0 + u + 1 < NG) tw4_load(A + (size_t)(g0 + u + 1) * TW4_GROUP_STRIDE, nx[u]);
            else { nx[u][0] = b0; nx[u][1] = nx[u][2] = nx[u][3] = 0; }
            tw4_load(B + (size_t)(g0 + u - HG) * TW4_GROUP_STRIDE, mm[u]);
        }
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
#endif
        for (int u = 0; u < UG; ++u) {
            const uint64_t* a = (u == 0) ? cur : nx[u - 1];
            uint64_t        o[4];
            o[0] = mm[u][0] ^ mt_mix(a[0], a[1]);
            o[1] = mm[u][1] ^ mt_mix(a[1], a[2]);
            o[2] = mm[u][2] ^ mt_mix(a[2], a[3]);
            o[3] = mm[u][3] ^ mt_mix(a[3], nx[u][0]);
            tw4_store(B + (size_t)(g0 + u) * TW4_GROUP_STRIDE, o);
        }
        for (int i = 0; i < 4; ++i) cur[i] = nx[UG - 1][i];
    }
}

// The same generation in one pass over A: step g computes group g of B (first part) and, from it,
// group g + 39 (second part: B[k + 156] = B[k] ^ mix(A[k + 156], A[k + 157])), so every group of A
// is loaded once -- the two-part form loads A's groups 40 .. 77 twice and reads B's first half back.
// A's word 312 (after the last) is B's word 0, as in the two-part form.
template <int UG>
SP_HD void mt_twist_grouped4_fused(const uint64_t* __restrict__ A, uint64_t* __restrict__ B)
{
    constexpr int NG = MT_N / 4;            // 78 groups
    constexpr int HG = (MT_N - MT_M) / 4;   // 39
    static_assert(MT_N % 4 == 0 && MT_N == 2 * MT_M && HG % UG == 0, "whole groups, two equal halves");
    uint64_t cur[4], curm[4], b0 = 0;
    tw4_load(A, cur);
    tw4_load(A + (size_t)HG * TW4_GROUP_STRIDE, curm);
    for (int g0 = 0; g0 < HG; g0 += UG) {
        uint64_t nx[UG][4], mx[UG][4];
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
#endif
        for (int u = 0; u < UG; ++u) {
            tw4_load(A + (size_t)(g0 + u + 1) * TW4_GROUP_STRIDE, nx[u]);
            if (g0 + u + HG + 1 < NG) tw4_load(A + (size_t)(g0 + u + HG + 1) * TW4_GROUP_STRIDE, mx[u]);
            else mx[u][0] = mx[u][1] = mx[u][2] = mx[u][3] = 0;
        }
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
#endif
        for (int u = 0; u < UG; ++u) {
            const uint64_t* a = (u == 0) ? cur : nx[u - 1];
            const uint64_t* m = (u == 0) ? curm : mx[u - 1];
            uint64_t        o[4], o2[4];
            o[0] = m[0] ^ mt_mix(a[0], a[1]);
            o[1] = m[1] ^ mt_mix(a[1], a[2]);
            o[2] = m[2] ^ mt_mix(a[2], a[3]);
            o[3] = m[3] ^ mt_mix(a[3], nx[u][0]);
            if (g0 + u == 0) b0 = o[0];
            const uint64_t m4 = (g0 + u + HG + 1 < NG) ? mx[u][0] : b0;
            o2[0] = o[0] ^ mt_mix(m[0], m[1]);
            o2[1] = o[1] ^ mt_mix(m[1], m[2]);
            o2[2] = o[2] ^ mt_mix(m[2], m[3]);
            o2[3] = o[3] ^ mt_mix(m[3], m4);
            tw4_store(B + (size_t)(g0 + u) * TW4_GROUP_STRIDE, o);
            tw4_store(B + (size_t)(g0 + u + HG) * TW4_GROUP_STRIDE, o2);
        }
        for (int i = 0; i < 4; ++i) {
            cur[i]  = nx[UG - 1][i];
            curm[i] = mx[UG - 1][i];
        }
    }
}

// The one-pass twist word by word on any lane layout (off(k): word k's offset from the lane's base),
// U words per block of loads.
template <int U, class Off>
SP_HD void mt_twist_fused(const uint64_t* __restrict__ A, uint64_t* __restrict__ B, Off off)
{
    constexpr int H = MT_N - MT_M; // 156 = M
    static_assert(MT_N == 2 * MT_M, "two equal halves");
    uint64_t a = A[0], m = A[off(H)], b0 = 0;
    for (int k0 = 0; k0 < H; k0 += U) {
        uint64_t a1[U], m1[U];
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
#endif
        for (int j = 0; j < U; ++j)
            if (k0 + j < H) {
                a1[j] = A[off(k0 + j + 1)];
                m1[j] = (k0 + j + H + 1 < MT_N) ? A[off(k0 + j + H + 1)] : 0;
            }
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
#endif
        for (int j = 0; j < U; ++j)
            if (k0 + j < H) {
                const int      k  = k0 + j;
                const uint64_t bk = m ^ mt_mix(a, a1[j]);
                if (k == 0) b0 = bk;
                const uint64_t mn = (k + H + 1 < MT_N) ? m1[j] : b0;
                B[off(k)]         = bk;
                B[off(k + H)]     = bk ^ mt_mix(m, mn);
                a                 = a1[j];
                m                 = m1[j];
            }
    }
}

} // namespace spm
