// sp_rng.h -- the reference's two per-pixel samplers, bit-exact.
//
// IncoherentSampler (math/Sampler.h:96): std::mt19937_64 seeded with a 32-bit Seed, drawn through
// std::uniform_real_distribution<float>.  libstdc++ (GCC 11, the toolchain of this image)
// implements the draw as generate_canonical<float, 24>: one 64-bit output u, float(u) / 2^64,
// clamped to nextafter(1, 0).  The engine is the published MT19937-64 (Matsumoto & Nishimura,
// 2000; w=64 n=312 m=156 r=31, a=0xB5026F5AA96619E9, tempering u=29 d=0x5555555555555555
// s=17 b=0x71D67FFFEDA60000 t=37 c=0xFFF7EEE000000000 l=43, init f=6364136223846793005).
//
// RSequenceSampler (math/Sampler.h:138): the R_d low-discrepancy sequence
// frac(float(seed)/FLT_MAX + alpha_i * (n + 1)), alpha computed on the host with glibc powf
// exactly as RSequence's constructor does (sp_rsequence_alphas in the host code).
#pragma once
#include "sp_math.h"

namespace spm {

constexpr int      MT_N     = 312;
constexpr int      MT_M     = 156;
constexpr uint64_t MT_A     = 0xB5026F5AA96619E9ull;
constexpr uint64_t MT_UPPER = 0xFFFFFFFF80000000ull;
constexpr uint64_t MT_LOWER = 0x000000007FFFFFFFull;

SP_HD uint64_t mt_temper(uint64_t z)
{
    z ^= (z >> 29) & 0x5555555555555555ull;
    z ^= (z << 17) & 0x71D67FFFEDA60000ull;
    z ^= (z << 37) & 0xFFF7EEE000000000ull;
    z ^= (z >> 43);
    return z;
}

SP_HD uint64_t mt_mix(uint64_t lo_word, uint64_t hi_word)
{
    const uint64_t y = (lo_word & MT_UPPER) | (hi_word & MT_LOWER);
    return (y >> 1) ^ ((y & 1ull) ? MT_A : 0ull);
}

// std::mt19937_64::seed(value): x[0] = value; x[i] = f*(x[i-1] ^ (x[i-1] >> 62)) + i
SP_HD uint64_t mt_seed_next(uint64_t prev, uint64_t i)
{
    return 6364136223846793005ull * (prev ^ (prev >> 62)) + i;
}

// generate_canonical<float,24>(mt19937_64): float(u) / 2^64, clamped below 1.
SP_HD float canonical_from_u64(uint64_t u)
{
    const float f = (float)u;
    float r = f * 5.42101086242752217004e-20f; // exact: 2^-64
    if (r >= 1.0f) r = u2f(0x3f7fffffu);
    return r;
}

// RSequence::mod1 uses std::modf: the fractional part (exact).
SP_HD float modf_frac(float f)
{
    return f - __builtin_truncf(f);
}

// RSequence<dim>::r_sequence (math/Sampler.h:35)
SP_HD float rseq_component(uint32_t seed, float alpha, uint32_t n)
{
    const float fseed = (float)seed / 3.40282346638528859812e+38f;
    return modf_frac(fseed + alpha * ((float)n + 1.0f));
}

// Host-side reference engine (used by host code paths and the tests).
struct Mt64 {
    uint64_t x[MT_N];
    int      p;
};

SP_HD void mt_init(Mt64& s, uint32_t seed)
{
    s.x[0] = (uint64_t)seed;
    for (int i = 1; i < MT_N; ++i) s.x[i] = mt_seed_next(s.x[i - 1], (uint64_t)i);
    s.p = MT_N;
}

SP_HD void mt_twist_inplace(Mt64& s)
{
    for (int k = 0; k < MT_N - MT_M; ++k) s.x[k] = s.x[k + MT_M] ^ mt_mix(s.x[k], s.x[k + 1]);
    for (int k = MT_N - MT_M; k < MT_N - 1; ++k) s.x[k] = s.x[k + (MT_M - MT_N)] ^ mt_mix(s.x[k], s.x[k + 1]);
    s.x[MT_N - 1] = s.x[MT_M - 1] ^ mt_mix(s.x[MT_N - 1], s.x[0]);
    s.p = 0;
}

SP_HD uint64_t mt_next(Mt64& s)
{
    if (s.p >= MT_N) mt_twist_inplace(s);
    return mt_temper(s.x[s.p++]);
}

} // namespace spm
