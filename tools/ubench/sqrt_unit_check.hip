// Exhaustive check of sp_path.hpp sqrt_unit against the compiler's correctly rounded f32 sqrt
// (__builtin_sqrtf, IEEE with denormals) over every non-negative float bit pattern and -0.
// sqrt_unit is used only where the argument is +-0 or at least 2^-48; mismatches
// below 2^-96 (inputs the fast form does not scale) are counted apart and expected.
#include "sp_path.hpp"
#include <cstdio>

__global__ void check(uint32_t base, unsigned long long* bad)
{
    const uint32_t u = base + blockIdx.x * blockDim.x + threadIdx.x;
    if (u > 0x7f800000u && u != 0x80000000u) return; // NaN / negative (outside the domain)
    const float x = __uint_as_float(u);
    const float a = spd::sqrt_unit(x), b = __builtin_sqrtf(x);
    const uint32_t m = u & 0x7fffffffu; // +-0 and [2^-96, inf] are the domain
    if (__float_as_uint(a) != __float_as_uint(b)) atomicAdd(bad + ((m != 0u && m < 0x0f800000u) ? 1 : 0), 1ull);
}

int main()
{
    unsigned long long* d;
    (void)hipMalloc(&d, 2 * sizeof(unsigned long long));
    (void)hipMemset(d, 0, 2 * sizeof(unsigned long long));
    const uint32_t chunk = 1u << 28;
    for (uint64_t base = 0; base < 0x80000000ull + chunk; base += chunk) check<<<chunk / 256, 256>>>((uint32_t)base, d);
    unsigned long long h[2];
    (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    printf("sqrt_unit vs IEEE sqrtf: %llu mismatches at +-0 and x >= 2^-96 (domain, must be 0), %llu in (0, 2^-96)\n", h[0], h[1]);
    return h[0] ? 1 : 0;
}
