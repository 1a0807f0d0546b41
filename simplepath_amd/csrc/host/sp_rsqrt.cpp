// sp_rsqrt.cpp -- capture of the host CPU's RSQRTSS approximation for device-side emulation.
//
// The reference normalises every vector with sp::rsqrt (math/Math.h:205): RSQRTSS followed by
// one Newton-Raphson step.  RSQRTSS is a hardware table lookup whose exact output differs
// between CPU vendors, so the reference's results are those of the CPU it runs on.  We read the
// instruction's outputs on the host at start-up, find how many leading mantissa bits determine
// them (exponent parity + k bits; Intel: k = 10), and verify the table against the instruction on
// exhaustive mantissa sweeps plus random inputs over the whole exponent range.  The device then
// reproduces RSQRTSS bit for bit with one table load (spm::rsqrtss_emulated).
#include "sp_host.hpp"

#include <atomic>
#include <mutex>
#include <random>

namespace sph {

namespace {
uint32_t rs_bits(uint32_t in) { return spm::f2u(spm::rsqrtss_host(spm::u2f(in))); }

bool build_and_verify(int bits, RsqrtCapture& cap)
{
    cap.bits = bits;
    cap.entries.assign(size_t(2) << bits, 0u);
    for (uint32_t p = 0; p < 2; ++p)
        for (uint32_t m = 0; m < (1u << bits); ++m)
            cap.entries[(p << bits) | m] = rs_bits(((127u + p) << 23) | (m << (23 - bits)));
    cap.zero_result   = rs_bits(0u);
    cap.denorm_result = rs_bits(1u);
    spm::RsqrtTable t{ cap.entries.data(), cap.bits, cap.zero_result, cap.denorm_result };
    // exhaustive mantissa sweep at four exponents
    const uint32_t exps[] = { 1u, 126u, 127u, 128u, 129u, 200u, 253u, 254u };
    for (uint32_t e : exps)
        for (uint32_t m = 0; m < (1u << 23); m += ((e == 127u || e == 128u) ? 1u : 7u)) {
            const uint32_t in = (e << 23) | m;
            if (spm::f2u(spm::rsqrtss_emulated(spm::u2f(in), t)) != rs_bits(in)) return false;
        }
    // random normal inputs over every exponent
    std::mt19937 rng(12345u);
    for (int i = 0; i < (1 << 21); ++i) {
        const uint32_t e  = 1u + (rng() % 254u);
        const uint32_t in = (e << 23) | (rng() & 0x7fffffu);
        if (spm::f2u(spm::rsqrtss_emulated(spm::u2f(in), t)) != rs_bits(in)) return false;
    }
    return true;
}
} // namespace

const RsqrtCapture& rsqrt_capture()
{
    static RsqrtCapture   cap;
    static std::once_flag once;
    std::call_once(once, [] {
        const int candidates[] = { 10, 11, 12, 13, 14, 16, 18, 20, 23 };
        for (int b : candidates) {
            if (build_and_verify(b, cap)) {
                cap.verified = true;
                break;
            }
        }
        if (cap.verified) {
            // special classes used by normalize(): zero, denormals, inf, NaN
            spm::RsqrtTable t{ cap.entries.data(), cap.bits, cap.zero_result, cap.denorm_result };
            const uint32_t specials[] = { 0u, 1u, 0x3ffu, 0x7fffffu, 0x7f800000u, 0x7fc00000u, 0x7f800001u,
                                          0x80000000u, 0xbf800000u, 0xff800000u, 0xffc00000u };
            for (uint32_t s : specials)
                if (spm::f2u(spm::rsqrtss_emulated(spm::u2f(s), t)) != rs_bits(s)) {
                    cap.verified = false; // table is right for normals; flag the class mismatch
                }
        }
    });
    return cap;
}

namespace {
std::mutex   g_override_mu;
RsqrtCapture g_override;                       // valid when g_use_override
std::atomic<bool> g_use_override{ false };
} // namespace

const RsqrtCapture& rsqrt_active()
{
    if (g_use_override.load(std::memory_order_acquire)) return g_override;
    return rsqrt_capture();
}

void rsqrt_set_override(const uint32_t* entries, int32_t bits, uint32_t zero_result, uint32_t denorm_result)
{
    std::lock_guard<std::mutex> lk(g_override_mu);
    if (!entries) {
        g_use_override.store(false, std::memory_order_release);
        return;
    }
    if (bits < 1 || bits > 23) throw SpError(SP_ERR_ARG, "RSQRTSS table: bits must be 1..23");
    g_use_override.store(false, std::memory_order_release);
    g_override.bits          = bits;
    g_override.entries.assign(entries, entries + (size_t(2) << bits));
    g_override.zero_result   = zero_result;
    g_override.denorm_result = denorm_result;
    g_override.verified      = true; // as given: the table of the CPU that produced the reference
    g_use_override.store(true, std::memory_order_release);
}

float rsqrtss_active(float a)
{
    if (!g_use_override.load(std::memory_order_acquire)) return spm::rsqrtss_host(a);
    const spm::RsqrtTable t{ g_override.entries.data(), g_override.bits, g_override.zero_result,
                             g_override.denorm_result };
    return spm::rsqrtss_emulated(a, t);
}

} // namespace sph
