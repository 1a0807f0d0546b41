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

#include <algorithm>
#include <atomic>
#include <memory>
#include <mutex>
#include <random>
#include <string>
#include <vector>

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
// Installed tables are immutable and never freed, so a reader's pointer stays valid while another
// thread installs the next one: no lock on the read path, which runs once per normalize() of every
// mesh normal while a scene is built.  An install that equals a table already kept reuses it, so
// the set grows only with the number of DISTINCT tables a process installs (a handful: one per
// CPU whose images it reproduces), however often sp_rsqrt_table_set is called.
std::mutex                               g_override_mu;
std::vector<std::unique_ptr<RsqrtCapture>> g_installed; // owned for the life of the process
std::atomic<const RsqrtCapture*>         g_override{ nullptr };
// Largest table the device copies into LDS next to the traversal stacks: 2 << 13 words (64 KB
// as 32-bit entries).  Real CPUs need 11 (Intel) or 12 (AMD) bits.
constexpr int k_max_table_bits = 13;
} // namespace

const RsqrtCapture& rsqrt_active()
{
    if (const RsqrtCapture* o = g_override.load(std::memory_order_acquire)) return *o;
    return rsqrt_capture();
}

void rsqrt_set_override(const uint32_t* entries, int32_t bits, uint32_t zero_result, uint32_t denorm_result)
{
    std::lock_guard<std::mutex> lk(g_override_mu);
    if (!entries) {
        g_override.store(nullptr, std::memory_order_release);
        return;
    }
    if (bits < 1 || bits > k_max_table_bits)
        throw SpError(SP_ERR_ARG, "RSQRTSS table: bits must be 1.." + std::to_string(k_max_table_bits) +
                                      " (2 << bits entries must fit the device's LDS copy)");
    const size_t n = size_t(2) << bits;
    for (const auto& kept : g_installed)
        if (kept->bits == bits && kept->zero_result == zero_result && kept->denorm_result == denorm_result &&
            std::equal(entries, entries + n, kept->entries.begin())) {
            g_override.store(kept.get(), std::memory_order_release);
            return;
        }
    auto cap           = std::make_unique<RsqrtCapture>();
    cap->bits          = bits;
    cap->entries.assign(entries, entries + n);
    cap->zero_result   = zero_result;
    cap->denorm_result = denorm_result;
    cap->verified      = true; // as given: the table of the CPU that produced the reference
    g_override.store(cap.get(), std::memory_order_release);
    g_installed.push_back(std::move(cap));
}

float rsqrtss_active(float a)
{
    const RsqrtCapture* o = g_override.load(std::memory_order_acquire);
    if (!o) return spm::rsqrtss_host(a);
    const spm::RsqrtTable t{ o->entries.data(), o->bits, o->zero_result, o->denorm_result };
    return spm::rsqrtss_emulated(a, t);
}

} // namespace sph
