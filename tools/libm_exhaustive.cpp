// Exhaustive bit-exactness check of spm::lm_* (simplepath_amd/csrc/common/sp_libm.h) against the
// host glibc float libm.  Usage: libm_exhaustive <func> [stride] [threads]
//   func: sinf cosf sincosf expf logf erff acosf atanf fmod1 roundf powf atan2f
// Prints "<func> checked=<n> mismatches=<m>" and up to 8 examples.
#include "../simplepath_amd/csrc/common/sp_libm.h"
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <random>
#include <string>
#include <thread>
#include <vector>

static uint32_t bits(float f) { uint32_t u; std::memcpy(&u, &f, 4); return u; }
static float flt(uint32_t u) { float f; std::memcpy(&f, &u, 4); return f; }

int main(int argc, char** argv)
{
    const std::string fn = argc > 1 ? argv[1] : "expf";
    const uint64_t stride = argc > 2 ? std::stoull(argv[2]) : 1;
    const int nth = argc > 3 ? std::stoi(argv[3]) : (int)std::thread::hardware_concurrency();
    std::atomic<uint64_t> checked{0}, bad{0};
    std::vector<std::string> examples;
    std::atomic<int> nex{0};
    char buf[256];
    auto report = [&](float a, float b, float got, float want) {
        if (nex.fetch_add(1) < 8) {
            std::snprintf(buf, sizeof buf, "  x=%a (0x%08x) y=%a got=0x%08x want=0x%08x", a, bits(a), b, bits(got), bits(want));
            std::printf("%s\n", buf);
        }
    };
    if (fn == "atan2f") {  // pairs: random bits, unit-vector components (the reference's use), specials
        std::vector<std::thread> th;
        for (int t = 0; t < nth; ++t)
            th.emplace_back([&, t] {
                std::mt19937_64 rng(777 + t);
                uint64_t c = 0, b = 0;
                const uint64_t n = (stride > 1 ? 4000000ull : 100000000ull) / nth;
                const float sp[] = {0.0f, -0.0f, 1.0f, -1.0f, INFINITY, -INFINITY, NAN, 1e-38f, -1e-38f, 1e38f, -1e38f, 1e-45f};
                for (uint64_t i = 0; i < n; ++i) {
                    float x, y;
                    const int mode = i % 4;
                    if (mode == 0) { y = flt((uint32_t)rng()); x = flt((uint32_t)rng()); }
                    else if (mode == 1) {
                        y = (float)((double)(rng() >> 11) * 0x1.0p-53 * 2.0 - 1.0);
                        x = (float)((double)(rng() >> 11) * 0x1.0p-53 * 2.0 - 1.0);
                    } else if (mode == 2) {
                        y = sp[rng() % 12]; x = ((rng() & 1) ? sp[rng() % 12] : flt((uint32_t)rng()));
                        if (rng() & 1) std::swap(x, y);
                    } else { const float a = flt((uint32_t)rng()); y = a * (float)(int)(rng() % 7 - 3); x = a * (float)(int)(rng() % 7 - 3) + flt((uint32_t)rng() & 0x807fffffu); }
                    const float want = atan2f(y, x), got = spm::lm_atan2f(y, x);
                    ++c;
                    if (bits(want) != bits(got)) { ++b; report(y, x, got, want); }
                }
                checked += c;
                bad += b;
            });
        for (auto& x : th) x.join();
    } else if (fn == "powf") {
        std::vector<std::thread> th;
        for (int t = 0; t < nth; ++t)
            th.emplace_back([&, t] {
                std::mt19937_64 rng(1234 + t);
                uint64_t c = 0, b = 0;
                const uint64_t n = (stride > 1 ? 4000000ull : 40000000ull) / nth;
                for (uint64_t i = 0; i < n; ++i) {
                    float x, y;
                    const int mode = i % 4;
                    if (mode == 0) { x = flt((uint32_t)rng()); y = flt((uint32_t)rng()); }
                    else if (mode == 1) {  // the reference's use: pow(1 - sample_x, fit)
                        x = (float)((rng() >> 40) * (1.0 / 16777216.0));
                        y = 0.3f + (float)((rng() >> 40) * (1.0 / 16777216.0));
                    } else if (mode == 2) { x = flt(0x00000001u + (uint32_t)(rng() % 0x7f800000u)); y = (float)((int)(rng() % 64) - 32) * 0.5f; }
                    else { x = -flt((uint32_t)(rng() % 0x7f800001u)); y = (float)((int)(rng() % 41) - 20); }
                    const float want = powf(x, y), got = spm::lm_powf(x, y);
                    ++c;
                    if (bits(want) != bits(got)) { ++b; report(x, y, got, want); }
                }
                checked += c;
                bad += b;
            });
        for (auto& x : th) x.join();
    } else if (fn == "sincosf") {  // the fused forms: bounded where abstop <= 0x42e (|x| < 120), general elsewhere
        std::vector<std::thread> th;
        const uint64_t total = 1ull << 32;
        for (int t = 0; t < nth; ++t)
            th.emplace_back([&, t] {
                uint64_t c = 0, b = 0;
                for (uint64_t u = (uint64_t)t * stride; u < total; u += (uint64_t)nth * stride) {
                    const float x = flt((uint32_t)u);
                    float s, co;
                    if ((((uint32_t)u >> 20) & 0x7ffu) <= 0x42eu) spm::lm_sincosf_bounded(x, &s, &co);
                    else spm::lm_sincosf(x, &s, &co); // the general form's fallback
                    ++c;
                    if (bits(s) != bits(sinf(x))) { ++b; report(x, 0.0f, s, sinf(x)); }
                    if (bits(co) != bits(cosf(x))) { ++b; report(x, 1.0f, co, cosf(x)); }
                }
                checked += c;
                bad += b;
            });
        for (auto& x : th) x.join();
    } else {
        float (*ref)(float) = nullptr;
        float (*emu)(float) = nullptr;
        if (fn == "sinf") { ref = sinf; emu = [](float x) { return spm::lm_sinf(x); }; }
        else if (fn == "cosf") { ref = cosf; emu = [](float x) { return spm::lm_cosf(x); }; }
        else if (fn == "expf") { ref = expf; emu = [](float x) { return spm::lm_expf(x); }; }
        else if (fn == "logf") { ref = logf; emu = [](float x) { return spm::lm_logf(x); }; }
        else if (fn == "erff") { ref = erff; emu = [](float x) { return spm::lm_erff(x); }; }
        else if (fn == "acosf") { ref = acosf; emu = [](float x) { return spm::lm_acosf(x); }; }
        else if (fn == "atanf") { ref = atanf; emu = [](float x) { return spm::lm_atanf(x); }; }
        else if (fn == "fmod1") { ref = [](float x) { return fmodf(x, 1.0f); }; emu = [](float x) { return spm::fmod1(x); }; }
        else if (fn == "roundf") { ref = roundf; emu = [](float x) { return spm::round_f(x); }; }
        else { std::printf("unknown %s\n", fn.c_str()); return 2; }
        std::vector<std::thread> th;
        const uint64_t total = 1ull << 32;
        for (int t = 0; t < nth; ++t)
            th.emplace_back([&, t] {
                uint64_t c = 0, b = 0;
                for (uint64_t u = (uint64_t)t * stride; u < total; u += (uint64_t)nth * stride) {
                    const float x = flt((uint32_t)u);
                    const float want = ref(x), got = emu(x);
                    ++c;
                    if (bits(want) != bits(got)) { ++b; report(x, 0.0f, got, want); }
                }
                checked += c;
                bad += b;
            });
        for (auto& x : th) x.join();
    }
    std::printf("%s checked=%llu mismatches=%llu\n", fn.c_str(), (unsigned long long)checked.load(), (unsigned long long)bad.load());
    return bad.load() == 0 ? 0 : 1;
}
