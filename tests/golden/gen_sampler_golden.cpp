// Generates tests/golden/sampler_golden.npz inputs: the draws of libstdc++'s std::mt19937_64 +
// std::uniform_real_distribution<float> (the reference's IncoherentSampler, math/Sampler.h:96)
// for the per-pixel seeds main.cpp:73 uses, as raw float bits.  Output: text, one uint32 per line.
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>
int main()
{
    const uint32_t pix[][2] = { { 0, 0 }, { 1, 0 }, { 0, 1 }, { 17, 5 }, { 1919, 1079 }, { 640, 360 } };
    for (auto& p : pix) {
        const uint32_t seed = ((p[0] << 16u) | p[1]) ^ 0xb0ae9d99u;
        std::mt19937_64 rng(seed);
        std::uniform_real_distribution<float> dist;
        for (int i = 0; i < 1000; ++i) {
            float f;
            do { f = dist(rng); } while (f >= 1.0f);
            uint32_t u;
            std::memcpy(&u, &f, 4);
            std::printf("%u %u %u\n", p[0], p[1], u);
        }
    }
    return 0;
}
