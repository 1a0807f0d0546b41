// Host check of the twists of simplepath_amd/csrc/common/sp_twist4.h (4-word grouped, grouped
// one-pass, word-by-word one-pass with 12- and 24-word blocks): on the lane-blocked layout each must
// produce exactly std::mt19937_64's next generation, for every lane position, many seeds and
// consecutive generations.  Built and run by tests/test_numerics.py.
#include "sp_twist4.h"
#include <cstdio>
#include <random>
#include <vector>

using namespace spm;

int main()
{
    std::vector<uint64_t> A(78 * 256), B(78 * 256);
    int bad = 0, checked = 0;
    auto off4 = [](int k) { return (k / 4) * 256 + k % 4; };
    auto off1 = [](int k) { return k * 64; };
    for (int variant = 0; variant < 5; ++variant)
    for (int lane : { 0, 1, 31, 63 }) {
        for (uint32_t seed : { 1u, 0xb0ae9d99u, 12345u }) {
            std::mt19937_64 ref(seed);
            Mt64            s;
            mt_init(s, seed);
            for (int k = 0; k < MT_N; ++k) A[variant == 4 ? k * 64 + lane : (k / 4) * 256 + lane * 4 + k % 4] = s.x[k];
            for (int gen = 0; gen < 5; ++gen) {
                if (variant == 0) mt_twist_grouped4<3>(A.data() + lane * 4, B.data() + lane * 4);
                else if (variant == 1) mt_twist_grouped4_fused<3>(A.data() + lane * 4, B.data() + lane * 4);
                else if (variant == 2) mt_twist_fused<12>(A.data() + lane * 4, B.data() + lane * 4, off4);
                else if (variant == 3) mt_twist_fused<24>(A.data() + lane * 4, B.data() + lane * 4, off4);
                else mt_twist_fused<24>(A.data() + lane, B.data() + lane, off1); // interleaved words (chunk store)
                // the words std::mt19937_64 draws from this generation, tempered
                for (int k = 0; k < MT_N; ++k) {
                    ++checked;
                    if (mt_temper(B[variant == 4 ? k * 64 + lane : (k / 4) * 256 + lane * 4 + k % 4]) != ref()) { ++bad; break; }
                }
                std::swap(A, B);
            }
        }
    }
    std::printf("twist4: %d words checked, %d mismatching generations\n", checked, bad);
    return bad != 0;
}
