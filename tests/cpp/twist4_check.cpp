// Host check of the 4-word grouped twist (simplepath_amd/csrc/common/sp_twist4.h): on the
// lane-blocked layout it must produce exactly std::mt19937_64's next generation, for every lane
// position, many seeds and consecutive generations.  Built and run by tests/test_numerics.py.
#include "sp_twist4.h"
#include <cstdio>
#include <random>
#include <vector>

using namespace spm;

int main()
{
    std::vector<uint64_t> A(78 * 256), B(78 * 256);
    int bad = 0, checked = 0;
    for (int lane : { 0, 1, 31, 63 }) {
        for (uint32_t seed : { 1u, 0xb0ae9d99u, 12345u }) {
            std::mt19937_64 ref(seed);
            Mt64            s;
            mt_init(s, seed);
            for (int k = 0; k < MT_N; ++k) A[(k / 4) * 256 + lane * 4 + k % 4] = s.x[k];
            for (int gen = 0; gen < 5; ++gen) {
                mt_twist_grouped4<3>(A.data() + lane * 4, B.data() + lane * 4);
                // the words std::mt19937_64 draws from this generation, tempered
                for (int k = 0; k < MT_N; ++k) {
                    ++checked;
                    if (mt_temper(B[(k / 4) * 256 + lane * 4 + k % 4]) != ref()) { ++bad; break; }
                }
                std::swap(A, B);
            }
        }
    }
    std::printf("twist4: %d words checked, %d mismatching generations\n", checked, bad);
    return bad != 0;
}
