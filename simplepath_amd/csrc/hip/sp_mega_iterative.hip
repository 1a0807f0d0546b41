// sp_mega_iterative.hip -- BruteForceIntegratorIterative(RR) megakernels (lock-step samples).
#include "sp_mega.hpp"

namespace spd {
KernelFn mega_iterative(int integ)
{
    if (integ == SP_INTEGRATOR_BRUTE_FORCE_ITERATIVE_RR) return sp_render_kernel<SP_INTEGRATOR_BRUTE_FORCE_ITERATIVE_RR, 2>;
    return sp_render_kernel<SP_INTEGRATOR_BRUTE_FORCE_ITERATIVE, 2>;
}
} // namespace spd
